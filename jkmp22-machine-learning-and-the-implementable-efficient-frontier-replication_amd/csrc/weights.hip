// The sequential part of the PFML weight recursion (PFML_best_hps.py:168-218, eq. (17)):
//
//   for t:  d      = (w_start - w_aim_t) / a_t
//           w_opt  = w_aim_t + a_t o (m_tilde_t d)           (m_t = diag(a) m_tilde diag(1/a))
//           w_start(t+1)[r] = hit[r] ? w_opt[map[r]] * grow_t[map[r]] : 0
//
// Every month depends on the previous one; each month is one launch of ROWS_WG-row
// workgroups (all launched from the host loop below, no host round trip): every workgroup
// rebuilds the N-vector d of its month in LDS from the previous month's w_opt (drift gather),
// then computes its rows of m_tilde_t d with one wave per row (coalesced row reads, 8 loads per
// lane in flight, shuffle reduction).  m_tilde_t (N x N, the only large operand) is read once
// per month spread over N / ROWS_WG workgroups, so a month costs about one memory round trip:
// a single persistent workgroup was bound by one CU's bandwidth (39 ms for 360 months at
// N = 500), 16-row workgroups walking their rows one load pair at a time by latency (14 ms).
#include "common.h"

namespace {

constexpr int WT = 256;
constexpr int ROWS_WG = 4;             // 4 waves x 1 row
constexpr int WMAX = 4096;             // N held in LDS (32 KB)

__global__ __launch_bounds__(WT) void weights_month_kernel(
    const double* __restrict__ mt, int64_t ldm, int64_t sm, const double* __restrict__ a,
    const double* __restrict__ wa, const double* __restrict__ grow,
    const int64_t* __restrict__ nmap, const double* __restrict__ hit, int64_t sv,
    const double* __restrict__ ws0, int m, int B, int N, double* __restrict__ Wst,
    double* __restrict__ Wopt, double* __restrict__ ws_out) {
  __shared__ double d[WMAX];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // w_start of month m: ws0 (m == 0) or the drifted w_opt of month m - 1
  const double* wop = Wopt + (int64_t)(m - 1) * sv;
  const double* gp = grow + (int64_t)(m - 1) * sv;
  const int64_t* np_ = nmap + (int64_t)(m - 1) * sv;
  const double* hp = hit + (int64_t)(m - 1) * sv;
  const bool last = m == B;                       // final call: only w_start of month B
  const double* am = a + (int64_t)m * sv;
  const double* wam = wa + (int64_t)m * sv;
  for (int j = t; j < N; j += WT) {
    double ws;
    if (m == 0) {
      ws = ws0[j];
    } else {
      const int64_t q = np_[j];
      ws = (wop[q] * gp[q]) * hp[j];
    }
    if (last) {
      if (blockIdx.x == 0) ws_out[j] = ws;
    } else {
      if (blockIdx.x == 0) Wst[(int64_t)m * sv + j] = ws;
      d[j] = (ws - wam[j]) / am[j];
    }
  }
  if (last) return;
  __syncthreads();
  const double* M = mt + (int64_t)m * sm;
  const int i = blockIdx.x * ROWS_WG + w;
  if (i >= N) return;
  const double* row = M + (int64_t)i * ldm;
  double s = 0.0;
  for (int j0 = 0; j0 < N; j0 += 8 * 64) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + 64 * u + lane;
      x[u] = (j < N) ? row[j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + 64 * u + lane;
      s += (j < N) ? x[u] * d[j] : 0.0;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) Wopt[(int64_t)m * sv + i] = wam[i] + am[i] * s;
}

}  // namespace

extern "C" int pfml_weights_chain_max_n() { return WMAX; }

// mt: [B, N, N] (row stride ldm, batch stride sm); a, wa, grow, hit: [B, N] doubles and nmap
// [B, N] int64 (batch stride sv, entries in [0, N)); ws0 [N]; outputs Wst, Wopt [B, N] (stride
// sv) and ws_out [N] (the w_start of the month after the last).  B + 1 launches on `st`.
extern "C" hipError_t pfml_weights_chain(const double* mt, int64_t ldm, int64_t sm,
                                         const double* a, const double* wa, const double* grow,
                                         const int64_t* nmap, const double* hit, int64_t sv,
                                         const double* ws0, int B, int N, double* Wst,
                                         double* Wopt, double* ws_out, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  if (N > WMAX) return hipErrorInvalidValue;
  const int grid = (N + ROWS_WG - 1) / ROWS_WG;
  for (int m = 0; m <= B; ++m)
    hipLaunchKernelGGL(weights_month_kernel, dim3(m == B ? 1 : grid), dim3(WT), 0, st, mt, ldm,
                       sm, a, wa, grow, nmap, hit, sv, ws0, m, B, N, Wst, Wopt, ws_out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Aim portfolios (PFML_aim_fun.py:138-163, K18): w_aim = s_t beta for every OOS month in ONE
// launch instead of a per-month library GEMV from a Python loop.  Job j (one month): S_j =
// rows [0, nrow_j) of a row-major [*, ld_j] signal block at sptr_j (the S4 signal views, no
// copy), beta_j = coef row j (nk_j = p + 1 entries), out[off_j + r].  One wave per output row:
// lane l sums k = l, l + 64, ... in order, then a fixed butterfly - the same order for a row
// wherever its month sits in the launch (aims are bitwise independent of the sharding).
namespace {
struct AimJob {
  const double* s;
  int64_t ld;
  int64_t off;
  int nrow;
  int nk;
};

__global__ __launch_bounds__(256) void aim_gemv_kernel(const AimJob* __restrict__ jobs,
                                                       const double* __restrict__ coef,
                                                       int64_t ldc, double* __restrict__ out) {
  const AimJob jb = jobs[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= jb.nrow) return;
  const double* srow = jb.s + (int64_t)r * jb.ld;
  const double* c = coef + (int64_t)blockIdx.y * ldc;
  double acc = 0.0;
  for (int k = lane; k < jb.nk; k += 64) acc = fma(srow[k], c[k], acc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) out[jb.off + r] = acc;
}
}  // namespace

extern "C" int pfml_aim_job_size() { return (int)sizeof(AimJob); }

// jobs: device AimJob[njobs]; coef: [njobs, ldc]; rows per job <= max_rows.
extern "C" hipError_t pfml_aim_gemv(const void* jobs, int njobs, int max_rows, const double* coef,
                                    int64_t ldc, double* out, hipStream_t st) {
  if (njobs <= 0 || max_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(aim_gemv_kernel, dim3((max_rows + 3) / 4, njobs), dim3(256), 0, st,
                     static_cast<const AimJob*>(jobs), coef, ldc, out);
  return hipGetLastError();
}
