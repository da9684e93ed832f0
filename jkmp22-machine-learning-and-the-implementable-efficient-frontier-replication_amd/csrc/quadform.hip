// Out-of-sample validation utilities (PFML_hp_reals.py:81-102):
//
//     obj[job, l] = r_t^T beta_l - 1/2 beta_l^T D_t beta_l
//
// for every (g, year, p) cell, every one of its 12 validation months t and all 101 lambdas.
// The reference evaluates 513,888 of these quadratic forms one at a time from Python.  Here a
// job = (cell, month); the kernel computes the GEMM  U = D_t[:n,:n] * B  (B = [beta_l], n x L)
// on fp64 MFMA (upper block triangle only: D_t is symmetric) and folds the two reductions
// into the epilogue, so U never leaves registers.
//
// Tile: 64 rows of D x 112 lambda columns (L <= 112) per 256-thread workgroup (3 per CU); each
// wave owns 16 rows x 7 MFMA 16x16 accumulators.  Every workgroup writes a deterministic per-row-tile
// partial; a second tiny kernel sums the partials in a fixed order (bitwise reproducible, no
// float atomics).
#include "common.h"
#include <cstdlib>

namespace {

constexpr int BK = 16, NCOL = 112, NTILE = NCOL / 16;
// Row tile: 64 rows / 4 waves (default) or 128 rows / 8 waves (PFML_QUAD_ROWS=128: every beta
// tile staged in LDS feeds twice the MFMAs, half the workgroups and prologues).  Measured on
// the headline step: 6.64 ms (64) vs 6.76 ms (128) - the longer triangular K loops of the
// 128-row tiles cost more than the shared beta staging saves - so 64 stays the default.
int quad_rows() {
  static int r = [] {
    const char* e = getenv("PFML_QUAD_ROWS");
    return (e && atoi(e) == 128) ? 128 : 64;
  }();
  return r;
}
int quad_pf() {
  const char* e = getenv("PFML_QUAD_PF");
  return (e && atoi(e) == 2) ? 2 : 1;
}
// Both operands are staged k-contiguous, as they sit in HBM ([row][k] for D, [lambda][k] for
// beta), with a row stride of BK + 2 = 18 doubles: the coalesced global rows are stored
// without bank conflicts, and a fragment read (16 rows x 2 k per 32-lane group) hits 32
// distinct bank pairs.  (A [k][row] image made every staging store a 16-way conflict.)
constexpr int KS = BK + 2;

struct JobDesc {
  int64_t d_off;     // offset of D_t (P x P, ld ldD)
  int64_t r_off;     // offset of r_t
  int64_t b_off;     // offset of beta block [L][ldB]
  int64_t o_off;     // offset of this job's L utilities in obj
  int n;             // p + 1
  int ptile0;        // first partial slot of this job
};

// PF: global->register prefetch distance.  PF = 1 (default): one register set and the
// epilogue's cross-wave sums in the A staging buffer, so the kernel fits 3 workgroups per CU
// (155 VGPRs, 51.6 KB LDS) and the other workgroups hide the shorter prefetch.  PF = 2
// (PFML_QUAD_PF=2): two register sets, the loads of step k+2 in flight while step k computes,
// 222 VGPRs + AGPRs, 2 workgroups per CU.  Measured (tools/bench_quad.py, n = 513 jobs of the
// headline step): 1.20 ms (PF 1) vs 1.33 ms (PF 2); headline step 6.37-6.49 vs 6.52-6.60 ms
// (profiles/r02_quad_pf_ab.json).
template <int BM, int PF>
__global__ __launch_bounds__(BM * 4, PF == 1 ? 3 : 1) void quadform_kernel(
    const double* __restrict__ D, int64_t ldD, const double* __restrict__ R,
    const double* __restrict__ Bt, int64_t ldB, const JobDesc* __restrict__ jobs,
    const int* __restrict__ tile_job, int L, double* __restrict__ partial) {
  constexpr int NT = BM * 4;                      // threads: one wave per 16 rows
  constexpr int NW = NT / 64;
  __shared__ double As[2][BM][KS];
  __shared__ double Bs[2][NCOL][KS];
  __shared__ double red_own[PF == 1 ? 1 : NW][NCOL];
  static_assert(NW * NCOL <= 2 * BM * KS, "cross-wave sums must fit in the A buffers");
  double (*red)[NCOL] = PF == 1 ? reinterpret_cast<double (*)[NCOL]>(&As[0][0][0]) : red_own;

  // tile_job[tile] = job << 5 | row tile: the host lists the tiles longest-first (all row
  // tiles 0, then all 1, ...: the triangular K loop shrinks with the row tile), so the launch
  // ends on short tiles instead of a 33-step one; the partial slot stays ptile0 + rt
  const int tile = blockIdx.x;
  const int tj = tile_job[tile];
  const int j = tj >> 5;
  const JobDesc jd = jobs[j];
  const int rt = tj & 31;                    // row tile within the job
  const int i0 = rt * BM;
  const int n = jd.n;
  const double* Dm = D + jd.d_off;
  const double* r = R + jd.r_off;
  const double* bt = Bt + jd.b_off;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;

  double4_t acc[NTILE];
#pragma unroll
  for (int q = 0; q < NTILE; ++q) acc[q] = double4_t{0.0, 0.0, 0.0, 0.0};

  // D_t is symmetric:  b'Db = sum_I b_I'(D_II b_I + 2 sum_{K>I} D_IK b_K).  A row tile I only
  // walks K >= I, with the diagonal block weighted 1/2, so  acc = U_I / 2  and half the
  // flops and D bytes of the full product are spent.  K tiles are double-buffered in LDS
  // and prefetched two steps ahead through registers (one barrier per K step).
  constexpr int AQ = (BM * BK) / NT;              // D elements per thread per K step
  constexpr int BQ = (NCOL * BK + NT - 1) / NT;   // beta elements per thread per K step
  // two register sets: the global loads of step k+2 are in flight while step k is computed
  // from LDS and step k+1 is written to the other LDS buffer (prefetch distance 2).
  double ra0[AQ], rb0[BQ], ra1[AQ], rb1[BQ];
  // Loads are unconditional (indices clamped into the matrix) and the masking / diagonal
  // weight is applied when the registers are written to LDS: a load under a branch with its
  // use in the same block made the compiler wait for every D element right after issuing it.
  auto gload = [&](int k0, double (&ra)[AQ], double (&rb)[BQ]) {
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
      const int e = t + q * NT, i = e / BK, k = e % BK;
      ra[q] = Dm[(int64_t)min(i0 + i, n - 1) * ldD + min(k0 + k, n - 1)];
    }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int e = min(t + q * NT, NCOL * BK - 1), l = e / BK, k = e % BK;
      rb[q] = bt[(int64_t)min(l, L - 1) * ldB + min(k0 + k, n - 1)];
    }
  };
  auto sstore = [&](int buf, int k0, const double (&ra)[AQ], const double (&rb)[BQ]) {
    const double wdiag = (k0 < i0 + BM) ? 0.5 : 1.0;
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
      const int e = t + q * NT, i = e / BK, k = e % BK;
      As[buf][i][k] = (i0 + i < n && k0 + k < n) ? wdiag * ra[q] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int e = t + q * NT, l = e / BK, k = e % BK;
      if (e < NCOL * BK) Bs[buf][l][k] = (l < L && k0 + k < n) ? rb[q] : 0.0;
    }
  };
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const double a = As[buf][w * 16 + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
      for (int q = 0; q < NTILE; ++q)
        acc[q] = mfma_f64_16x16x4(a, Bs[buf][q * 16 + (lane & 15)][kk + (lane >> 4)], acc[q]);
    }
  };
  if constexpr (PF == 1) {
    gload(i0, ra0, rb0);
    sstore(0, i0, ra0, rb0);
    __syncthreads();
    int buf = 0;
    for (int k0 = i0;;) {
      const bool more = k0 + BK < n;
      if (more) gload(k0 + BK, ra0, rb0);
      compute(buf);
      if (!more) break;
      sstore(buf ^ 1, k0 + BK, ra0, rb0);
      __syncthreads();
      k0 += BK;
      buf ^= 1;
    }
    __syncthreads();                          // red reuses As
  } else {
  gload(i0, ra0, rb0);
  sstore(0, i0, ra0, rb0);
  if (i0 + BK < n) gload(i0 + BK, ra1, rb1);
  __syncthreads();
  for (int k0 = i0;;) {
    if (k0 + 2 * BK < n) gload(k0 + 2 * BK, ra0, rb0);
    compute(0);
    if (k0 + BK >= n) break;
    sstore(1, k0 + BK, ra1, rb1);
    __syncthreads();
    k0 += BK;
    if (k0 + 2 * BK < n) gload(k0 + 2 * BK, ra1, rb1);
    compute(1);
    if (k0 + BK >= n) break;
    sstore(0, k0 + BK, ra0, rb0);
    __syncthreads();
    k0 += BK;
  }
  }

  // epilogue: sum over this wave's 16 rows of  beta_l[i] * (r_i - 1/2 U[i][l])
#pragma unroll
  for (int q = 0; q < NTILE; ++q) {
    const int l = q * 16 + (lane & 15);
    double s = 0.0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int gi = i0 + w * 16 + PFML_F64_CROW(lane, rr);
      if (gi < n && l < L) {
        const double b = bt[(int64_t)l * ldB + gi];
        s += b * (r[gi] - acc[q][rr]);          // acc = U / 2 (symmetric half)
      }
    }
    // lanes l, l+16, l+32, l+48 share the column
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (lane < 16) red[w][l] = s;
  }
  __syncthreads();
  if (t < NCOL) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += red[q][t];
    if (t < L) partial[(int64_t)(jd.ptile0 + rt) * L + t] = s;
  }
}

__global__ void quadform_reduce_kernel(const double* __restrict__ partial,
                                       const JobDesc* __restrict__ jobs, int njobs, int L,
                                       int BM, double* __restrict__ obj) {
  const int j = blockIdx.x;
  const int l = threadIdx.x;
  if (j >= njobs || l >= L) return;
  const JobDesc jd = jobs[j];
  const int nt = (jd.n + BM - 1) / BM;
  double s = 0.0;
  for (int q = 0; q < nt; ++q) s += partial[(int64_t)(jd.ptile0 + q) * L + l];
  obj[jd.o_off + l] = s;
}

}  // namespace

extern "C" int pfml_quadform_job_desc_size() { return (int)sizeof(JobDesc); }
extern "C" int pfml_quadform_rows_per_tile() { return quad_rows(); }

extern "C" hipError_t pfml_quadform(const double* D, int64_t ldD, const double* R,
                                    const double* Bt, int64_t ldB, const void* jobs, int njobs,
                                    const int* tile_job, int ntiles, int L, double* partial,
                                    double* obj, hipStream_t st) {
  if (njobs <= 0) return hipSuccess;
  if (L > NCOL) return hipErrorInvalidValue;
  const int bm = quad_rows();
  if (bm == 128)
    hipLaunchKernelGGL((quadform_kernel<128, 2>), dim3(ntiles), dim3(512), 0, st, D, ldD, R, Bt,
                       ldB, static_cast<const JobDesc*>(jobs), tile_job, L, partial);
  else if (quad_pf() == 1)
    hipLaunchKernelGGL((quadform_kernel<64, 1>), dim3(ntiles), dim3(256), 0, st, D, ldD, R, Bt,
                       ldB, static_cast<const JobDesc*>(jobs), tile_job, L, partial);
  else
    hipLaunchKernelGGL((quadform_kernel<64, 2>), dim3(ntiles), dim3(256), 0, st, D, ldD, R, Bt,
                       ldB, static_cast<const JobDesc*>(jobs), tile_job, L, partial);
  hipLaunchKernelGGL(quadform_reduce_kernel, dim3(njobs), dim3(128), 0, st, partial,
                     static_cast<const JobDesc*>(jobs), njobs, L, bm, obj);
  return hipGetLastError();
}
