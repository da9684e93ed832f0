// The sequential part of the PFML weight recursion (PFML_best_hps.py:168-218, eq. (17)):
//
//   for t:  d      = (w_start - w_aim_t) / a_t
//           w_opt  = w_aim_t + a_t o (m_tilde_t d)           (m_t = diag(a) m_tilde diag(1/a))
//           w_start(t+1)[r] = hit[r] ? w_opt[map[r]] * grow_t[map[r]] : 0
//
// Every month depends on the previous one, so the chain is one persistent workgroup that
// loops over the months (one launch instead of ~7 small launches + a host round trip per
// month).  The N-vectors live in LDS; m_tilde_t (N x N, the only large operand) streams
// through once per month in coalesced row reads, 16 waves x one row each per pass, the dot
// products reduced across the wave with DPP/shuffles.  Every wave exits after the last month
// (no waiting on other workgroups: the grid is this one workgroup).
#include "common.h"

namespace {

constexpr int WT = 1024;
constexpr int WW = WT / 64;
constexpr int WMAX = 2048;             // N held in LDS (3 vectors: 48 KB)

__global__ __launch_bounds__(WT) void weights_chain_kernel(
    const double* __restrict__ mt, int64_t ldm, int64_t sm, const double* __restrict__ a,
    const double* __restrict__ wa, const double* __restrict__ grow,
    const int64_t* __restrict__ nmap, const double* __restrict__ hit, int64_t sv,
    const double* __restrict__ ws0, int B, int N, double* __restrict__ Wst,
    double* __restrict__ Wopt, double* __restrict__ ws_out) {
  __shared__ double ws[WMAX], d[WMAX], wo[WMAX];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int j = t; j < N; j += WT) ws[j] = ws0[j];
  __syncthreads();
  for (int m = 0; m < B; ++m) {
    const double* am = a + (int64_t)m * sv;
    const double* wam = wa + (int64_t)m * sv;
    for (int j = t; j < N; j += WT) {
      Wst[(int64_t)m * sv + j] = ws[j];
      d[j] = (ws[j] - wam[j]) / am[j];
    }
    __syncthreads();
    const double* M = mt + (int64_t)m * sm;
    for (int i = w; i < N; i += WW) {
      const double* row = M + (int64_t)i * ldm;
      double s0 = 0.0, s1 = 0.0;
      int j = lane;
      for (; j + 64 < N; j += 128) {
        s0 += row[j] * d[j];
        s1 += row[j + 64] * d[j + 64];
      }
      if (j < N) s0 += row[j] * d[j];
      double s = s0 + s1;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
      if (lane == 0) {
        const double v = wam[i] + am[i] * s;
        wo[i] = v;
        Wopt[(int64_t)m * sv + i] = v;
      }
    }
    __syncthreads();
    const double* gm = grow + (int64_t)m * sv;
    const int64_t* nm = nmap + (int64_t)m * sv;
    const double* hm = hit + (int64_t)m * sv;
    for (int r = t; r < N; r += WT) {
      const int64_t q = nm[r];
      ws[r] = (wo[q] * gm[q]) * hm[r];
    }
    __syncthreads();
  }
  for (int j = t; j < N; j += WT) ws_out[j] = ws[j];
}

}  // namespace

extern "C" int pfml_weights_chain_max_n() { return WMAX; }

// mt: [B, N, N] (row stride ldm, batch stride sm); a, wa, grow, hit: [B, N] doubles and nmap
// [B, N] int64 (batch stride sv, entries in [0, N)); ws0 [N]; outputs Wst, Wopt [B, N] (stride
// sv) and ws_out [N] (the w_start of the month after the last).
extern "C" hipError_t pfml_weights_chain(const double* mt, int64_t ldm, int64_t sm,
                                         const double* a, const double* wa, const double* grow,
                                         const int64_t* nmap, const double* hit, int64_t sv,
                                         const double* ws0, int B, int N, double* Wst,
                                         double* Wopt, double* ws_out, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  if (N > WMAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(weights_chain_kernel, dim3(1), dim3(WT), 0, st, mt, ldm, sm, a, wa, grow,
                     nmap, hit, sv, ws0, B, N, Wst, Wopt, ws_out);
  return hipGetLastError();
}
