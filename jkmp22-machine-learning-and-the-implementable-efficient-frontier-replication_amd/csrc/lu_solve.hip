// Batched general solve  A X = B  by blocked Gauss-Jordan elimination with partial pivoting
// (omega = solve(const, Omega), PFML_Input_Data.py:455-456; np.linalg.solve
// semantics - const = sum_theta agg_theta is not symmetric).
//
// The system is stored augmented, one row per equation: M = [ ... B (m cols) ... A (n cols) ...]
// with B at column b0 and A at column a0 of each row (leading dimension ldm).  This is exactly
// the layout the Horner aggregation produces ([Omega | const]), so no copies are made.
// For each block column k (width NB) of A:
//   1. pivot search: partial-pivoting LU of the panel A[k0:, k-block] in LDS picks NB pivot rows
//      (LAPACK-style sequential swap list);
//   2. the swaps are applied to every live column (A cols >= k0 and all B cols);
//   3. P = A_kk^-1 (Gauss-Jordan in LDS, pivots non-zero by construction);
//   4. row panel R = P M_k (live columns); the column panel C = M[:, k-block] is read in place;
//   5. all other rows: M_i -= C_i R  (rank-NB update on fp64 MFMA); block rows: M_k = R.
// Columns of A left of the current block are never touched again (they would hold the
// identity), so the work is n^3 + 2 n^2 m flops like an LU solve.
#include "common.h"

namespace {

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// Block width NB and the panel rows PMAX held in LDS: NB = 32 for n <= 512 (half the passes
// over the augmented rows of NB = 16; the 512 x 33 panel is 135 KB of LDS), NB = 16 up to
// n = 1024; longer panels (n <= 3072, the 3000-stock stress) are pivoted in registers
// (lu_pivot_reg_kernel).  The trailing update is bandwidth-bound (each pass reads and writes the live
// part of every row), so the pass count sets its time.

// live column v (0 .. nlive-1) -> physical column
__device__ __forceinline__ int live_col(int v, int nA_live, int a_first, int b0) {
  return v < nA_live ? a_first + v : b0 + (v - nA_live);
}

// 1024 threads (16 waves): the panel takes 135 KB of LDS, so one workgroup per CU - the
// row loops of the argmax and the elimination are spread over 16 waves instead of 4.
template <int NB, int PMAX>
__global__ __launch_bounds__(1024) void lu_pivot_kernel(const double* __restrict__ M, int n,
                                                        int64_t ldm, int64_t sM, int a0, int k0,
                                                        int nb, int* __restrict__ piv,
                                                        int* __restrict__ status) {
  constexpr int NT = 1024, NW = NT / 64;
  __shared__ double Pn[PMAX][NB + 1];
  __shared__ double rv[NW];
  __shared__ int ri[NW];
  const int b = blockIdx.x;
  const double* Mb = M + (int64_t)b * sM;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int rows = n - k0;
  for (int e = t; e < rows * nb; e += NT) {
    const int i = e / nb, j = e % nb;
    Pn[i][j] = Mb[(int64_t)(k0 + i) * ldm + a0 + k0 + j];
  }
  __syncthreads();
  for (int j = 0; j < nb; ++j) {
    // argmax |Pn[i][j]|, i in [j, rows)
    double best = -1.0;
    int bi = j;
    for (int i = j + t; i < rows; i += NT) {
      const double v = fabs(Pn[i][j]);
      if (v > best) { best = v; bi = i; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_xor(best, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane == 0) { rv[w] = best; ri[w] = bi; }
    __syncthreads();
    if (t == 0) {
      double bv = rv[0];
      int bx = ri[0];
      for (int q = 1; q < NW; ++q)
        if (rv[q] > bv || (rv[q] == bv && ri[q] < bx)) { bv = rv[q]; bx = ri[q]; }
      ri[0] = bx;
      piv[(int64_t)b * NB + j] = k0 + bx;
      if (!(bv > 0.0) || !isfinite(bv)) status[b] = 1;
    }
    __syncthreads();
    const int p = ri[0];
    if (p != j && t < nb) {
      const double tmp = Pn[j][t];
      Pn[j][t] = Pn[p][t];
      Pn[p][t] = tmp;
    }
    __syncthreads();
    const double pv = Pn[j][j];
    // (rows x columns of the trailing panel over all 1024 threads)
    const int nc = nb - j - 1;
    if (nc > 0) {
      for (int e = t; e < (rows - j - 1) * nc; e += NT) {
        const int i = j + 1 + e / nc, c = j + 1 + e % nc;
        Pn[i][c] -= (Pn[i][j] / pv) * Pn[j][c];
      }
    }
    __syncthreads();
    // the multipliers column is not stored (only the pivot order leaves the kernel)
  }
}

// Pivot search for tall panels (n - k0 > 1024 rows, up to R * 1024): the panel lives in
// REGISTERS of a 1024-thread workgroup - thread t holds rows t, t + 1024, ... (R rows x NB
// columns; the last RL row sets in a thread-private LDS slot when R rows would spill) -
// instead of a shared LDS panel (a 3000 x 16 panel is 384 KB).  One barrier per column: before it
// each wave posts its best candidate row (value, index, the row's NB entries) and thread j
// posts the current row j, so after it every thread knows the pivot row's values and the
// owners of rows j and p swap in registers (double-buffered posts: the next column writes the
// other buffer).  Same pivot choice (first index of the maximum |a|) and the same elimination
// arithmetic as lu_pivot_kernel, so both forms pick the same pivots.
template <int NB, int R, int RL, int NTT = 1024>
__global__ __launch_bounds__(NTT) void lu_pivot_reg_kernel(const double* __restrict__ M, int n,
                                                           int64_t ldm, int64_t sM, int a0,
                                                           int k0, int nb,
                                                           int* __restrict__ piv,
                                                           int* __restrict__ status) {
  constexpr int NT = NTT, NW = NT / 64, RR = R - RL;
  static_assert(NT > NB, "thread j posts row j");
  __shared__ double cand[2][NW][NB];
  __shared__ double cval[2][NW];
  __shared__ int cidx[2][NW];
  __shared__ double rowj[2][NB];
  __shared__ double al[RL > 0 ? RL : 1][NB][NT];   // the last RL row sets (thread-private)
  const int b = blockIdx.x;
  const double* Mb = M + (int64_t)b * sM;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int rows = n - k0;
  double a[RR][NB];
  // element (row set r, column c) of this thread: registers for r < RR, LDS for the rest
  auto el = [&](auto RI, int c) -> double& {
    constexpr int r = decltype(RI)::value;
    if constexpr (r < RR) return a[r][c];
    else return al[r - RR][c][t];
  };
  static_for<0, R>([&](auto RI) {
    constexpr int r = decltype(RI)::value;
    const int i = t + r * NT;
    const double* src = Mb + (int64_t)(k0 + min(i, rows - 1)) * ldm + a0 + k0;
#pragma unroll
    for (int c = 0; c < NB; ++c) el(RI, c) = (i < rows && c < nb) ? src[min(c, nb - 1)] : 0.0;
  });
  static_for<0, NB>([&](auto J) {
    constexpr int j = decltype(J)::value;
    if (j >= nb) return;                            // (uniform: nb is a kernel argument)
    const int buf = j & 1;
    // own candidate: first row of the largest |a[.][j]| among rows i >= j
    double best = -1.0;
    int bi = 0x7fffffff;
    static_for<0, R>([&](auto RI) {
      constexpr int r = decltype(RI)::value;
      const int i = t + r * NT;
      const double v = fabs(el(RI, j));
      if (i >= j && i < rows && v > best) { best = v; bi = i; }
    });
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_xor(best, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane == 0) { cval[buf][w] = best; cidx[buf][w] = bi; }
    if (bi != 0x7fffffff && (bi % NT) == t) {      // the wave's winner posts its row
      static_for<0, R>([&](auto RI) {
        constexpr int r = decltype(RI)::value;
        if (r == bi / NT) {
#pragma unroll
          for (int c = 0; c < NB; ++c) cand[buf][w][c] = el(RI, c);
        }
      });
    }
    if (t == j) {                                   // current row j (rows < 32: set 0)
#pragma unroll
      for (int c = 0; c < NB; ++c) rowj[buf][c] = a[0][c];
    }
    __syncthreads();
    double bv = cval[buf][0];
    int bx = cidx[buf][0], bw = 0;
#pragma unroll
    for (int q = 1; q < NW; ++q) {
      const double v = cval[buf][q];
      const int x = cidx[buf][q];
      if (v > bv || (v == bv && x < bx)) { bv = v; bx = x; bw = q; }
    }
    if (t == 0) {
      piv[(int64_t)b * NB + j] = k0 + bx;
      if (!(bv > 0.0) || !isfinite(bv)) status[b] = 1;
    }
    const double* prow = cand[buf][bw];             // pivot row, read from LDS where used
    // swap: row j <- pivot row, row p <- old row j
    if (bx != j && (bx % NT) == t) {
      static_for<0, R>([&](auto RI) {
        constexpr int r = decltype(RI)::value;
        if (r == bx / NT) {
#pragma unroll
          for (int c = 0; c < NB; ++c) el(RI, c) = rowj[buf][c];
        }
      });
    }
    if (t == j) {
#pragma unroll
      for (int c = 0; c < NB; ++c) a[0][c] = prow[c];
    }
    const double pv = prow[j];
    static_for<0, R>([&](auto RI) {
      constexpr int r = decltype(RI)::value;
      const int i = t + r * NT;
      if (i > j && i < rows) {
        const double l = el(RI, j) / pv;
#pragma unroll
        for (int c = j + 1; c < NB; ++c) el(RI, c) -= l * prow[c];
      }
    });
  });
}

// pivot search of block k0 by the LDS form (rows <= PMAX) or the register form (longer panels)
template <int NB, int PMAX>
hipError_t lu_pivot_launch(const double* M, int n, int64_t ldm, int64_t sM, int a0, int k0,
                           int nb, int* piv, int* status, int batch, hipStream_t st) {
  const int rows = n - k0;
#ifndef PFML_LU_PIVOT_LDS
  // 32-wide panels of up to 1024 rows in registers (one row per thread): one barrier per
  // column and ~8 KB of LDS, so two workgroups share a CU - the LDS form's 135 KB panel
  // allowed one, and its elimination spent an integer division per element (same pivots,
  // same arithmetic)
  // (the workgroup shrinks with the panel: 256 / 512 threads for panels of <= 256 / 512 rows,
  // so more matrices' panels run per CU - the panel's rows, not the threads, are the work)
  if constexpr (NB == 32) {
    if (rows <= 256) {
      hipLaunchKernelGGL((lu_pivot_reg_kernel<NB, 1, 0, 256>), dim3(batch), dim3(256), 0, st, M,
                         n, ldm, sM, a0, k0, nb, piv, status);
      return hipSuccess;
    }
    if (rows <= 512) {
      hipLaunchKernelGGL((lu_pivot_reg_kernel<NB, 1, 0, 512>), dim3(batch), dim3(512), 0, st, M,
                         n, ldm, sM, a0, k0, nb, piv, status);
      return hipSuccess;
    }
    if (rows <= 1024) {
      hipLaunchKernelGGL((lu_pivot_reg_kernel<NB, 1, 0>), dim3(batch), dim3(1024), 0, st, M, n,
                         ldm, sM, a0, k0, nb, piv, status);
      return hipSuccess;
    }
  }
#endif
  if (rows <= PMAX) {
    hipLaunchKernelGGL((lu_pivot_kernel<NB, PMAX>), dim3(batch), dim3(1024), 0, st, M, n, ldm,
                       sM, a0, k0, nb, piv, status);
    return hipSuccess;
  }
  if constexpr (NB == 16) {          // (NB = 32 panels would not fit the register budget)
    if (rows <= 2048) {
      hipLaunchKernelGGL((lu_pivot_reg_kernel<NB, 2, 0>), dim3(batch), dim3(1024), 0, st, M, n,
                         ldm, sM, a0, k0, nb, piv, status);
      return hipSuccess;
    }
    if (rows <= 3072) {
      hipLaunchKernelGGL((lu_pivot_reg_kernel<NB, 3, 1>), dim3(batch), dim3(1024), 0, st, M, n,
                         ldm, sM, a0, k0, nb, piv, status);
      return hipSuccess;
    }
  }
  return hipErrorInvalidValue;
}

// apply the NB sequential row swaps of block k0 to every live column (+ block k's own A cols)
template <int NB>
__global__ __launch_bounds__(256) void lu_swap_kernel(double* __restrict__ M, int64_t ldm,
                                                      int64_t sM, int ncol, int a_first, int nA,
                                                      int b0, int k0, int nb,
                                                      const int* __restrict__ piv) {
  const int b = blockIdx.y;
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= ncol) return;
  const int c = live_col(v, nA, a_first, b0);
  double* Mb = M + (int64_t)b * sM;
  const int* pb = piv + (int64_t)b * NB;
  for (int j = 0; j < nb; ++j) {
    const int p = pb[j];
    if (p != k0 + j) {
      double* x = Mb + (int64_t)(k0 + j) * ldm + c;
      double* y = Mb + (int64_t)p * ldm + c;
      const double tmp = *x;
      *x = *y;
      *y = tmp;
    }
  }
}

// P = A_kk^-1 by Gauss-Jordan without pivoting (rows already pivoted)
template <int NB>
__global__ __launch_bounds__(256) void lu_blockinv_kernel(const double* __restrict__ M,
                                                          int64_t ldm, int64_t sM, int a0, int k0,
                                                          int nb, double* __restrict__ Pbuf) {
  __shared__ double P[NB][NB + 1];
  const int b = blockIdx.x;
  const double* Mb = M + (int64_t)b * sM;
  const int t = threadIdx.x;
  for (int e = t; e < nb * nb; e += 256) P[e / nb][e % nb] = Mb[(int64_t)(k0 + e / nb) * ldm + a0 + k0 + e % nb];
  __syncthreads();
  for (int p = 0; p < nb; ++p) {
    const double inv = 1.0 / P[p][p];
    __syncthreads();
    for (int e = t; e < nb * nb; e += 256) {
      const int i = e / nb, j = e % nb;
      if (i != p && j != p) P[i][j] -= P[i][p] * P[p][j] * inv;
    }
    __syncthreads();
    for (int e = t; e < nb; e += 256)
      if (e != p) { P[p][e] *= inv; P[e][p] *= -inv; }
    if (t == 0) P[p][p] = inv;
    __syncthreads();
  }
  for (int e = t; e < NB * NB; e += 256) {
    const int i = e / NB, j = e % NB;
    Pbuf[(int64_t)b * NB * NB + e] = (i < nb && j < nb) ? P[i][j] : 0.0;
  }
}

// The same inverse for NB = 32 with the block in registers (thread (ti, tj) of 256 holds rows
// 2 ti.., columns 2 tj..): the owners post pivot row / column p to a double-buffered LDS line,
// ONE barrier per pivot instead of four (the LDS form re-read and re-wrote the whole block
// around each pivot: ~33 us per call, latency, at the ~60-matrix batches of a many-GPU run's
// per-rank S4).  Every element takes the same operations on the same values in the same
// order: bitwise the LDS form.
template <int NB>
__global__ __launch_bounds__(256) void lu_blockinv_reg_kernel(const double* __restrict__ M,
                                                              int64_t ldm, int64_t sM, int a0,
                                                              int k0, int nb,
                                                              double* __restrict__ Pbuf) {
  static_assert(NB == 32, "2 x 2 elements per thread of 256");
  __shared__ double rowp[2][NB], colp[2][NB];
  const int b = blockIdx.x, t = threadIdx.x;
  const int ti = t >> 4, tj = t & 15;
  const double* Mb = M + (int64_t)b * sM;
  double x[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int i = 2 * ti + u, j = 2 * tj + v;
      x[u][v] = (i < nb && j < nb) ? Mb[(int64_t)(k0 + i) * ldm + a0 + k0 + j] : 0.0;
    }
  for (int p = 0; p < nb; ++p) {
    const int buf = p & 1, h = p & 1;
    if (ti == (p >> 1)) {
      rowp[buf][2 * tj] = x[h][0];
      rowp[buf][2 * tj + 1] = x[h][1];
    }
    if (tj == (p >> 1)) {
      colp[buf][2 * ti] = x[0][h];
      colp[buf][2 * ti + 1] = x[1][h];
    }
    __syncthreads();
    const double inv = 1.0 / rowp[buf][p];
    const double rp[2] = {rowp[buf][2 * tj], rowp[buf][2 * tj + 1]};
    const double cp[2] = {colp[buf][2 * ti], colp[buf][2 * ti + 1]};
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int i = 2 * ti + u, j = 2 * tj + v;
        if (i < nb && j < nb) {
          if (i != p && j != p) x[u][v] -= cp[u] * rp[v] * inv;
          else if (i == p && j != p) x[u][v] *= inv;
          else if (i != p) x[u][v] *= -inv;
          else x[u][v] = inv;
        }
      }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int i = 2 * ti + u, j = 2 * tj + v;
      Pbuf[(int64_t)b * NB * NB + i * NB + j] = (i < nb && j < nb) ? x[u][v] : 0.0;
    }
}

template <int NB>
void lu_blockinv_launch(const double* M, int64_t ldm, int64_t sM, int a0, int k0, int nb,
                        double* Pbuf, int batch, hipStream_t st) {
  if constexpr (NB == 32)
    hipLaunchKernelGGL((lu_blockinv_reg_kernel<NB>), dim3(batch), dim3(256), 0, st, M, ldm, sM,
                       a0, k0, nb, Pbuf);
  else
    hipLaunchKernelGGL((lu_blockinv_kernel<NB>), dim3(batch), dim3(256), 0, st, M, ldm, sM, a0,
                       k0, nb, Pbuf);
}

// R = P M_k over live columns (excluding block k's own A columns) -> Rbuf [NB][nlive].  Live
// columns v >= vz are virtual: the two-level form's Z columns of the current inner block, whose
// rows k0.. hold the unit vectors e_(v - vz) (not stored: no zero-fill or unit pass of Z)
template <int NB>
__global__ __launch_bounds__(256) void lu_rowpanel_kernel(const double* __restrict__ M, int64_t ldm,
                                                          int64_t sM, int nlive, int a_first,
                                                          int nA, int b0, int k0, int nb,
                                                          const double* __restrict__ Pbuf,
                                                          double* __restrict__ Rbuf, int vz) {
  __shared__ double P[NB][NB + 1];
  const int b = blockIdx.y;
  const int t = threadIdx.x;
  for (int e = t; e < NB * NB; e += 256) P[e / NB][e % NB] = Pbuf[(int64_t)b * NB * NB + e];
  __syncthreads();
  const int v = blockIdx.x * 256 + t;
  if (v >= nlive) return;
  const int c = live_col(v, nA, a_first, b0);
  const double* Mb = M + (int64_t)b * sM;
  double col[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q)
    col[q] = (v >= vz) ? (q == v - vz ? 1.0 : 0.0)
                       : ((q < nb) ? Mb[(int64_t)(k0 + q) * ldm + c] : 0.0);
  double* Rb = Rbuf + (int64_t)b * NB * nlive;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NB; ++q) s += P[i][q] * col[q];
    if (i < nb) Rb[(int64_t)i * nlive + v] = s;
  }
}

// rows outside block k: M_i -= C_i R ; block rows: M_k = R   (live columns only; virtual
// columns v >= vz, see lu_rowpanel_kernel, read as 0).  C = block k's own A columns (from
// column c0 = a0 + k0), read in place: they are not live, so no tile of this launch writes
// them (a snapshot copy of them per step cost a pass of its own).
template <int NB>
__global__ __launch_bounds__(256) void lu_update_kernel(double* __restrict__ M, int n, int64_t ldm,
                                                        int64_t sM, int nlive, int a_first, int nA,
                                                        int b0, int k0, int nb,
                                                        const double* __restrict__ Rbuf, int c0,
                                                        int vz) {
  constexpr int BT = 64;
  __shared__ double Cs[NB][BT + 16];
  __shared__ double Rs[NB][BT + 16];
  const int b = blockIdx.y;
  double* Mb = M + (int64_t)b * sM;
  const double* Rb = Rbuf + (int64_t)b * NB * nlive;
  const double* Cb = Mb + c0;
  const int tc = (nlive + BT - 1) / BT;
  const int I0 = (blockIdx.x / tc) * BT, V0 = (blockIdx.x % tc) * BT;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  // staging: every load in flight at once (clamped, unconditional), masked at the LDS store
  constexpr int QS = BT * NB / 256;
  double cv[QS], rv[QS];
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    const int e = t + u * 256;
    cv[u] = Cb[(int64_t)min(I0 + e / NB, n - 1) * ldm + min(e % NB, nb - 1)];
    rv[u] = Rb[(int64_t)min(e / BT, nb - 1) * nlive + min(V0 + e % BT, nlive - 1)];
  }
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    const int e = t + u * 256;
    const int i = e / NB, q = e % NB;
    Cs[q][i] = (I0 + i < n && q < nb) ? cv[u] : 0.0;
    const int q2 = e / BT, j = e % BT;
    Rs[q2][j] = (V0 + j < nlive && q2 < nb) ? rv[u] : 0.0;
  }
  __syncthreads();
  double4_t acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = double4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < NB; q += 4) {
    double a[2], bb[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) a[x] = Cs[q + (lane >> 4)][wm * 32 + x * 16 + (lane & 15)];
#pragma unroll
    for (int y = 0; y < 2; ++y) bb[y] = Rs[q + (lane >> 4)][wn * 32 + y * 16 + (lane & 15)];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = mfma_f64_16x16x4(a[x], bb[y], acc[x][y]);
  }
  // epilogue: gather the old values (and the new block rows) first, then write - one memory
  // latency for the tile instead of one read-modify-write round trip per element
  double old[2][2][4], nrow[2][2][4];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = min(I0 + wm * 32 + x * 16 + PFML_F64_CROW(lane, r), n - 1);
        const int v = min(V0 + wn * 32 + y * 16 + (lane & 15), nlive - 1);
        // (virtual live columns v >= vz: zero outside the block rows, which take R)
        old[x][y][r] = v >= vz ? 0.0 : Mb[(int64_t)i * ldm + live_col(v, nA, a_first, b0)];
        nrow[x][y][r] = Rb[(int64_t)min(max(i - k0, 0), nb - 1) * nlive + v];
      }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = I0 + wm * 32 + x * 16 + PFML_F64_CROW(lane, r);
        const int v = V0 + wn * 32 + y * 16 + (lane & 15);
        if (i >= n || v >= nlive) continue;
        Mb[(int64_t)i * ldm + live_col(v, nA, a_first, b0)] =
            (i >= k0 && i < k0 + nb) ? nrow[x][y][r] : old[x][y][r] - acc[x][y][r];
      }
}


template <int NB, int PMAX>
hipError_t lu_solve_nb(double* M, int n, int m, int64_t ldm, int64_t sM, int a0, int b0,
                       int batch, double* work, int* status, hipStream_t st) {
  double* Pbuf = work;
  double* Rbuf = Pbuf + (int64_t)batch * NB * NB;
  int* piv = reinterpret_cast<int*>(Rbuf + (int64_t)batch * NB * (n + m));
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int nb = (n - k0 < NB) ? (n - k0) : NB;
    hipError_t e = lu_pivot_launch<NB, PMAX>(M, n, ldm, sM, a0, k0, nb, piv, status, batch, st);
    if (e != hipSuccess) return e;
    const int nswap = (n - k0) + m;           // A cols >= k0 and all B cols
    hipLaunchKernelGGL((lu_swap_kernel<NB>), dim3((nswap + 255) / 256, batch), dim3(256), 0, st,
                       M, ldm, sM, nswap, a0 + k0, n - k0, b0, k0, nb, piv);
    lu_blockinv_launch<NB>(M, ldm, sM, a0, k0, nb, Pbuf, batch, st);
    const int nA = n - (k0 + nb);            // live A columns right of the block
    const int nlive = nA + m;
    if (nlive > 0) {
      hipLaunchKernelGGL((lu_rowpanel_kernel<NB>), dim3((nlive + 255) / 256, batch), dim3(256), 0,
                         st, M, ldm, sM, nlive, a0 + k0 + nb, nA, b0, k0, nb, Pbuf, Rbuf, nlive);
      const int tiles = ((n + 63) / 64) * ((nlive + 63) / 64);
      hipLaunchKernelGGL((lu_update_kernel<NB>), dim3(tiles, batch), dim3(256), 0, st, M, n, ldm,
                         sM, nlive, a0 + k0 + nb, nA, b0, k0, nb, Rbuf, a0 + k0, nlive);
    }
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Two-level form (n <= 3072): 128-wide outer panels.  The 32-wide (n > 512: 16-wide) inner steps above run on the
// panel's own A columns plus a 128-column block Z of M (the inner update touches <= 256
// columns instead of all n + m), and Z accumulates the panel's Gauss-Jordan transform:
// the unit vector of each pivot row enters Z when its inner block is reached (after that
// block's row swaps), so at the end Z = T E_K with T the panel's transform after all of its
// swaps.  Z is never zero-filled or seeded: a block's Z columns are VIRTUAL in its own step
// (the row panel reads them as the unit vectors, the update as zeros outside the block rows)
// and that step's update writes every row of them.  The rest of M (A columns right of the panel and the B columns) then takes the
// swaps and T in one go:  R <- Perm R,  R_K <- Z_K R_K,  R_other <- R_other + Z_other R_K,
// i.e. three K = 128 fp64 MFMA GEMMs per column range (csrc/gemm_f64.hip) in place of four
// bandwidth-bound rank-32 passes over every live column.
constexpr int LU_KB = 128;

// RK[b][r][v] = M[K0 + r][live column v]   (rest columns: A right of the panel, then B)
__global__ __launch_bounds__(256) void lu_rk_kernel(const double* __restrict__ M, int64_t ldm,
                                                    int64_t sM, int K0, int kb, int nrest,
                                                    int a_first, int nA, int b0,
                                                    double* __restrict__ RK) {
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)kb * nrest) return;
  const int r = (int)(e / nrest), v = (int)(e % nrest);
  RK[(int64_t)b * kb * nrest + e] =
      M[(int64_t)b * sM + (int64_t)(K0 + r) * ldm + live_col(v, nA, a_first, b0)];
}

}  // namespace

extern "C" hipError_t pfml_dgemm(int ta, int tb, int M, int N, int K, int batch, double alpha,
                                 const double* A, int64_t lda, int64_t sA, const double* B,
                                 int64_t ldb, int64_t sB, double beta, double* C, int64_t ldc,
                                 int64_t sC, const double* rs, int64_t srs, const double* cs,
                                 int64_t scs, hipStream_t st);

namespace {

template <int NB, int PMAX>
hipError_t lu_solve_2level(double* M, int n, int m, int64_t ldm, int64_t sM, int a0, int b0,
                           int z0, int batch, double* work, int* status, hipStream_t st) {
  double* Pbuf = work;
  double* Rbuf = Pbuf + (int64_t)batch * NB * NB;
  double* RK = Rbuf + (int64_t)batch * NB * (2 * LU_KB);
  int* piv = reinterpret_cast<int*>(RK + (int64_t)batch * LU_KB * (n + m));
  for (int K0 = 0; K0 < n; K0 += LU_KB) {
    const int kb = (n - K0 < LU_KB) ? (n - K0) : LU_KB;
    const int aend = K0 + kb;
    for (int k0 = K0; k0 < aend; k0 += NB) {
      const int nb = (aend - k0 < NB) ? (aend - k0) : NB;
      int* pv = piv + (int64_t)((k0 - K0) / NB) * batch * NB;
      hipError_t e = lu_pivot_launch<NB, PMAX>(M, n, ldm, sM, a0, k0, nb, pv, status, batch, st);
      if (e != hipSuccess) return e;
      // live set of the inner step: A columns k0 .. aend (swap) / right of the block, and the
      // Z columns populated so far - the unit columns of the earlier inner blocks (swap) plus
      // this block's (update).  Z's later columns are still zero: a swap or a rank-NB update
      // of them is an exact no-op (x - C 0 = x), so they are not touched (the update streams
      // 128 + 128 instead of 224 / 192 / 160 / 128 columns per inner block)
      const int zlive = k0 - K0;
      const int nswap = (aend - k0) + zlive;
      hipLaunchKernelGGL((lu_swap_kernel<NB>), dim3((nswap + 255) / 256, batch), dim3(256), 0, st,
                         M, ldm, sM, nswap, a0 + k0, aend - k0, z0, k0, nb, pv);
      lu_blockinv_launch<NB>(M, ldm, sM, a0, k0, nb, Pbuf, batch, st);
      const int nA = aend - (k0 + nb);
      const int nlive = nA + zlive + nb;
      hipLaunchKernelGGL((lu_rowpanel_kernel<NB>), dim3((nlive + 255) / 256, batch), dim3(256), 0,
                         st, M, ldm, sM, nlive, a0 + k0 + nb, nA, z0, k0, nb, Pbuf, Rbuf,
                         nA + zlive);
      const int tiles = ((n + 63) / 64) * ((nlive + 63) / 64);
      hipLaunchKernelGGL((lu_update_kernel<NB>), dim3(tiles, batch), dim3(256), 0, st, M, n, ldm,
                         sM, nlive, a0 + k0 + nb, nA, z0, k0, nb, Rbuf, a0 + k0, nA + zlive);
    }
    // the rest: swaps in sequence order, then R_K <- Z_K R_K, R_other += Z_other R_K
    const int nAr = n - aend;
    const int nrest = nAr + m;
    if (nrest <= 0) continue;
    for (int k0 = K0; k0 < aend; k0 += NB) {
      const int nb = (aend - k0 < NB) ? (aend - k0) : NB;
      const int* pv = piv + (int64_t)((k0 - K0) / NB) * batch * NB;
      hipLaunchKernelGGL((lu_swap_kernel<NB>), dim3((nrest + 255) / 256, batch), dim3(256), 0, st,
                         M, ldm, sM, nrest, a0 + aend, nAr, b0, k0, nb, pv);
    }
    hipLaunchKernelGGL(lu_rk_kernel, dim3((int)(((int64_t)kb * nrest + 255) / 256), batch),
                       dim3(256), 0, st, M, ldm, sM, K0, kb, nrest, a0 + aend, nAr, b0, RK);
    const int64_t sRK = (int64_t)kb * nrest;
    const int ranges[2][3] = {{a0 + aend, nAr, 0}, {b0, m, nAr}};   // (column, width, RK offset)
    for (int c = 0; c < 2; ++c) {
      const int col = ranges[c][0], wdt = ranges[c][1], off = ranges[c][2];
      if (wdt <= 0) continue;
      const double* Bp = RK + off;
      const double* Zr = M + z0;
      hipError_t e;
      if (K0 > 0 && (e = pfml_dgemm(0, 0, K0, wdt, kb, batch, 1.0, Zr, ldm, sM, Bp, nrest, sRK,
                                    1.0, M + col, ldm, sM, nullptr, 0, nullptr, 0, st)) != hipSuccess)
        return e;
      if ((e = pfml_dgemm(0, 0, kb, wdt, kb, batch, 1.0, Zr + (int64_t)K0 * ldm, ldm, sM, Bp,
                          nrest, sRK, 0.0, M + (int64_t)K0 * ldm + col, ldm, sM, nullptr, 0,
                          nullptr, 0, st)) != hipSuccess)
        return e;
      if (n - aend > 0 &&
          (e = pfml_dgemm(0, 0, n - aend, wdt, kb, batch, 1.0, Zr + (int64_t)aend * ldm, ldm, sM,
                          Bp, nrest, sRK, 1.0, M + (int64_t)aend * ldm + col, ldm, sM, nullptr,
                          0, nullptr, 0, st)) != hipSuccess)
        return e;
    }
  }
  return hipGetLastError();
}

}  // namespace

extern "C" int pfml_lu_panel_cols() { return LU_KB; }

extern "C" int64_t pfml_lu_solve_work_doubles(int n, int m, int batch) {
  const int64_t NB = 32;                     // the larger block: enough for every variant
  return (int64_t)batch * (NB * NB + NB * (n + m + 2 * LU_KB) + (int64_t)LU_KB * (n + m)) +
         (int64_t)batch * LU_KB;             // pivots (ints, 4 inner blocks of NB)
}

// Solve A X = B in place for `batch` augmented systems (see header); X overwrites B.
extern "C" int pfml_lu_solve_max_n() { return 3072; }

extern "C" hipError_t pfml_lu_solve(double* M, int n, int m, int64_t ldm, int64_t sM, int a0,
                                    int b0, int batch, double* work, int* status,
                                    hipStream_t st) {
  if (n <= 0 || batch <= 0) return hipSuccess;
  if (n <= 512) return lu_solve_nb<32, 512>(M, n, m, ldm, sM, a0, b0, batch, work, status, st);
  if (n <= 3072) return lu_solve_nb<16, 1024>(M, n, m, ldm, sM, a0, b0, batch, work, status, st);
  return hipErrorInvalidValue;
}

// Two-level solve; M must hold LU_KB free columns at z0 (scratch for the panel transform).
extern "C" int pfml_lu_solve2_max_n() { return 3072; }

extern "C" hipError_t pfml_lu_solve2(double* M, int n, int m, int64_t ldm, int64_t sM, int a0,
                                     int b0, int z0, int batch, double* work, int* status,
                                     hipStream_t st) {
  if (n <= 0 || batch <= 0) return hipSuccess;
  if (n <= 512)
    return lu_solve_2level<32, 512>(M, n, m, ldm, sM, a0, b0, z0, batch, work, status, st);
  if (n <= 3072)
    return lu_solve_2level<16, 1024>(M, n, m, ldm, sM, a0, b0, z0, batch, work, status, st);
  return hipErrorInvalidValue;
}
