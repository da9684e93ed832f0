// Device repair of the ridge systems the band path could not factor (PFML_Search_Coef.py:
// 131-133 solves every (p, lambda) with np.linalg.solve, i.e. LU with partial pivoting; the
// band path uses a banded Cholesky and marks a lambda whose pivot went non-positive - lambda
// = 0 on a rank-deficient Dbar, a tiny lambda on a near-singular one - with a NaN beta).
//
// Two launches with fixed grids, queued between the ridge grid and the utilities on the same
// stream, so nothing waits on the host and the utilities read the repaired betas:
//   ridge_flag_kernel      one thread per (cell, lambda): a NaN beta appends c * L + l to a
//                          device list (vector global atomic on the count)
//   ridge_lu_repair_kernel REPAIR_WG workgroups walk the list; each builds
//                          M = [Dbar_c * scale + lambda I | rbar_c * scale] in its own global
//                          scratch and runs an unblocked right-looking LU with partial
//                          pivoting (LAPACK dgetf2 pivot order), then the two triangular
//                          solves.  A zero pivot (exactly singular, where the reference
//                          raises LinAlgError) leaves the NaN.  Workgroups with no entry exit
//                          at once, so the no-repair case costs two tiny launches.
// The count stays on the device; the host reads it only when it reports counters.
#include "common.h"
#include "ridge_desc.h"

namespace {

constexpr int REPAIR_WG = 64;
constexpr int RT = 256;

__global__ __launch_bounds__(256) void ridge_flag_kernel(const RidgeCellDesc* __restrict__ cells,
                                                         int ncells, int L,
                                                         const double* __restrict__ beta,
                                                         int64_t ldo, int* __restrict__ list,
                                                         int* __restrict__ count, int cap) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ncells * L) return;
  const int c = e / L, l = e % L;
  const RidgeCellDesc cd = cells[c];
  const double* b = beta + cd.out + (int64_t)l * ldo;
  const double x0 = b[0], x1 = b[cd.n - 1];
  if (x0 != x0 || x1 != x1) {
    const int slot = atomicAdd(count, 1);
    if (slot < cap) list[slot] = e;
  }
}

// block-wide argmax of |v| (ties: lowest row) over the 256 threads; every thread gets it
__device__ __forceinline__ int block_argmax(double v, int i, double* sv, int* si) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off, 64);
    const int oi = __shfl_xor(i, off, 64);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
  if (lane == 0) { sv[w] = v; si[w] = i; }
  __syncthreads();
  double bv = sv[0];
  int bi = si[0];
  for (int q = 1; q < RT / 64; ++q)
    if (sv[q] > bv || (sv[q] == bv && si[q] < bi)) { bv = sv[q]; bi = si[q]; }
  __syncthreads();
  return bi;
}

__global__ __launch_bounds__(RT) void ridge_lu_repair_kernel(
    const double* __restrict__ SD, int64_t ldS, const double* __restrict__ Sr,
    const RidgeCellDesc* __restrict__ cells, const double* __restrict__ lvec, int L,
    double* __restrict__ beta, int64_t ldo, const int* __restrict__ list,
    const int* __restrict__ count, int cap, double* __restrict__ scratch, int nmax) {
  __shared__ double sv[RT / 64];
  __shared__ int si[RT / 64];
  __shared__ double piv_s;
  const int total = min(*count, cap);
  const int t = threadIdx.x;
  const int ld = nmax + 1;                               // [A | r] row stride
  double* M = scratch + (int64_t)blockIdx.x * nmax * ld;
  for (int q = blockIdx.x; q < total; q += gridDim.x) {
    const int e = list[q];
    const int c = e / L, l = e % L;
    const RidgeCellDesc cd = cells[c];
    const int n = cd.n;
    const double lam = lvec[l];
    const double* S = SD + cd.src;
    const double* r = Sr + cd.rsrc;
    for (int64_t x = t; x < (int64_t)n * (n + 1); x += RT) {
      const int i = (int)(x / (n + 1)), j = (int)(x % (n + 1));
      double v = (j < n) ? S[(int64_t)i * ldS + j] * cd.scale : r[i] * cd.scale;
      if (j == i) v += lam;
      M[(int64_t)i * ld + j] = v;
    }
    __syncthreads();
    bool singular = false;
    for (int k = 0; k < n; ++k) {
      // pivot: argmax_i>=k |M[i][k]|
      double best = -1.0;
      int bi = k;
      for (int i = k + t; i < n; i += RT) {
        const double a = fabs(M[(int64_t)i * ld + k]);
        if (a > best) { best = a; bi = i; }
      }
      const int p = block_argmax(best, bi, sv, si);
      if (p != k)
        for (int j = t; j <= n; j += RT) {
          const double a = M[(int64_t)k * ld + j];
          M[(int64_t)k * ld + j] = M[(int64_t)p * ld + j];
          M[(int64_t)p * ld + j] = a;
        }
      __syncthreads();
      if (t == 0) piv_s = M[(int64_t)k * ld + k];
      __syncthreads();
      const double piv = piv_s;
      if (piv == 0.0 || piv != piv) { singular = true; break; }
      const double inv = 1.0 / piv;
      // rows below: multiplier in column k, rank-1 update of [A | r] right of k
      for (int i = k + 1 + t; i < n; i += RT) M[(int64_t)i * ld + k] *= inv;
      __syncthreads();
      const int rows = n - k - 1, cols = n - k;          // columns k+1 .. n (incl. rhs)
      for (int64_t x = t; x < (int64_t)rows * cols; x += RT) {
        const int i = k + 1 + (int)(x / cols), j = k + 1 + (int)(x % cols);
        M[(int64_t)i * ld + j] -= M[(int64_t)i * ld + k] * M[(int64_t)k * ld + j];
      }
      __syncthreads();
    }
    double* out = beta + cd.out + (int64_t)l * ldo;
    if (!singular) {
      // back substitution on U x = y (y in column n); unit-lower forward solve was applied
      // to the rhs during elimination
      for (int i = n - 1; i >= 0; --i) {
        double s = 0.0;
        for (int j = i + 1 + t; j < n; j += RT) s += M[(int64_t)i * ld + j] * M[(int64_t)j * ld + n];
        s = block_sum(s, sv);
        if (t == 0) M[(int64_t)i * ld + n] = (M[(int64_t)i * ld + n] - s) / M[(int64_t)i * ld + i];
        __syncthreads();
      }
      for (int j = t; j < n; j += RT) out[j] = M[(int64_t)j * ld + n];
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int pfml_ridge_repair_wg() { return REPAIR_WG; }

// workgroups of one repair launch: never more than the systems it can be handed (cap)
static int repair_wgs(int cap) { return cap < REPAIR_WG ? (cap > 0 ? cap : 1) : REPAIR_WG; }

// scratch doubles of a launch with list capacity `cap`: one nmax x (nmax + 1) system per
// workgroup (64 x 1025 x 1026 doubles = 540 MB at nmax = 1025 only when >= 64 systems can
// fail; a launch of few cells sizes it by its own capacity)
extern "C" int64_t pfml_ridge_repair_work_doubles_cap(int nmax, int cap) {
  return (int64_t)repair_wgs(cap) * nmax * (nmax + 1);
}

extern "C" int64_t pfml_ridge_repair_work_doubles(int nmax) {
  return (int64_t)REPAIR_WG * nmax * (nmax + 1);
}

// list: cap ints, count: 1 int (zeroed by the caller, on the stream), work: see above.
extern "C" hipError_t pfml_ridge_repair(const double* SD, int64_t ldS, const double* Sr,
                                        const void* cells, int ncells, int nmax,
                                        const double* lvec, int L, double* beta, int64_t ldo,
                                        int* list, int* count, int cap, double* work,
                                        hipStream_t st) {
  if (ncells <= 0 || L <= 0) return hipSuccess;
  const RidgeCellDesc* cd = static_cast<const RidgeCellDesc*>(cells);
  const int tot = ncells * L;
  hipLaunchKernelGGL(ridge_flag_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, cd, ncells, L,
                     beta, ldo, list, count, cap);
  hipLaunchKernelGGL(ridge_lu_repair_kernel, dim3(repair_wgs(cap)), dim3(RT), 0, st, SD, ldS, Sr, cd,
                     lvec, L, beta, ldo, list, count, cap, work, nmax);
  return hipGetLastError();
}
