// Segmented sums over the month axis.
//
// The reference keeps running sums of r_tilde and denom, adding each hyper-parameter year's
// 12 new months (PFML_Search_Coef.py:68-121).  The engine instead sums each window segment
// (burn-in block, then one block per hp year) in one bandwidth-bound pass over the resident
// [T, E] stack and prefix-sums the per-segment totals (53 x E, negligible).  For the 513 x 513
// denom stack this reads 2.1 MB per month exactly once; rows of even length that are 16-byte
// aligned take the double2 (16 B per lane) path.
#include "common.h"

namespace {

template <int VEC>
__global__ __launch_bounds__(256) void segsum_kernel(const double* __restrict__ X, int64_t E,
                                                     const int* __restrict__ seg_start,
                                                     const int* __restrict__ seg_stop,
                                                     double* __restrict__ out) {
  const int s = blockIdx.y;
  const int64_t e0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * VEC;
  if (e0 >= E) return;
  const int a = seg_start[s], b = seg_stop[s];
  if (VEC == 2) {
    double2 acc = {0.0, 0.0};
    for (int tm = a; tm < b; ++tm) {
      const double2 x = *reinterpret_cast<const double2*>(X + (int64_t)tm * E + e0);
      acc.x += x.x;
      acc.y += x.y;
    }
    *reinterpret_cast<double2*>(out + (int64_t)s * E + e0) = acc;
  } else {
    double acc = 0.0;
    for (int tm = a; tm < b; ++tm) acc += X[(int64_t)tm * E + e0];
    out[(int64_t)s * E + e0] = acc;
  }
}

}  // namespace

// X: [T, E] row-major, out: [S, E]; segment s sums rows [seg_start[s], seg_stop[s]).
extern "C" hipError_t pfml_segsum(const double* X, int64_t E, const int* seg_start,
                                  const int* seg_stop, int nseg, double* out, hipStream_t st) {
  if (nseg <= 0 || E <= 0) return hipSuccess;
  const bool vec = (E % 2 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  if (vec) {
    dim3 grid((unsigned)((E / 2 + 255) / 256), nseg);
    hipLaunchKernelGGL(segsum_kernel<2>, grid, dim3(256), 0, st, X, E, seg_start, seg_stop, out);
  } else {
    dim3 grid((unsigned)((E + 255) / 256), nseg);
    hipLaunchKernelGGL(segsum_kernel<1>, grid, dim3(256), 0, st, X, E, seg_start, seg_stop, out);
  }
  return hipGetLastError();
}
