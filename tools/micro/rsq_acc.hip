// Accuracy of v_rsq_f64 / v_rcp_f64 seeds and of 1..3 Newton refinements, measured against
// the IEEE 1/sqrt(x) and 1/x (max error in ulps over random x spanning 1e-30 .. 1e30).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include <random>

__global__ void k_rsq(const double* x, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  double y = __builtin_amdgcn_rsq(v);
  const double h = 0.5 * v;
  out[8 * i + 0] = y;
  for (int it = 1; it <= 3; ++it) { y = y * fma(-h * y, y, 1.5); out[8 * i + it] = y; }
  double r = __builtin_amdgcn_rcp(v);
  out[8 * i + 4] = r;
  for (int it = 1; it <= 3; ++it) { r = fma(r, fma(-v, r, 1.0), r); out[8 * i + 4 + it] = r; }
}

int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), o(8 * (size_t)n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> e(-30.0, 30.0), m(1.0, 10.0);
  for (int i = 0; i < n; ++i) x[i] = m(g) * std::pow(10.0, e(g));
  double *dx, *dout;
  if (hipMalloc(&dx, n * 8) != hipSuccess || hipMalloc(&dout, 8 * (size_t)n * 8) != hipSuccess) return 1;
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_rsq, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
  hipMemcpy(o.data(), dout, 8 * (size_t)n * 8, hipMemcpyDeviceToHost);
  double worst[8] = {0};
  for (int i = 0; i < n; ++i) {
    const double rs = 1.0 / std::sqrt(x[i]), rc = 1.0 / x[i];
    for (int k = 0; k < 8; ++k) {
      const double ref = k < 4 ? rs : rc;
      const double ulp = std::nextafter(std::fabs(ref), INFINITY) - std::fabs(ref);
      const double err = std::fabs(o[8 * (size_t)i + k] - ref) / ulp;
      if (err > worst[k]) worst[k] = err;
    }
  }
  printf("{\"rsq_seed_ulp\": %.3g, \"rsq_newton1\": %.3g, \"rsq_newton2\": %.3g, \"rsq_newton3\": %.3g, "
         "\"rcp_seed_ulp\": %.3g, \"rcp_newton1\": %.3g, \"rcp_newton2\": %.3g, \"rcp_newton3\": %.3g}\n",
         worst[0], worst[1], worst[2], worst[3], worst[4], worst[5], worst[6], worst[7]);
  hipFree(dx); hipFree(dout);
  return 0;
}
