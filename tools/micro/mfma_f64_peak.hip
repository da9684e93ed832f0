// Micro-benchmark: sustained v_mfma_f64_16x16x4 rate (independent accumulators, all CUs),
// plus fp64 VALU FMA rate, to calibrate the fp64 kernels' roofline on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double double4_t __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters) {
  double4_t acc[NACC];
  for (int q = 0; q < NACC; ++q) acc[q] = double4_t{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
  }
  double s = 0;
  for (int q = 0; q < NACC; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_loop(double* out, int iters) {
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  const double m = 0.999999, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x0 = fma(x0, m, c); x1 = fma(x1, m, c); x2 = fma(x2, m, c); x3 = fma(x3, m, c);
      x4 = fma(x4, m, c); x5 = fma(x5, m, c); x6 = fma(x6, m, c); x7 = fma(x7, m, c);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

int main() {
  double* d;
  const int blocks = 256 * 8;
  hipMalloc(&d, sizeof(double) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms;
  const int iters = 2000;
  printf("{");
  auto run = [&](auto kern, int nacc, const char* name) {
    kern<<<blocks, 256>>>(d, 10);
    hipEventRecord(e0);
    kern<<<blocks, 256>>>(d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double flops = 2.0 * 16 * 16 * 4 * nacc * (double)iters * (blocks * 4.0);
    printf("\"%s\": %.2f, ", name, flops / (ms * 1e-3) / 1e12);
  };
  run(mfma_loop<1>, 1, "mfma_acc1_tflops");
  run(mfma_loop<4>, 4, "mfma_acc4_tflops");
  run(mfma_loop<8>, 8, "mfma_acc8_tflops");
  run(mfma_loop<16>, 16, "mfma_acc16_tflops");
  double flops;
  fma_loop<<<blocks, 256>>>(d, 10);
  hipEventRecord(e0);
  fma_loop<<<blocks, 256>>>(d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  flops = 2.0 * 64 * iters * (double)blocks * 256;
  printf("\"valu_fma_f64_tflops\": %.2f}\n", flops / (ms * 1e-3) / 1e12);
  hipFree(d);
  return 0;
}
