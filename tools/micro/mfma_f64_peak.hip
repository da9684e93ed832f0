// Micro-benchmark: sustained v_mfma_f64_16x16x4 rate on gfx950, the roofline anchor of the
// fp64 kernels.  Round 1's version fed every MFMA the same two loop-invariant registers and
// measured 45.8 TF/s - below the 54-61 TF/s the GEMMs reach - so it under-reported the pipe.
// Here every lane's A/B operands are distinct random-ish values that change each iteration
// (a, b advanced by one VALU add per 8 MFMAs, which co-issues beside the matrix pipe), the
// accumulator count and the waves per SIMD are swept, and the in-kernel clock
// (s_memtime / s_memrealtime) is reported so the rate can be read as flops per cycle per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double double4_t __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, long long* clk, int iters) {
  double4_t acc[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) acc[q] = double4_t{0.25, -0.5, 0.125, 1.0};
  double a = 1.0 + (threadIdx.x * 2654435761u % 1000) * 1e-4;
  double b = -1.0 + (blockIdx.x * 40503u % 977) * 1e-4;
  const double da = 1e-9, db = -1e-9;
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  const long long r0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
    a += da;
    b += db;
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  const long long r1 = (long long)__builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
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
  long long* clk;
  const int maxblocks = 256 * 8;
  hipMalloc(&d, sizeof(double) * maxblocks * 256);
  hipMalloc(&clk, sizeof(long long) * maxblocks * 2);
  long long* hclk = new long long[maxblocks * 2];
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms;
  const int iters = 4000;
  printf("{");
  bool first = true;
  double best = 0.0;
  auto run = [&](auto kern, int nacc, int wps, const char* name) {
    const int blocks = 256 * wps;   // 256-thread blocks: wps waves per SIMD
    for (int rep = 0; rep < 3; ++rep) kern<<<blocks, 256>>>(d, clk, iters / 4);   // warm the clock
    hipEventRecord(e0);
    kern<<<blocks, 256>>>(d, clk, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(hclk, clk, sizeof(long long) * blocks * 2, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int b = 0; b < blocks; ++b) { cyc += hclk[2 * b]; rt += hclk[2 * b + 1]; }
    const double ghz = cyc / (rt / 100e6) / 1e9;   // s_memrealtime ticks at 100 MHz
    const double flops = 2.0 * 16 * 16 * 4 * nacc * (double)iters * (blocks * 4.0);
    const double tf = flops / (ms * 1e-3) / 1e12;
    // MFMAs per SIMD per cycle from the in-kernel clock: waves/SIMD * nacc * iters / cycles
    const double cyc_per_mfma = (cyc / blocks) / ((double)nacc * iters * wps);
    if (tf > best) best = tf;
    printf("%s\"%s_w%d\": {\"tflops\": %.2f, \"ghz\": %.3f, \"simd_cycles_per_mfma\": %.2f}",
           first ? "" : ", ", name, wps, tf, ghz, cyc_per_mfma);
    first = false;
  };
  for (int wps : {1, 2, 4}) {
    run(mfma_loop<4>, 4, wps, "mfma_acc4");
    run(mfma_loop<8>, 8, wps, "mfma_acc8");
    run(mfma_loop<16>, 16, wps, "mfma_acc16");
  }
  const int blocks = maxblocks;
  fma_loop<<<blocks, 256>>>(d, 10);
  hipEventRecord(e0);
  fma_loop<<<blocks, 256>>>(d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 64 * iters * (double)blocks * 256;
  printf(", \"valu_fma_f64_tflops\": %.2f, \"mfma_best_tflops\": %.2f}\n",
         flops / (ms * 1e-3) / 1e12, best);
  hipFree(d);
  hipFree(clk);
  delete[] hclk;
  return 0;
}
