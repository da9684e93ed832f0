// LDS bank-conflict counter check (profiles/r05_lds_conflict_counter.txt): three kernels with
// KNOWN LDS access patterns, run under rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT, to
// tell whether the counter's ratio on the DGEMM kernels (r04_dgemm_pmc.txt: conflicts ~2.7x
// the LDS instructions) measures real conflicts or counts something else on gfx950.
//   lds_linear_b64  lane l reads double l (+ a per-iteration offset): 64 consecutive doubles,
//                   the textbook conflict-free ds_read_b64
//   lds_linear_b32  lane l reads float l: conflict-free ds_read_b32
//   lds_stride_b64  lane l reads double 64 l: every lane in the same bank pair (64-way)
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/lds_conflict.hip -o tools/micro/lds_conflict
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NT = 256, ITERS = 4096;

__global__ __launch_bounds__(NT) void lds_linear_b64(double* out) {
  __shared__ double s[64 * 65];
  for (int e = threadIdx.x; e < 64 * 65; e += NT) s[e] = e;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
  for (int it = 0; it < ITERS; ++it) acc += s[lane + ((it * 64) & 4095)];
  out[blockIdx.x * NT + threadIdx.x] = acc;
}

__global__ __launch_bounds__(NT) void lds_linear_b32(float* out) {
  __shared__ float s[64 * 65];
  for (int e = threadIdx.x; e < 64 * 65; e += NT) s[e] = e;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  float acc = 0.f;
  for (int it = 0; it < ITERS; ++it) acc += s[lane + ((it * 64) & 4095)];
  out[blockIdx.x * NT + threadIdx.x] = acc;
}

__global__ __launch_bounds__(NT) void lds_stride_b64(double* out) {
  __shared__ double s[64 * 65];
  for (int e = threadIdx.x; e < 64 * 65; e += NT) s[e] = e;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
  for (int it = 0; it < ITERS; ++it) acc += s[64 * lane + (it & 63)];
  out[blockIdx.x * NT + threadIdx.x] = acc;
}

int main() {
  const int blocks = 1024;
  double* d;
  if (hipMalloc(&d, sizeof(double) * blocks * NT) != hipSuccess) return 1;
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(lds_linear_b64, dim3(blocks), dim3(NT), 0, 0, d);
    hipLaunchKernelGGL(lds_linear_b32, dim3(blocks), dim3(NT), 0, 0, (float*)d);
    hipLaunchKernelGGL(lds_stride_b64, dim3(blocks), dim3(NT), 0, 0, d);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  double h = 0.0;
  (void)hipMemcpy(&h, d, sizeof(double), hipMemcpyDeviceToHost);
  printf("ok %g\n", h);
  (void)hipFree(d);
  return 0;
}
