// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of the PFML engine.
//
// Conventions used by every kernel in this directory:
//  * 64-lane wavefronts (hard-coded, never warpSize-32 idioms);
//  * all matrices are row-major with an explicit leading dimension;
//  * every launcher is `extern "C"`, takes a hipStream_t (the caller's torch stream) and
//    returns hipError_t so the Python layer can fail loudly;
//  * fp64 everywhere on the production path (the reference is float64 end to end).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PFML_WAVE 64

typedef double double4_t __attribute__((ext_vector_type(4)));

// v_mfma_f64_16x16x4_f64 fragment maps (cdna_hip_programming.md §3, f64 entry):
//   A operand: lane l holds A[i = l & 15][k = l >> 4]
//   B operand: lane l holds B[k = l >> 4][j = l & 15]
//   C/D      : lane l, reg r holds C[row = (l >> 4) + 4*r][col = l & 15]
// The C/D row map of the f64 instruction differs from the f32/bf16 16x16 forms; it is
// isolated here so that tests/test_gpu_kernels.py::test_mfma_f64_layout pins it on hardware.
#ifndef PFML_F64_CROW
#define PFML_F64_CROW(lane, r) (((lane) >> 4) + 4 * (r))
#endif

__device__ __forceinline__ double4_t mfma_f64_16x16x4(double a, double b, double4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, PFML_WAVE);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, PFML_WAVE));
  return v;
}

// Block-wide sum of one double per thread; `scratch` must hold blockDim.x/64 doubles.
// Returns the total to every thread.
__device__ __forceinline__ double block_sum(double v, double* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < nw; ++w) t += scratch[w];
  return t;
}

// XCD-aware bijective remap of a 1-D block id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD (same L2).  Speed only.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

#define PFML_LAUNCH_CHECK() return hipGetLastError()
