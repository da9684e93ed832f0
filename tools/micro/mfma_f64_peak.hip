// Micro-benchmark: sustained v_mfma_f64_16x16x4 rate on gfx950, the roofline anchor of the
// fp64 kernels.
//
// Round 1 fed every MFMA two loop-invariant registers and timed the launch with events
// (45.8 TF/s); round 2 varied the operands but still divided the flops by the EVENT time,
// which counts blocks that wait for a free slot (47 TF/s, below the 54-61 TF/s the GEMMs
// reach).  Here the rate is taken per SIMD from the hardware itself: every wave records its
// HW_ID (XCC, SE, SH, CU, SIMD) and s_memtime stamps around its MFMA loop; the host groups
// the waves by SIMD and divides each SIMD's span (first start to last end) by the MFMAs its
// waves issued.  cycles / MFMA per SIMD x 1024 SIMDs x the measured shader clock is the chip
// rate a kernel can reach when every SIMD is fed - the number a % of peak is quoted against.
// The event-timed rate is reported beside it.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>
typedef double double4_t __attribute__((ext_vector_type(4)));

struct WaveRec {
  unsigned hwid, xcc;
  long long t0, t1, r0, r1;
};

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, WaveRec* rec, int iters) {
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
  if ((threadIdx.x & 63) == 0) {
    WaveRec w;
    w.hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
    w.xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);     // HW_REG_XCC_ID
    w.t0 = t0;
    w.t1 = t1;
    w.r0 = r0;
    w.r1 = r1;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = w;   // vector store
  }
}

// the same loop with the accumulators pinned to AGPRs (inline asm, "a" constraint): the
// library DGEMMs keep their C tiles in the accumulation registers
template <int NACC>
__global__ __launch_bounds__(256) void mfma_agpr_loop(double* out, WaveRec* rec, int iters) {
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
    for (int q = 0; q < NACC; ++q)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(acc[q]) : "v"(a), "v"(b));
    a += da;
    b += db;
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  const long long r1 = (long long)__builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    WaveRec w;
    w.hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    w.xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    w.t0 = t0;
    w.t1 = t1;
    w.r0 = r0;
    w.r1 = r1;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = w;
  }
}

// distinct, loop-invariant A / B registers per accumulator (a GEMM's operands differ per MFMA;
// no VALU write of an operand between MFMAs)
template <int NACC>
__global__ __launch_bounds__(256) void mfma_ops_loop(double* out, WaveRec* rec, int iters) {
  double4_t acc[NACC];
  double av[NACC], bv[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) {
    acc[q] = double4_t{0.25, -0.5, 0.125, 1.0};
    av[q] = 1.0 + ((threadIdx.x + 7 * q) * 2654435761u % 1000) * 1e-4;
    bv[q] = -1.0 + ((blockIdx.x + 3 * q) * 40503u % 977) * 1e-4;
  }
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  const long long r0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], bv[q], acc[q], 0, 0, 0);
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  const long long r1 = (long long)__builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    WaveRec w;
    w.hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    w.xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    w.t0 = t0;
    w.t1 = t1;
    w.r0 = r0;
    w.r1 = r1;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = w;
  }
}

// VGPR-form MFMA through inline asm ("+v": the accumulators stay in VGPRs for the whole
// loop).  The builtin variants above were compiled to the AGPR form with every accumulator
// copied VGPR -> AGPR before and AGPR -> VGPR after each MFMA group (8 v_accvgpr moves per
// MFMA, llvm-objdump of this file): they measured those moves (~104 cycles / MFMA), not the
// MFMA pipe.  This loop has no other instruction between the MFMAs.
template <int NACC>
__global__ __launch_bounds__(256) void mfma_vgpr_loop(double* out, WaveRec* rec, int iters) {
  double4_t acc[NACC];
  double av[NACC], bv[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) {
    acc[q] = double4_t{0.25, -0.5, 0.125, 1.0};
    av[q] = 1.0 + ((threadIdx.x + 7 * q) * 2654435761u % 1000) * 1e-4;
    bv[q] = -1.0 + ((blockIdx.x + 3 * q) * 40503u % 977) * 1e-4;
  }
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  const long long r0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NACC; ++q)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[q]) : "v"(av[q]), "v"(bv[q]));
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  const long long r1 = (long long)__builtin_amdgcn_s_memrealtime();
  asm volatile("s_nop 15" ::: "memory");
  double s = 0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    WaveRec w;
    w.hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    w.xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    w.t0 = t0;
    w.t1 = t1;
    w.r0 = r0;
    w.r1 = r1;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = w;
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
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int nsimd = 4 * ncu;
  const int maxblocks = ncu * 8;
  double* d;
  WaveRec* rec;
  hipMalloc(&d, sizeof(double) * maxblocks * 256);
  hipMalloc(&rec, sizeof(WaveRec) * maxblocks * 4);
  std::vector<WaveRec> h(maxblocks * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  printf("{\"cus\": %d", ncu);
  double best_simd = 0.0, best_event = 0.0, best_ghz = 0.0;
  int ncu_run = ncu;               // CUs the grid is sized for (partial-chip runs: fewer)
  auto run = [&](auto kern, int nacc, int wps, const char* name) {
    const int blocks = ncu_run * wps;   // 256-thread blocks: wps waves per SIMD when spread evenly
    for (int rep = 0; rep < 3; ++rep) kern<<<blocks, 256>>>(d, rec, iters / 4);   // warm clocks
    hipEventRecord(e0);
    kern<<<blocks, 256>>>(d, rec, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const int nw = blocks * 4;
    hipMemcpy(h.data(), rec, sizeof(WaveRec) * nw, hipMemcpyDeviceToHost);
    // per SIMD: MFMAs issued by its waves / (last end - first start)
    struct Span { long long t0 = (1LL << 62), t1 = 0, r0 = (1LL << 62), r1 = 0; int waves = 0; };
    std::map<unsigned long long, Span> simd;
    for (int w = 0; w < nw; ++w) {
      const unsigned hw = h[w].hwid;
      const unsigned long long key = ((unsigned long long)(h[w].xcc & 0xf) << 32) |
                                     (hw & 0x0000FF30u);   // SE/SH/CU/SIMD fields, no wave slot
      Span& s = simd[key];
      s.t0 = std::min(s.t0, h[w].t0);
      s.t1 = std::max(s.t1, h[w].t1);
      s.r0 = std::min(s.r0, h[w].r0);
      s.r1 = std::max(s.r1, h[w].r1);
      s.waves++;
    }
    std::vector<double> cpm;   // cycles per MFMA per SIMD
    double cyc = 0.0, rt = 0.0;
    int maxw = 0;
    for (auto& kv : simd) {
      const double mf = (double)kv.second.waves * nacc * (double)iters;
      cpm.push_back((double)(kv.second.t1 - kv.second.t0) / mf);
      cyc += (double)(kv.second.t1 - kv.second.t0);
      rt += (double)(kv.second.r1 - kv.second.r0);
      maxw = std::max(maxw, kv.second.waves);
    }
    std::sort(cpm.begin(), cpm.end());
    const double med = cpm[cpm.size() / 2];
    const double ghz = cyc / (rt / 100e6) / 1e9;            // s_memrealtime ticks at 100 MHz
    const double simd_tf = 2.0 * 16 * 16 * 4 / med * nsimd * ghz * 1e9 / 1e12;   // whole chip
    const double flops = 2.0 * 16 * 16 * 4 * nacc * (double)iters * (blocks * 4.0);
    const double ev_tf = flops / (ms * 1e-3) / 1e12;
    if (simd_tf > best_simd) { best_simd = simd_tf; best_ghz = ghz; }
    best_event = std::max(best_event, ev_tf);
    printf(", \"%s_w%d\": {\"simds_seen\": %zu, \"max_waves_per_simd\": %d, "
           "\"cycles_per_mfma_median\": %.2f, \"cycles_per_mfma_min\": %.2f, \"ghz\": %.3f, "
           "\"per_simd_tflops\": %.2f, \"event_tflops\": %.2f}",
           name, wps, simd.size(), maxw, med, cpm.front(), ghz, simd_tf, ev_tf);
  };
  for (int wps : {1, 2, 4}) {
    run(mfma_vgpr_loop<4>, 4, wps, "mfma_vgpr_acc4");
    run(mfma_vgpr_loop<8>, 8, wps, "mfma_vgpr_acc8");
    run(mfma_vgpr_loop<16>, 16, wps, "mfma_vgpr_acc16");
  }
  // the builtin forms (AGPR shuffles around every MFMA group, see mfma_vgpr_loop): kept as the
  // record of what rounds 1-2 measured
  run(mfma_loop<8>, 8, 4, "builtin_acc8");
  run(mfma_ops_loop<8>, 8, 4, "builtin_ops_acc8");
  // partial chip (1/8 and 1/2 of the CUs busy): is the full-chip rate a pipe limit or a
  // chip-level power / current limit?
  for (int frac : {8, 2}) {
    ncu_run = ncu / frac;
    char nm[64];
    snprintf(nm, sizeof(nm), "part%d_vgpr_acc8", frac);
    run(mfma_vgpr_loop<8>, 8, 4, nm);
  }
  ncu_run = ncu;
  const int blocks = maxblocks;
  fma_loop<<<blocks, 256>>>(d, 10);
  hipEventRecord(e0);
  fma_loop<<<blocks, 256>>>(d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 64 * iters * (double)blocks * 256;
  printf(", \"valu_fma_f64_tflops\": %.2f, \"mfma_peak_tflops\": %.2f, \"mfma_peak_ghz\": %.3f, "
         "\"mfma_event_best_tflops\": %.2f}\n",
         flops / (ms * 1e-3) / 1e12, best_simd, best_ghz, best_event);
  hipFree(d);
  hipFree(rec);
  return 0;
}
