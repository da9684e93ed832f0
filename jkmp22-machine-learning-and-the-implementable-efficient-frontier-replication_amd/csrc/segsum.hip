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

// ---------------------------------------------------------------------------------------
// Expanding-window sums of symmetric month matrices (K14, fused prefix):
//   out[g, s] = sum over segments s' <= s of sum_{t in [start_s', stop_s')} X[g, t]
// X: [G, T, P, P] (each X[g, t] symmetric), out: [G, S, P, P] (full, symmetric).
// Pass 1 sums every (row, segment) over the UPPER triangle only (half the bytes of a dense
// pass, one workgroup per (row, segment, g) for full-chip parallelism) into out; pass 2 runs
// the prefix over segments in place and mirrors (i, j) to (j, i).  The dense segment sums +
// torch cumsum it replaces read 2x and wrote 3x as much.
namespace {

// Segment s's sums live in out[g][s - skip] for s >= skip and in scratch[g][s] for the
// leading `skip` segments (e.g. the burn-in block, needed only as a prefix): the output is
// the contiguous [G][nseg - skip] stack the ridge grid consumes, with no slicing copy.
__device__ __forceinline__ double* seg_slot(double* out, double* scratch, int g, int s, int nseg,
                                            int skip, int64_t PP) {
  return s < skip ? scratch + ((int64_t)g * skip + s) * PP
                  : out + ((int64_t)g * (nseg - skip) + (s - skip)) * PP;
}

__global__ __launch_bounds__(256) void wsum_upper_kernel(const double* __restrict__ X, int P,
                                                         int T, const int* __restrict__ seg_start,
                                                         const int* __restrict__ seg_stop,
                                                         int nseg, int skip,
                                                         double* __restrict__ out,
                                                         double* __restrict__ scratch) {
  const int i = blockIdx.x, s = blockIdx.y, g = blockIdx.z;
  const int a = seg_start[s], b = seg_stop[s];
  const int64_t PP = (int64_t)P * P;
  const double* src = X + (int64_t)g * T * PP + (int64_t)i * P;
  double* dst = seg_slot(out, scratch, g, s, nseg, skip, PP) + (int64_t)i * P;
  for (int j = i + threadIdx.x; j < P; j += 256) {
    // four independent chains: four month loads in flight per lane
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    int tm = a;
    for (; tm + 4 <= b; tm += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += src[(int64_t)(tm + u) * PP + j];
    }
    for (; tm < b; ++tm) acc[0] += src[(int64_t)tm * PP + j];
    dst[j] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
}

// pass 2 on 32 x 32 tiles (I <= J) of the upper triangle: running sum over segments in
// registers, tile (I, J) and its transpose (J, I) both written row-contiguous via LDS.  The
// next segment's tile is loaded while the current one is written (loads clamped into the
// matrix, masked on use).
__global__ __launch_bounds__(256) void wsum_prefix_mirror_kernel(int P, int nseg, int skip,
                                                                 double* __restrict__ out,
                                                                 double* __restrict__ scratch) {
  __shared__ double Ts[32][33];
  const int g = blockIdx.y;
  int tile = blockIdx.x;
  const int nt = (P + 31) / 32;
  int I = 0;                                    // upper tiles enumerated row by row
  while (tile >= nt - I) { tile -= nt - I; ++I; }
  const int J = I + tile;
  const int64_t PP = (int64_t)P * P;
  const int t = threadIdx.x, c = t & 31, r0 = t >> 5;
  double acc[4] = {0.0, 0.0, 0.0, 0.0}, nx[4];
  auto fetch = [&](int s) {
    const double* o = seg_slot(out, scratch, g, s, nseg, skip, PP);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = min(I * 32 + r0 + 8 * q, P - 1), j = min(J * 32 + c, P - 1);
      nx[q] = o[(int64_t)i * P + j];
    }
  };
  fetch(0);
  for (int s = 0; s < nseg; ++s) {
    double cur[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = nx[q];
    if (s + 1 < nseg) fetch(s + 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + 8 * q, i = I * 32 + r, j = J * 32 + c;
      const bool valid = i < P && j < P && (I != J || c >= r);
      acc[q] += valid ? cur[q] : 0.0;
      Ts[r][c] = acc[q];
    }
    __syncthreads();
    if (s >= skip) {
      double* o = seg_slot(out, scratch, g, s, nseg, skip, PP);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = r0 + 8 * q;
        const int i = I * 32 + r, j = J * 32 + c;
        if (i < P && j < P) o[(int64_t)i * P + j] = (I != J || c >= r) ? Ts[r][c] : Ts[c][r];
        const int i2 = J * 32 + r, j2 = I * 32 + c;     // transposed tile
        if (I != J && i2 < P && j2 < P) o[(int64_t)i2 * P + j2] = Ts[c][r];
      }
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" hipError_t pfml_window_prefix_sym(const double* X, int P, int T, int G,
                                             const int* seg_start, const int* seg_stop, int nseg,
                                             int skip, double* out, double* scratch,
                                             hipStream_t st) {
  if (nseg <= 0 || P <= 0 || G <= 0) return hipSuccess;
  if (skip < 0 || skip > nseg || (skip > 0 && scratch == nullptr)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wsum_upper_kernel, dim3(P, nseg, G), dim3(256), 0, st, X, P, T, seg_start,
                     seg_stop, nseg, skip, out, scratch);
  const int nt = (P + 31) / 32;
  hipLaunchKernelGGL(wsum_prefix_mirror_kernel, dim3(nt * (nt + 1) / 2, G), dim3(256), 0, st, P,
                     nseg, skip, out, scratch);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Expanding-window sums of the month VECTORS (r_tilde) in one launch:
//   out[g, s - skip, c] = sum over segments s' <= s of sum_{t in [start_s', stop_s')} X[g, t, c]
// X: [G, T, E], out: [G, nseg - skip, E].  Workgroup (64 columns, g): its 16 row groups sum
// the segments (eight months in flight per lane) into LDS, then one row group runs the
// prefix over the segments in segment order.  Replaces segment sums + a transposing copy,
// a scan and two copies (~55 us of small launches ahead of the ridge grid).
namespace {
constexpr int WV_COLS = 64, WV_SEG = 128, WV_T = 1024, WV_RG = WV_T / WV_COLS;
__global__ __launch_bounds__(WV_T) void window_prefix_vec_kernel(
    const double* __restrict__ X, int64_t E, int T, const int* __restrict__ seg_start,
    const int* __restrict__ seg_stop, int nseg, int skip, double* __restrict__ out) {
  __shared__ double part[WV_SEG][WV_COLS];
  const int lc = threadIdx.x % WV_COLS, ry = threadIdx.x / WV_COLS;
  const int g = blockIdx.y, c = blockIdx.x * WV_COLS + lc;
  const bool cv = c < E;
  const double* src = X + (int64_t)g * T * E + (cv ? c : 0);
  for (int s = ry; s < nseg; s += WV_RG) {
    const int a = seg_start[s], b = seg_stop[s];
    double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int tm = a; tm < b; tm += 8) {          // eight months in flight
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = (tm + u < b) ? src[(int64_t)(tm + u) * E] : 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += x[u];
    }
    part[s][lc] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
  __syncthreads();
  if (ry == 0 && cv) {
    double run = 0.0;
    double* o = out + (int64_t)g * (nseg - skip) * E + c;
    for (int s = 0; s < nseg; ++s) {
      run += part[s][lc];
      if (s >= skip) o[(int64_t)(s - skip) * E] = run;
    }
  }
}
}  // namespace

extern "C" int pfml_window_prefix_vec_max_segments() { return WV_SEG; }

extern "C" hipError_t pfml_window_prefix_vec(const double* X, int64_t E, int T, int G,
                                             const int* seg_start, const int* seg_stop, int nseg,
                                             int skip, double* out, hipStream_t st) {
  if (nseg <= 0 || E <= 0 || G <= 0 || nseg - skip <= 0) return hipSuccess;
  if (nseg > WV_SEG || skip < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(window_prefix_vec_kernel, dim3((unsigned)((E + WV_COLS - 1) / WV_COLS), G),
                     dim3(WV_T), 0, st, X, E, T, seg_start, seg_stop, nseg, skip, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Canonical chunked expanding-window sums (bitwise the same on every world size).
//
// A running sum over the segments of ONE rank re-associates differently for every sharding
// (world 1: ((S0 + S1) + S2) + ..., world N: (S_k + ...) + prefix of the lower ranks), so
// the utilities of an N-rank run differed from the 1-rank run in the last bits (2e-10 rel.)
// and a near-tie rank could flip.  The sums therefore follow ONE fixed association,
// independent of the world size:
//   * the months are cut into 2C canonical chunks: C burn-in pieces and C groups of whole
//     hp-year blocks (search.win_layout; C = 8 covers world 1, 2, 4, 8);
//   * chunk total T = left fold of its segment sums from 0 (kernel A, on the chunk's owner);
//   * E = left fold of the C burn-in totals, P_0 = E, P_{c+1} = P_c + TY_c;
//   * the window of a year in chunk c = left fold of c's year segments starting from P_c
//     (kernel B).
// Ranks own whole chunks; the totals cross ranks by one all-gather (P x P per owned chunk)
// and kernel B reads them through a canonical slot map, so no reordering copy.  Totals are
// chunk-major: slot k, g at tot + k * tstride + g * (P P or E).
namespace {

__device__ __forceinline__ bool tile_upper(int I, int J, int i, int j, int r, int c, int P) {
  return i < P && j < P && (I != J || c >= r);
}

// tot slot[lc] (upper triangle) = left fold of segments [cs[lc], ce[lc]) from 0; one
// workgroup per (tile, g, chunk): the chunks are independent, so the launch has nlc times
// the workgroups of a per-tile loop over them (that form was latency-bound: 306 workgroups
// walking 61 segment tiles one after another, 127 us for 128 MB).  Same per-element order.
__global__ __launch_bounds__(256) void wsum_chunk_totals_kernel(
    int P, int nseg, int skip, const double* __restrict__ out, const double* __restrict__ scratch,
    int nlc, const int* __restrict__ cs, const int* __restrict__ ce, const int* __restrict__ slot,
    double* __restrict__ tot, int64_t tstride) {
  const int g = blockIdx.y, lc = blockIdx.z;
  int tile = blockIdx.x;
  const int nt = (P + 31) / 32;
  int I = 0;
  while (tile >= nt - I) { tile -= nt - I; ++I; }
  const int J = I + tile;
  const int64_t PP = (int64_t)P * P;
  const int t = threadIdx.x, c = t & 31, r0 = t >> 5;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const int s0 = cs[lc], s1 = ce[lc];
  // all of a segment's loads in flight before the adds; the next segment's issued first
  double nx[4];
  auto fetch = [&](int s) {
    const double* o = seg_slot(const_cast<double*>(out), const_cast<double*>(scratch), g, s,
                               nseg, skip, PP);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = min(I * 32 + r0 + 8 * q, P - 1), j = min(J * 32 + c, P - 1);
      nx[q] = o[(int64_t)i * P + j];
    }
  };
  if (s0 < s1) fetch(s0);
  for (int s = s0; s < s1; ++s) {
    double cur[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = nx[q];
    if (s + 1 < s1) fetch(s + 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + 8 * q, i = I * 32 + r, j = J * 32 + c;
      if (tile_upper(I, J, i, j, r, c, P)) acc[q] += cur[q];
    }
  }
  double* d = tot + (int64_t)slot[lc] * tstride + (int64_t)g * PP;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + 8 * q, i = I * 32 + r, j = J * 32 + c;
    if (tile_upper(I, J, i, j, r, c, P)) d[(int64_t)i * P + j] = acc[q];
  }
}

// windows: E = fold(tot[sb[k]]), P_0 = E; chunk c with local year segments [ys[c], ye[c]):
// acc = P_c, acc += seg s, out[s - skip] = acc (full, mirrored); P_{c+1} = P_c + tot[sy[c]].
// One workgroup per (tile, g, chunk ch <= clast): it forms P_ch itself by the same left fold
// (E, then + tot[sy[0]], ..., + tot[sy[ch - 1]]), so every chunk's windows run in parallel
// and the bits are those of the sequential walk.
__global__ __launch_bounds__(256) void wsum_chunk_prefix_kernel(
    int P, int nseg, int skip, double* __restrict__ out, double* __restrict__ scratch, int C,
    const int* __restrict__ sb, const int* __restrict__ sy, const int* __restrict__ ys,
    const int* __restrict__ ye, const double* __restrict__ tot, int64_t tstride, int clast) {
  __shared__ double Ts[32][33];
  const int g = blockIdx.y, ch = blockIdx.z;
  const int s0 = ys[ch], s1 = ye[ch];
  if (s0 >= s1) return;                         // no local windows in this chunk
  int tile = blockIdx.x;
  const int nt = (P + 31) / 32;
  int I = 0;
  while (tile >= nt - I) { tile -= nt - I; ++I; }
  const int J = I + tile;
  const int64_t PP = (int64_t)P * P;
  const int t = threadIdx.x, c = t & 31, r0 = t >> 5;
  const double* tg = tot + (int64_t)g * PP;     // slot k at tg + k * tstride
  // the first segment's tile is in flight during the prefix, each next one while the current
  // is added and written (clamped loads, masked on use; the same adds in the same order)
  double nx[4];
  auto fetch = [&](int s) {
    const double* o = seg_slot(out, scratch, g, s, nseg, skip, PP);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = min(I * 32 + r0 + 8 * q, P - 1), j = min(J * 32 + c, P - 1);
      nx[q] = o[(int64_t)i * P + j];
    }
  };
  fetch(s0);
  // the C + ch prefix tiles, loaded together, then added in the canonical order
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const int nk = C + ch;
  for (int k0 = 0; k0 < nk; k0 += 8) {
    double v[8][4];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = min(k0 + u, nk - 1);
      const double* o = tg + (int64_t)(k < C ? sb[k] : sy[k - C]) * tstride;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = min(I * 32 + r0 + 8 * q, P - 1), j = min(J * 32 + c, P - 1);
        v[u][q] = o[(int64_t)i * P + j];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (k0 + u < nk) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = r0 + 8 * q, i = I * 32 + r, j = J * 32 + c;
          if (tile_upper(I, J, i, j, r, c, P)) acc[q] += v[u][q];
        }
      }
    }
  }
  for (int s = s0; s < s1; ++s) {
    double cur[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = nx[q];
    if (s + 1 < s1) fetch(s + 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + 8 * q, i = I * 32 + r, j = J * 32 + c;
      const double v = tile_upper(I, J, i, j, r, c, P) ? cur[q] : 0.0;
      acc[q] += v;
      Ts[r][c] = acc[q];
    }
    __syncthreads();
    if (s >= skip) {
      double* w = seg_slot(out, scratch, g, s, nseg, skip, PP);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = r0 + 8 * q;
        const int i = I * 32 + r, j = J * 32 + c;
        if (i < P && j < P) w[(int64_t)i * P + j] = (I != J || c >= r) ? Ts[r][c] : Ts[c][r];
        const int i2 = J * 32 + r, j2 = I * 32 + c;
        if (I != J && i2 < P && j2 < P) w[(int64_t)i2 * P + j2] = Ts[c][r];
      }
    }
    __syncthreads();
  }
}

// vectors (r_tilde): mode 0 = chunk totals into tot[g][slot[lc]][E], mode 1 = windows into
// out[g][s - skip][E].  Segment sums as window_prefix_vec_kernel (eight months in flight).
__global__ __launch_bounds__(WV_T) void wvec_chunk_kernel(
    const double* __restrict__ X, int64_t E, int T, const int* __restrict__ seg_start,
    const int* __restrict__ seg_stop, int nseg, int skip, int mode, int nlc,
    const int* __restrict__ cs, const int* __restrict__ ce, const int* __restrict__ slot, int C,
    const int* __restrict__ sb, const int* __restrict__ sy, const int* __restrict__ ys,
    const int* __restrict__ ye, int clast, double* __restrict__ tot, int64_t tstride,
    double* __restrict__ out) {
  __shared__ double part[WV_SEG][WV_COLS];
  const int lc = threadIdx.x % WV_COLS, ry = threadIdx.x / WV_COLS;
  const int g = blockIdx.y, col = blockIdx.x * WV_COLS + lc;
  const bool cv = col < E;
  const double* src = X + (int64_t)g * T * E + (cv ? col : 0);
  for (int s = ry; s < nseg; s += WV_RG) {
    const int a = seg_start[s], b = seg_stop[s];
    double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int tm = a; tm < b; tm += 8) {
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = (tm + u < b) ? src[(int64_t)(tm + u) * E] : 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += x[u];
    }
    part[s][lc] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
  __syncthreads();
  if (ry != 0 || !cv) return;
  double* tg = tot + (int64_t)g * E + col;     // slot k at tg + k * tstride
  if (mode == 0) {
    for (int k = 0; k < nlc; ++k) {
      double acc = 0.0;
      for (int s = cs[k]; s < ce[k]; ++s) acc += part[s][lc];
      tg[(int64_t)slot[k] * tstride] = acc;
    }
    return;
  }
  double pc = 0.0;
  for (int k = 0; k < C; ++k) pc += tg[(int64_t)sb[k] * tstride];
  double* o = out + (int64_t)g * (nseg - skip) * E + col;
  for (int ch = 0; ch <= clast; ++ch) {
    double acc = pc;
    for (int s = ys[ch]; s < ye[ch]; ++s) {
      acc += part[s][lc];
      if (s >= skip) o[(int64_t)(s - skip) * E] = acc;
    }
    if (ch < clast) pc += tg[(int64_t)sy[ch] * tstride];
  }
}

}  // namespace

// Kernel A for the matrices: segment sums (upper triangles) into the out / scratch slots,
// then the local chunk totals.  idx = [cs, ce, slot] (3 x nlc int32, device).
extern "C" hipError_t pfml_wsum_chunk_totals(const double* X, int P, int T, int G,
                                             const int* seg_start, const int* seg_stop, int nseg,
                                             int skip, double* out, double* scratch, int nlc,
                                             const int* idx, double* tot, int64_t tstride,
                                             hipStream_t st) {
  if (nseg <= 0 || P <= 0 || G <= 0) return hipSuccess;
  if (skip < 0 || skip > nseg || (skip > 0 && scratch == nullptr)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wsum_upper_kernel, dim3(P, nseg, G), dim3(256), 0, st, X, P, T, seg_start,
                     seg_stop, nseg, skip, out, scratch);
  if (nlc > 0) {
    const int nt = (P + 31) / 32;
    hipLaunchKernelGGL(wsum_chunk_totals_kernel, dim3(nt * (nt + 1) / 2, G, nlc), dim3(256), 0, st, P,
                       nseg, skip, out, scratch, nlc, idx, idx + nlc, idx + 2 * nlc, tot,
                       tstride);
  }
  return hipGetLastError();
}

// Kernel B for the matrices.  cidx = [sb, sy, ys, ye] (4 x C int32, device).
extern "C" hipError_t pfml_wsum_chunk_prefix(int P, int G, int nseg, int skip, double* out,
                                             double* scratch, int C, const int* cidx,
                                             const double* tot, int64_t tstride, int clast,
                                             hipStream_t st) {
  if (nseg <= 0 || P <= 0 || G <= 0 || clast < 0) return hipSuccess;
  const int nt = (P + 31) / 32;
  hipLaunchKernelGGL(wsum_chunk_prefix_kernel, dim3(nt * (nt + 1) / 2, G, clast + 1), dim3(256), 0, st, P,
                     nseg, skip, out, scratch, C, cidx, cidx + C, cidx + 2 * C, cidx + 3 * C, tot,
                     tstride, clast);
  return hipGetLastError();
}

// Vectors, both kernels (mode 0 / 1); idx and cidx as above.
extern "C" hipError_t pfml_wvec_chunk(const double* X, int64_t E, int T, int G,
                                      const int* seg_start, const int* seg_stop, int nseg,
                                      int skip, int mode, int nlc, const int* idx, int C,
                                      const int* cidx, int clast, double* tot, int64_t tstride,
                                      double* out, hipStream_t st) {
  if (nseg <= 0 || E <= 0 || G <= 0) return hipSuccess;
  if (nseg > WV_SEG || skip < 0) return hipErrorInvalidValue;
  if (mode == 1 && (clast < 0 || nseg - skip <= 0)) return hipSuccess;
  if (mode == 0 && nlc <= 0) return hipSuccess;
  hipLaunchKernelGGL(wvec_chunk_kernel, dim3((unsigned)((E + WV_COLS - 1) / WV_COLS), G),
                     dim3(WV_T), 0, st, X, E, T, seg_start, seg_stop, nseg, skip, mode, nlc, idx,
                     idx + nlc, idx + 2 * nlc, C, cidx, cidx + C, cidx + 2 * C, cidx + 3 * C,
                     clast, tot, tstride, out);
  return hipGetLastError();
}
