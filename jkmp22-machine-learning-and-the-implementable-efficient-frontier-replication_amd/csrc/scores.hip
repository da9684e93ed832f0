// Validation scores (K17; PFML_hp_reals.py:104-125): for one validation frame of the
// utilities obj[nV][G][C] (C = nP * L hyper-parameter combinations) and the g-range [g0, g1)
// it holds (all g' <= g in reference-compat mode, quirk Q2):
//
//   cum[r][c]  = mean of the non-NaN seq[0..r][c] over the frame's rows r = v * k + kk
//                (k = g1 - g0), seq[v * k + kk][c] = obj[v][g0 + kk][c]: pandas
//                expanding().mean() by (p, l), NaN until the first finite value
//   rank[v][i] = dense descending rank of cum[v * k + i / C][i % C] among the month's k * C
//                values; NaN cum gets a NaN rank and is not counted (pandas
//                rank(method='dense', ascending=False)), so a singular cell is never "rank 1"
//
// Two launches replace the ~25 small torch kernels (sort, scans, scatters) per frame, and
// pfml_validation_scores_all does every frame of a grid search in the same two launches:
//   prefix_mean_kernel  4 columns x 64 row chunks per workgroup: chunk sums, LDS offsets,
//                       chunk rescans, NaN carry fix-up (loads batched and clamped)
//   dense_rank_kernel   one workgroup per month: bitonic sort of <= 1024 (key, index) pairs in
//                       LDS (one 16-byte element each, order-preserving 64-bit keys), adjacent-difference + block scan for the dense rank, scatter back
#include "common.h"

namespace {

constexpr int RK_N = 1024;          // max values per month (k * C <= 1024)
constexpr int RK_T = 256;

constexpr int PM_COLS = 4, PM_RG = 64;    // prefix mean: 4 columns x 64 row chunks per WG
                                          // (short chunks: fewer dependent load rounds)

// Frames: blockIdx.y = f of nF frames; frame f covers g in [f0 + f, f1 + f) clipped as
// (g0, g1) = compat ? (0, f + 1) : (f, f + 1) when `multi`, else the single (g0, g0 + k).  Its
// cum rows start at cum + cum_off(f) (frame sizes nV * k_f * C before it).
__device__ __forceinline__ void frame_of(int f, bool multi, bool compat, int g0s, int ks,
                                         int nV, int C, int& g0, int& k, int64_t& off) {
  if (!multi) {
    g0 = g0s; k = ks; off = 0;
    return;
  }
  g0 = compat ? 0 : f;
  k = compat ? f + 1 : 1;
  // sum of the earlier frames' k: compat f (f + 1) / 2, else f
  off = (int64_t)nV * C * (compat ? (int64_t)f * (f + 1) / 2 : f);
}

__global__ __launch_bounds__(256) void prefix_mean_kernel(const double* __restrict__ obj, int nV,
                                                          int G, int g0s, int ks, int C,
                                                          double* __restrict__ cum_all,
                                                          int multi, int compat) {
  int g0, k;
  int64_t coff;
  frame_of(blockIdx.y, multi, compat, g0s, ks, nV, C, g0, k, coff);
  double* __restrict__ cum = cum_all + coff;
  // thread (rg, cg): rows [rg * chunk, (rg + 1) * chunk) of column c; chunk sums / counts of
  // the non-NaN values meet in LDS for the cross-chunk offsets, then each chunk is rescanned.
  // A NaN row must repeat the previous expanding mean BIT FOR BIT (pandas carries its running
  // state; ties then rank alike): inside a chunk the thread repeats its own last value, and
  // the NaN rows leading a chunk take the previous chunks' last value in a fix-up pass.
  __shared__ double part[PM_RG][PM_COLS];
  __shared__ double pcnt[PM_RG][PM_COLS];
  __shared__ double lastv[PM_RG][PM_COLS];
  __shared__ int haslast[PM_RG][PM_COLS];
  const int cg = threadIdx.x % PM_COLS, rg = threadIdx.x / PM_COLS;
  const int c = blockIdx.x * PM_COLS + cg;
  const bool cv = c < C;
  const int cc = cv ? c : C - 1;
  const int R = nV * k;
  const int chunk = (R + PM_RG - 1) / PM_RG;
  const int r0 = rg * chunk, r1 = min(R, r0 + chunk);
  auto at = [&](int r) {
    const int v = r / k, kk = r - v * k;
    return obj[((int64_t)v * G + g0 + kk) * C + cc];
  };
  double s = 0.0, n = 0.0;
  for (int r = r0; r < r1; r += 8) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = at(min(r + u, r1 - 1));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = (r + u < r1) && (x[u] == x[u]);
      s += ok ? x[u] : 0.0;
      n += ok ? 1.0 : 0.0;
    }
  }
  part[rg][cg] = s;
  pcnt[rg][cg] = n;
  __syncthreads();
  s = 0.0;
  n = 0.0;
  for (int q = 0; q < rg; ++q) {
    s += part[q][cg];
    n += pcnt[q][cg];
  }
  int lead = 0;                 // NaN rows before the chunk's first finite value
  bool seen = false;
  double last = __builtin_nan("");
  for (int r = r0; r < r1; r += 8) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = at(min(r + u, r1 - 1));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (r + u < r1) {
        if (x[u] == x[u]) {
          s += x[u];
          n += 1.0;
          last = s / n;
          seen = true;
        } else if (!seen) {
          ++lead;
        }
        if (cv && seen) cum[(int64_t)(r + u) * C + c] = last;
      }
    }
  }
  lastv[rg][cg] = last;
  haslast[rg][cg] = seen ? 1 : 0;
  __syncthreads();
  if (lead > 0 && cv) {
    // the value carried into this chunk: the last finite-based mean of the closest earlier
    // chunk that had one (NaN if none: no finite value yet)
    double carry = __builtin_nan("");
    for (int q = rg - 1; q >= 0; --q)
      if (haslast[q][cg]) { carry = lastv[q][cg]; break; }
    for (int r = r0; r < r0 + lead; ++r) cum[(int64_t)r * C + c] = carry;
  }
}

// Sort key of one value: an unsigned 64-bit word whose ASCENDING order is the rank order -
// descending value (order-preserving bit map of the double, then inverted), every NaN after
// every number (unranked), padding after everything; +0 and -0 share a key (equal values rank
// alike).  Ties are broken by the index, so the sort is a total order on (key, index).
__device__ __forceinline__ unsigned long long rank_key(double x) {
  if (x != x) return ~0ull - 1;
  if (x == 0.0) x = 0.0;
  const unsigned long long u = __double_as_longlong(x);
  const unsigned long long asc = (u >> 63) ? ~u : (u | (1ull << 63));   // ascending in x
  return ~asc - 2;                                                     // descending, < NaN
}
constexpr unsigned long long PAD_KEY = ~0ull;

__global__ __launch_bounds__(RK_T) void dense_rank_kernel(const double* __restrict__ cum_all,
                                                          int Ns, int nV, int C,
                                                          double* __restrict__ rank_all,
                                                          int multi, int compat) {
  // (key, index) pairs as one 16-byte LDS element: one ds_read_b128 / ds_write_b128 each
  __shared__ ulonglong2 el[RK_N];
  __shared__ int wsum[RK_T / 64];
  int g0, k;
  int64_t off;
  frame_of(blockIdx.y, multi, compat, 0, Ns / max(C, 1), nV, C, g0, k, off);
  const int N = multi ? k * C : Ns;
  const double* __restrict__ cum = cum_all + off;
  double* __restrict__ rank = rank_all + off;
  // sort width: the next power of two >= N (a 404-value month sorts 512, not 1024)
  int NS = 2;
  while (NS < N) NS <<= 1;
  const int v = blockIdx.x, t = threadIdx.x;
  const double* src = cum + (int64_t)v * N;
  for (int i = t; i < NS; i += RK_T) {
    ulonglong2 e;
    e.x = (i < N) ? rank_key(src[i]) : PAD_KEY;
    e.y = (unsigned long long)i;                     // padding: indices >= N
    el[i] = e;
  }
  __syncthreads();
  // bitonic sort of NS (key, index) pairs, ascending
  for (int size = 2; size <= NS; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = t; p < NS / 2; p += RK_T) {
        const int lo = 2 * p - (p & (stride - 1)), hi = lo + stride;
        const bool up = (lo & size) == 0;
        const ulonglong2 a = el[lo], b = el[hi];
        const bool gt = a.x > b.x || (a.x == b.x && a.y > b.y);
        if (gt == up) {
          el[lo] = b;
          el[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  // dense rank: new[i] = (i == 0) || key[i] != key[i-1] among the ranked (finite) keys;
  // inclusive scan, 4 per thread
  constexpr unsigned long long NAN_KEY = ~0ull - 1;
  int nw[4], run = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = 4 * t + q;
    const bool real = i < NS && el[i].x < NAN_KEY;
    nw[q] = real && (i == 0 || el[i].x != el[i - 1].x) ? 1 : 0;
    run += nw[q];
  }
  // block exclusive scan of run
  const int lane = t & 63, w = t >> 6;
  int incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int base = 0;
  for (int q = 0; q < w; ++q) base += wsum[q];
  int acc = base + incl - run;
  double* dst = rank + (int64_t)v * N;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = 4 * t + q;
    acc += nw[q];
    if (i < NS && el[i].x != PAD_KEY)
      dst[el[i].y] = (el[i].x < NAN_KEY) ? (double)acc : __builtin_nan("");
  }
}

}  // namespace

extern "C" int pfml_scores_max_per_month() { return RK_N; }

// obj [nV][G][C]; cum [nV * k][C]; rank [nV][k * C]; k = g1 - g0
extern "C" hipError_t pfml_validation_scores(const double* obj, int nV, int G, int g0, int g1,
                                             int C, double* cum, double* rank,
                                             hipStream_t st) {
  const int k = g1 - g0;
  if (nV <= 0 || C <= 0 || k <= 0) return hipSuccess;
  if (k * C > RK_N || g0 < 0 || g1 > G) return hipErrorInvalidValue;
  hipLaunchKernelGGL(prefix_mean_kernel, dim3((C + PM_COLS - 1) / PM_COLS), dim3(256), 0, st, obj,
                     nV, G, g0, k, C, cum, 0, 0);
  hipLaunchKernelGGL(dense_rank_kernel, dim3(nV), dim3(RK_T), 0, st, cum, k * C, nV, C, rank, 0,
                     0);
  return hipGetLastError();
}

// Every frame f = 0 .. G-1 of one grid search in two launches (blockIdx.y = frame): frame f
// holds g' <= f (compat, quirk Q2) or g = f alone.  cum / rank: the frames' [nV, k_f, C]
// blocks back to back (k_f = f + 1 or 1).
extern "C" hipError_t pfml_validation_scores_all(const double* obj, int nV, int G, int C,
                                                 int compat, double* cum, double* rank,
                                                 hipStream_t st) {
  if (nV <= 0 || C <= 0 || G <= 0) return hipSuccess;
  if ((compat ? G : 1) * C > RK_N) return hipErrorInvalidValue;
  hipLaunchKernelGGL(prefix_mean_kernel, dim3((C + PM_COLS - 1) / PM_COLS, G), dim3(256), 0, st,
                     obj, nV, G, 0, 1, C, cum, 1, compat);
  hipLaunchKernelGGL(dense_rank_kernel, dim3(nV, G), dim3(RK_T), 0, st, cum, C, nV, C, rank, 1,
                     compat);
  return hipGetLastError();
}
