// Panel-wide signal kernels of the PFML input stage.
//
// rff_sincos (K13, PFML_Input_Data.py:159-185,245): given Z = X W (computed by pfml_dgemm on
// MFMA), writes the interleaved signal row [1, cos z_1, sin z_1, cos z_2, sin z_2, ...] so every
// hyper-parameter p selects a leading column block.  One sincos per element (sincos shares
// the range reduction).
//
// standardize (K11/K12, :357-391): for each (month batch b, lag theta) tile of N gathered
// rows x P columns: demean the RFF columns (not the constant), scale every column to unit
// L2 norm over the N real rows, then divide each row by its stock's volatility.  One
// workgroup per (b, theta, 64-column strip); rows read twice (shifted first and second
// moments in one pass, then the scaled write) and written once, 8 gathered rows in flight per
// thread in both passes.
#include "common.h"

namespace {

// blockIdx.y -> (b, theta) tile: tiles are enumerated along the diagonals d = b - theta, so
// the TH tiles that gather the SAME month's rows (lag theta of month b reads month b - theta)
// are dispatched together and share those rows through the caches (row-major (b, theta) order
// re-read every gathered row from HBM once per lag).  Returns -1 for the padding slots of the
// first / last diagonals.
__device__ __forceinline__ int diag_tile(int y, int B, int TH) {
  const int d = y / TH, th = y - d * TH;
  const int b = d - (TH - 1) + th;
  return (b < 0 || b >= B) ? -1 : b * TH + th;
}

__global__ __launch_bounds__(256) void rff_sincos_kernel(const double* __restrict__ Z, int64_t R,
                                                         int half, double* __restrict__ out,
                                                         int64_t ldo) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= R * (int64_t)half) return;
  const int64_t r = e / half;
  const int i = (int)(e % half);
  double s, c;
  sincos(Z[e], &s, &c);
  double* o = out + r * ldo;
  o[1 + 2 * i] = c;
  o[2 + 2 * i] = s;
  if (i == 0) {
    o[0] = 1.0;
    for (int64_t q = 2 * (int64_t)half + 1; q < ldo; ++q) o[q] = 0.0;   // pad columns
  }
}

// rows: [B*TH, N] panel row indices (pad rows point to an all-zero row), n_real: [B] real
// rows per batch entry, vol: per panel row.  F: [*, ldf] panel signals (P real columns).
// out element (b*TH + theta, i, c) at out + (b*TH + theta) * so + i * ldo + c, for c < Pw
// (columns P..Pw-1 are written as zeros: the even-width padding of the S4 buffers).
__global__ __launch_bounds__(256) void standardize_kernel(const double* __restrict__ F, int P,
                                                          int64_t ldf,
                                                          const int64_t* __restrict__ rows,
                                                          const int* __restrict__ n_real, int B,
                                                          int TH, int N,
                                                          const double* __restrict__ vol,
                                                          double* __restrict__ out, int64_t ldo,
                                                          int64_t so, int Pw,
                                                          double* __restrict__ stats,
                                                          int64_t lds, int write_out,
                                                          const double* __restrict__ rsc,
                                                          int64_t srsc) {
  __shared__ double red[4][64], red2[4][64];
  __shared__ double colmean[64], colscale[64];
  const int bt = diag_tile(blockIdx.y, B, TH);   // (b, theta)
  if (bt < 0) return;
  const int b = bt / TH;
  const int c0 = blockIdx.x * 64;
  const int t = threadIdx.x, lane = t & 63, part = t >> 6;   // 4 row partitions
  const int c = c0 + lane;
  const int n = n_real[b];
  const int64_t* rw = rows + (int64_t)bt * N;
  // one pass: shifted sums S1 = sum (x - K), S2 = sum (x - K)^2 with K = the column's first
  // real value, so sum (x - mean)^2 = S2 - S1^2 / n without the cancellation of raw moments
  // (K is a sample of the column: |K - mean| is O(std), relative error O(eps)).  Four
  // independent row streams per thread keep loads in flight.
  const double K = (c < P && n > 0) ? F[rw[0] * ldf + c] : 0.0;
  double s1 = 0.0, s2 = 0.0;
  if (c < P) {
    int i = part;
    for (; i + 28 < n; i += 32) {
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = F[rw[i + 4 * u] * ldf + c] - K;
      s1 += ((x[0] + x[1]) + (x[2] + x[3])) + ((x[4] + x[5]) + (x[6] + x[7]));
      s2 += ((x[0] * x[0] + x[1] * x[1]) + (x[2] * x[2] + x[3] * x[3])) +
            ((x[4] * x[4] + x[5] * x[5]) + (x[6] * x[6] + x[7] * x[7]));
    }
    for (; i < n; i += 4) {
      const double x = F[rw[i] * ldf + c] - K;
      s1 += x;
      s2 += x * x;
    }
  }
  red[part][lane] = s1;
  red2[part][lane] = s2;
  __syncthreads();
  if (part == 0) {
    const double t1 = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    const double t2 = red2[0][lane] + red2[1][lane] + red2[2][lane] + red2[3][lane];
    if (c == 0) {                                          // constant column: not demeaned
      colmean[lane] = 0.0;
      const double tk = t1 + (double)n * K;                // sum x
      colscale[lane] = sqrt(1.0 / (t2 + 2.0 * K * tk - (double)n * K * K));
    } else {
      colmean[lane] = K + t1 / (double)n;
      colscale[lane] = sqrt(1.0 / (t2 - t1 * t1 / (double)n));
    }
  }
  __syncthreads();
  const double mu = colmean[lane];
  const double sc = colscale[lane];
  if (stats != nullptr && part == 0 && c < Pw) {   // (pad columns: scale 0 -> a zero addend)
    stats[(int64_t)bt * 2 * lds + c] = c < P ? mu : 0.0;
    stats[(int64_t)bt * 2 * lds + lds + c] = c < P ? sc : 0.0;
  }
  if (!write_out) return;
  double* o = out + (int64_t)bt * so;
  // scaled write: 8 rows per thread per iteration, every load issued before the first use (a
  // row-at-a-time loop waited on each gathered row's index and value in turn)
  if (c < Pw) {
    const int cc = min(c, P - 1);
    for (int i0 = part; i0 < N; i0 += 32) {
      int64_t ri[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) ri[u] = rw[min(i0 + 4 * u, N - 1)];
      double x[8], vv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        x[u] = F[ri[u] * ldf + cc];
        vv[u] = vol[ri[u]];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 4 * u;
        if (i < N) {
          double v = (i < n && c < P) ? (x[u] - mu) * sc / vv[u] : 0.0;
          if (rsc != nullptr) v *= rsc[(int64_t)b * srsc + i];
          o[(int64_t)i * ldo + c] = v;
        }
      }
    }
  }
}

// Register-resident form for N <= 16 * RPT rows (the S&P 500 universe): 1024 threads per
// (b, theta, 64-column strip), thread (part = t >> 6, lane) holds rows part + 16 u (u < RPT)
// of column c0 + lane in registers, so the gathered rows are read from HBM ONCE (the two-pass
// kernel above reads them twice; the stage is HBM-bound on those gathered reads + the write).
template <int RPT>
__global__ __launch_bounds__(1024) void standardize_reg_kernel(
    const double* __restrict__ F, int P, int64_t ldf, const int64_t* __restrict__ rows,
    const int* __restrict__ n_real, int B, int TH, int N, const double* __restrict__ vol,
    double* __restrict__ out, int64_t ldo, int64_t so, int Pw, double* __restrict__ stats,
    int64_t lds, int write_out, const double* __restrict__ rsc, int64_t srsc) {
  constexpr int NP = 16;
  __shared__ double red[NP][64], red2[NP][64];
  __shared__ double colmean[64], colscale[64];
  const int bt = diag_tile(blockIdx.y, B, TH);
  if (bt < 0) return;
  const int b = bt / TH;
  const int c0 = blockIdx.x * 64;
  const int t = threadIdx.x, lane = t & 63;
  const int part = __builtin_amdgcn_readfirstlane(t >> 6);
  const int c = c0 + lane;
  const int cc = min(c, P - 1);
  const int n = n_real[b];
  // row indices are < 2^31: read their low words (halves the scalar registers they take)
  const int* rw = reinterpret_cast<const int*>(rows + (int64_t)bt * N);
  const double K = (n > 0) ? F[(int64_t)rw[0] * ldf + cc] : 0.0;
  double x[RPT];
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const int i = part + NP * u;
    x[u] = (i < n) ? F[(int64_t)rw[2 * i] * ldf + cc] : K;          // rows >= n: x - K = 0
  }
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const double d = x[u] - K;
    s1 += d;
    s2 += d * d;
  }
  red[part][lane] = s1;
  red2[part][lane] = s2;
  __syncthreads();
  if (part == 0) {
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      t1 += red[q][lane];
      t2 += red2[q][lane];
    }
    if (c == 0) {                                          // constant column: not demeaned
      colmean[lane] = 0.0;
      const double tk = t1 + (double)n * K;
      colscale[lane] = sqrt(1.0 / (t2 + 2.0 * K * tk - (double)n * K * K));
    } else {
      colmean[lane] = K + t1 / (double)n;
      colscale[lane] = sqrt(1.0 / (t2 - t1 * t1 / (double)n));
    }
  }
  __syncthreads();
  if (c >= Pw) return;
  const double mu = colmean[lane];
  const double sc = colscale[lane];
  if (stats != nullptr && part == 0) {             // (pad columns: scale 0 -> a zero addend)
    stats[(int64_t)bt * 2 * lds + c] = c < P ? mu : 0.0;
    stats[(int64_t)bt * 2 * lds + lds + c] = c < P ? sc : 0.0;
  }
  if (!write_out) return;
  double* o = out + (int64_t)bt * so;
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const int i = part + NP * u;
    if (i < N) {
      double v = (i < n && c < P) ? (x[u] - mu) * sc / vol[rw[2 * i]] : 0.0;
      if (rsc != nullptr) v *= rsc[(int64_t)b * srsc + i];     // (a separate rounding step)
      o[(int64_t)i * ldo + c] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Signal statistics of lags 1..10 by differences (models/pfml_inputs.py run_plan).  Lag theta
// of month b standardises the rows of b's universe at date d = b - theta; the ten months that
// read date d have nearly the same universe (a few names enter or leave per month), so the
// column sums over U(d) = the union of those universes' rows at d are formed ONCE per date
// (date_sums_kernel) and each (b, theta) subtracts the few rows of U(d) outside its own
// universe (excl_stats_kernel) - instead of re-reading ~N gathered rows per (b, theta).
//   dsum[d] = [S1 = sum (x - K), S2 = sum (x - K)^2, K] over U(d), K = x of U(d)'s first row
//   (t1, t2) = (S1, S2) - the same sums over the excluded rows, then the standardize kernels'
//   mean / scale formulas (shifted moments: no cancellation of raw ones).
// U(d) is built from the GLOBAL month grid and every sum runs in a fixed order, so a month's
// statistics are bitwise the same however the months are sharded or batched.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void date_sums_kernel(const double* __restrict__ F, int P,
                                                         int64_t ldf,
                                                         const int64_t* __restrict__ urows,
                                                         const int* __restrict__ un, int umax,
                                                         int Pw, double* __restrict__ dsum) {
  constexpr int NP = 16;
  __shared__ double red[NP][64], red2[NP][64];
  const int d = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63;
  const int part = __builtin_amdgcn_readfirstlane(t >> 6);
  const int c = blockIdx.x * 64 + lane;
  const int cc = min(c, P - 1);
  const int n = un[d];
  const int64_t* rw = urows + (int64_t)d * umax;
  const double K = (n > 0) ? F[rw[0] * ldf + cc] : 0.0;
  double s1 = 0.0, s2 = 0.0;
  for (int i0 = part; i0 < n; i0 += 8 * NP) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + NP * u;
      x[u] = (i < n) ? F[rw[i] * ldf + cc] - K : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s1 += x[u];
      s2 += x[u] * x[u];
    }
  }
  red[part][lane] = s1;
  red2[part][lane] = s2;
  __syncthreads();
  if (part == 0 && c < Pw) {
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      t1 += red[q][lane];
      t2 += red2[q][lane];
    }
    double* o = dsum + (int64_t)d * 3 * Pw;
    o[c] = t1;
    o[Pw + c] = t2;
    o[2 * Pw + c] = K;
  }
}

__global__ __launch_bounds__(256) void excl_stats_kernel(
    const double* __restrict__ F, int P, int64_t ldf, const int64_t* __restrict__ erows,
    const int* __restrict__ en, int emax, const int* __restrict__ dpos,
    const double* __restrict__ dsum, const int* __restrict__ n_real, int TH, int Pw,
    double* __restrict__ stats, int64_t lds) {
  constexpr int NP = 4;
  __shared__ double red[NP][64], red2[NP][64];
  const int bt = blockIdx.y, b = bt / TH;
  const int t = threadIdx.x, lane = t & 63;
  const int part = __builtin_amdgcn_readfirstlane(t >> 6);
  const int c = blockIdx.x * 64 + lane;
  const int cc = min(c, P - 1);
  const int ne = en[bt];
  const int64_t* rw = erows + (int64_t)bt * emax;
  const double* ds = dsum + (int64_t)dpos[bt] * 3 * Pw;
  const int cw = min(c, Pw - 1);
  const double K = ds[2 * Pw + cw];
  double e1 = 0.0, e2 = 0.0;
  for (int i0 = part; i0 < ne; i0 += 4 * NP) {
    double x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + NP * u;
      x[u] = (i < ne) ? F[rw[i] * ldf + cc] - K : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      e1 += x[u];
      e2 += x[u] * x[u];
    }
  }
  red[part][lane] = e1;
  red2[part][lane] = e2;
  __syncthreads();
  if (part != 0 || c >= Pw) return;
  double u1 = 0.0, u2 = 0.0;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    u1 += red[q][lane];
    u2 += red2[q][lane];
  }
  const double t1 = ds[c] - u1, t2 = ds[Pw + c] - u2;
  const double n = (double)n_real[b];
  double mu, sc;
  if (c == 0) {                                          // constant column: not demeaned
    mu = 0.0;
    const double tk = t1 + n * K;
    sc = sqrt(1.0 / (t2 + 2.0 * K * tk - n * K * K));
  } else {
    mu = K + t1 / n;
    sc = sqrt(1.0 / (t2 - t1 * t1 / n));
  }
  stats[(int64_t)bt * 2 * lds + c] = c < P ? mu : 0.0;
  stats[(int64_t)bt * 2 * lds + lds + c] = c < P ? sc : 0.0;
}

}  // namespace

// per-date shifted column sums over U(d): urows [nd, umax] panel rows (first un[d] real),
// dsum [nd, 3, Pw] (S1, S2, K rows)
extern "C" hipError_t pfml_date_sums(const double* F, int P, int64_t ldf, const int64_t* urows,
                                     const int* un, int umax, int nd, int Pw, double* dsum,
                                     hipStream_t st) {
  if (nd <= 0) return hipSuccess;
  if (Pw < P || ldf < P) return hipErrorInvalidValue;
  hipLaunchKernelGGL(date_sums_kernel, dim3((Pw + 63) / 64, nd), dim3(1024), 0, st, F, P, ldf,
                     urows, un, umax, Pw, dsum);
  return hipGetLastError();
}

// statistics of the B x TH tiles (b, theta) from their date's sums minus their excluded rows:
// erows [B * TH, emax] (first en[.] real), dpos [B * TH] date slot, stats as pfml_standardize
extern "C" hipError_t pfml_excl_stats(const double* F, int P, int64_t ldf, const int64_t* erows,
                                      const int* en, int emax, const int* dpos,
                                      const double* dsum, const int* n_real, int B, int TH,
                                      int Pw, double* stats, int64_t lds, hipStream_t st) {
  if (B <= 0 || TH <= 0) return hipSuccess;
  if (Pw < P || ldf < P || lds < Pw) return hipErrorInvalidValue;
  hipLaunchKernelGGL(excl_stats_kernel, dim3((Pw + 63) / 64, B * TH), dim3(256), 0, st, F, P, ldf,
                     erows, en, emax, dpos, dsum, n_real, TH, Pw, stats, lds);
  return hipGetLastError();
}

extern "C" hipError_t pfml_rff_sincos(const double* Z, int64_t R, int half, double* out,
                                      int64_t ldo, hipStream_t st) {
  const int64_t tot = R * (int64_t)half;
  if (tot <= 0) return hipSuccess;
  if (ldo < 2 * (int64_t)half + 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rff_sincos_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, Z,
                     R, half, out, ldo);
  return hipGetLastError();
}

// stats (nullable): the column means and scales of every (b, theta) tile, [B*TH][2][lds]
// (mean row, then scale row; columns P..Pw-1 zero); write_out = 0: the stats only (the
// standardised values are then formed where they are consumed: the Horner GEMM's gathered
// addend, csrc/gemm_f64.hip).  rsc (nullable): an output row scale rsc[b * srsc + i] applied
// after the standardisation (the k-scale of the Horner step that reads the block: T_11's
// signal block is written in place, scaled, with no separate pass)
extern "C" hipError_t pfml_standardize(const double* F, int P, int64_t ldf, const int64_t* rows,
                                       const int* n_real, int B, int TH, int N,
                                       const double* vol, double* out, int64_t ldo, int64_t so,
                                       int Pw, double* stats, int64_t lds, int write_out,
                                       const double* rsc, int64_t srsc, hipStream_t st) {
  if (B <= 0 || N <= 0) return hipSuccess;
  if (Pw < P || ldf < P || (write_out && ldo < Pw) || (stats && lds < Pw) ||
      (!write_out && !stats))
    return hipErrorInvalidValue;
  dim3 grid((Pw + 63) / 64, (B + TH - 1) * TH);     // diagonal order (diag_tile)
  if (N <= 16 * 32)
    hipLaunchKernelGGL(standardize_reg_kernel<32>, grid, dim3(1024), 0, st, F, P, ldf, rows,
                       n_real, B, TH, N, vol, out, ldo, so, Pw, stats, lds, write_out, rsc,
                       srsc);
  else
    hipLaunchKernelGGL(standardize_kernel, grid, dim3(256), 0, st, F, P, ldf, rows, n_real, B, TH,
                       N, vol, out, ldo, so, Pw, stats, lds, write_out, rsc, srsc);
  return hipGetLastError();
}
