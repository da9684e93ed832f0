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
// moments in one pass, then the scaled write) and written once.
#include "common.h"

namespace {

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
                                                          const int* __restrict__ n_real, int TH,
                                                          int N, const double* __restrict__ vol,
                                                          double* __restrict__ out, int64_t ldo,
                                                          int64_t so, int Pw) {
  __shared__ double red[4][64], red2[4][64];
  __shared__ double colmean[64], colscale[64];
  const int bt = blockIdx.y;                  // (b, theta)
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
    for (; i + 12 < n; i += 16) {
      const double x0 = F[rw[i] * ldf + c] - K, x1 = F[rw[i + 4] * ldf + c] - K;
      const double x2 = F[rw[i + 8] * ldf + c] - K, x3 = F[rw[i + 12] * ldf + c] - K;
      s1 += (x0 + x1) + (x2 + x3);
      s2 += (x0 * x0 + x1 * x1) + (x2 * x2 + x3 * x3);
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
  double* o = out + (int64_t)bt * so;
  if (c < Pw)
    for (int i = part; i < N; i += 4) {
      double v = 0.0;
      if (i < n && c < P) v = (F[rw[i] * ldf + c] - mu) * sc / vol[rw[i]];
      o[(int64_t)i * ldo + c] = v;
    }
}

}  // namespace

extern "C" hipError_t pfml_rff_sincos(const double* Z, int64_t R, int half, double* out,
                                      int64_t ldo, hipStream_t st) {
  const int64_t tot = R * (int64_t)half;
  if (tot <= 0) return hipSuccess;
  if (ldo < 2 * (int64_t)half + 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rff_sincos_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, Z,
                     R, half, out, ldo);
  return hipGetLastError();
}

extern "C" hipError_t pfml_standardize(const double* F, int P, int64_t ldf, const int64_t* rows,
                                       const int* n_real, int B, int TH, int N,
                                       const double* vol, double* out, int64_t ldo, int64_t so,
                                       int Pw, hipStream_t st) {
  if (B <= 0 || N <= 0) return hipSuccess;
  if (Pw < P || ldo < Pw || ldf < P) return hipErrorInvalidValue;
  dim3 grid((Pw + 63) / 64, B * TH);
  hipLaunchKernelGGL(standardize_kernel, grid, dim3(256), 0, st, F, P, ldf, rows, n_real, TH, N,
                     vol, out, ldo, so, Pw);
  return hipGetLastError();
}
