// Barra risk-model kernels for gfx950.
//
//   K21  daily_ols_kernel      per trading day: Z = [X | y] staged through LDS 64 rows at a time,
//                              Z'Z (32 x 32) on v_mfma_f64_16x16x4 (so X'X and X'y come out of
//                              one MFMA pass), LU with partial pivoting of X'X in LDS, residuals.
//                              Reference: Estimate Covariance Matrix.py:214-233 - one Python
//                              iteration per day with a full-array boolean mask (≈182 s); here
//                              rows are CSR-segmented by day and every day is one workgroup.
//                              An exactly-zero pivot is LAPACK's LinAlgError; the reference then
//                              uses coef = pinv(X'X) X'y (:226-229).  The same workgroup does
//                              that on the device: [X'X | X'y] is rebuilt from the MFMA
//                              accumulators, X'X = V diag(e) V' by cyclic Jacobi in LDS, and
//                              coef = V diag(1/e) V' X'y over |e| > 1e-15 max|e| (numpy pinv's
//                              default rcond on the singular values); status = 2 marks the day.
//   K22  ewma_factor_cov_kernel per calc month-end: the trailing <= obs days of factor returns,
//                              normalised EWMA weights for the correlation (hl_cor) and the
//                              variance (hl_var), weighted means, centred weighted Gram matrices
//                              on MFMA, unbiased 1/(1 - sum w^2) (R cov.wt), and the fused
//                              epilogue F = sd cor sd * scale (General_functions.py:745-835,
//                              Estimate Covariance Matrix.py:297-335).
//   K23  ewma_vol_kernel       zero-mean EWMA volatility per stock (the numba @njit kernel,
//                              Estimate Covariance Matrix.py:345-386): one wave per stock, the
//                              affine recurrence var_i = a_i var_{i-1} + b_i scanned 64 rows at a
//                              time with a wave-level (a, b) composition scan (NaN x: a=1, b=0).
#include "common.h"

namespace {

constexpr int KP = 32;         // padded factor count: K + 1 <= 32 (y rides as column K)
constexpr int ZS = KP + 16;    // LDS row stride (doubles): rows 16 apart land 32 banks apart
constexpr int OLS_ROWS = 64;

// ---------------------------------------------------------------------------------------
// K21
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void daily_ols_kernel(
    const double* __restrict__ X, const double* __restrict__ y, const int64_t* __restrict__ off,
    int K, double* __restrict__ coef, double* __restrict__ resid, int* __restrict__ status) {
  __shared__ double Zs[OLS_ROWS][ZS];
  __shared__ double G[KP][KP + 1];
  __shared__ double beta_s[KP];
  __shared__ int piv_s;
  __shared__ int bad_s;
  const int d = blockIdx.x;
  const int64_t a = off[d], b = off[d + 1];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int ti = (w >> 1) * 16, tj = (w & 1) * 16;

  double4_t acc = {0.0, 0.0, 0.0, 0.0};
  for (int64_t r0 = a; r0 < b; r0 += OLS_ROWS) {
    for (int e = t; e < OLS_ROWS * KP; e += 256) {
      const int i = e / KP, c = e % KP;
      const int64_t r = r0 + i;
      double v = 0.0;
      if (r < b) v = (c < K) ? X[r * K + c] : ((c == K) ? y[r] : 0.0);
      Zs[i][c] = v;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < OLS_ROWS; k += 4) {
      const double av = Zs[k + (lane >> 4)][ti + (lane & 15)];
      const double bv = Zs[k + (lane >> 4)][tj + (lane & 15)];
      acc = mfma_f64_16x16x4(av, bv, acc);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) G[ti + PFML_F64_CROW(lane, r)][tj + (lane & 15)] = acc[r];
  if (t == 0) bad_s = 0;
  __syncthreads();

  // LU with partial pivoting on [X'X | X'y] (dgesv): first index of the max |pivot|.
  for (int k = 0; k < K; ++k) {
    if (w == 0) {
      double v = (lane >= k && lane < K) ? fabs(G[lane][k]) : -1.0;
      int idx = lane;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(idx, o, 64);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
      }
      if (lane == 0) {
        piv_s = idx;
        if (!(v > 0.0)) bad_s = 1;      // exactly singular (or NaN): LinAlgError
      }
    }
    __syncthreads();
    if (bad_s) break;
    const int p = piv_s;
    if (p != k && t <= K) {
      const double tmp = G[k][t];
      G[k][t] = G[p][t];
      G[p][t] = tmp;
    }
    __syncthreads();
    const int wd = K - k;                     // columns k+1..K (incl. the rhs)
    const double pk = G[k][k];
    for (int e = t; e < (K - k - 1) * wd; e += 256) {
      const int i = k + 1 + e / wd, j = k + 1 + e % wd;
      G[i][j] -= (G[i][k] / pk) * G[k][j];
    }
    __syncthreads();
  }
  if (bad_s) {
    // ---- pinv fallback: rebuild G = [X'X | X'y] from the accumulators ------------------
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) G[ti + PFML_F64_CROW(lane, r)][tj + (lane & 15)] = acc[r];
    __shared__ double V[KP][KP + 1];
    __shared__ double rot[2];
    for (int e = t; e < KP * KP; e += 256) V[e / KP][e % KP] = (e / KP == e % KP) ? 1.0 : 0.0;
    __syncthreads();
    if (t < K) beta_s[t] = G[t][K];                          // X'y (G's column K)
    // cyclic Jacobi sweeps on the K x K block (uniform control flow, threads k < K update
    // column / row k); rotations below the classic threshold are skipped
    for (int sweep = 0; sweep < 16; ++sweep) {
      for (int pp = 0; pp < K - 1; ++pp)
        for (int qq = pp + 1; qq < K; ++qq) {
          __syncthreads();
          if (t == 0) {
            const double app = G[pp][pp], aqq = G[qq][qq], apq = G[pp][qq];
            double c = 1.0, sn = 0.0;
            if (fabs(apq) > 1e-300 && fabs(apq) > 1e-18 * sqrt(fabs(app * aqq))) {
              const double th = (aqq - app) / (2.0 * apq);
              const double tt = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
              c = 1.0 / sqrt(tt * tt + 1.0);
              sn = tt * c;
            }
            rot[0] = c;
            rot[1] = sn;
          }
          __syncthreads();
          const double c = rot[0], sn = rot[1];
          if (sn == 0.0) continue;                             // uniform: same in every thread
          if (t < K) {                                         // columns p, q (A and V)
            const double akp = G[t][pp], akq = G[t][qq];
            G[t][pp] = c * akp - sn * akq;
            G[t][qq] = sn * akp + c * akq;
            const double vkp = V[t][pp], vkq = V[t][qq];
            V[t][pp] = c * vkp - sn * vkq;
            V[t][qq] = sn * vkp + c * vkq;
          }
          __syncthreads();
          if (t < K) {                                         // rows p, q
            const double apk = G[pp][t], aqk = G[qq][t];
            G[pp][t] = c * apk - sn * aqk;
            G[qq][t] = sn * apk + c * aqk;
          }
        }
    }
    __syncthreads();
    // coef = V diag(1/e) V' X'y over |e| > 1e-15 max |e|
    if (w == 0) {
      double emax = 0.0;
      for (int k = 0; k < K; ++k) emax = fmax(emax, fabs(G[k][k]));
      const double cut = 1e-15 * emax;
      double proj = 0.0;                                     // lane k: (V' X'y)_k / e_k
      if (lane < K) {
        for (int j = 0; j < K; ++j) proj += V[j][lane] * beta_s[j];
        const double ek = G[lane][lane];
        proj = (fabs(ek) > cut) ? proj / ek : 0.0;
      }
      double ci = 0.0;
      for (int k = 0; k < K; ++k) {
        const double pk = __shfl(proj, k, 64);
        if (lane < K) ci += V[lane][k] * pk;
      }
      __builtin_amdgcn_wave_barrier();
      if (lane < K) {
        beta_s[lane] = ci;
        coef[(int64_t)d * K + lane] = ci;
      }
      if (lane == 0) status[d] = 2;
    }
  } else {
    // back substitution U beta = c (wave 0; lane j keeps beta_j)
    if (w == 0) {
      double bj = 0.0;
      for (int i = K - 1; i >= 0; --i) {
        const double part = (lane > i && lane < K) ? G[i][lane] * bj : 0.0;
        const double s = wave_sum(part);
        const double bi = (G[i][K] - s) / G[i][i];
        if (lane == i) bj = bi;
      }
      if (lane < K) {
        beta_s[lane] = bj;
        coef[(int64_t)d * K + lane] = bj;
      }
      if (lane == 0) status[d] = 0;
    }
  }
  __syncthreads();
  for (int64_t r = a + t; r < b; r += 256) {
    double s = 0.0;
    for (int j = 0; j < K; ++j) s += X[r * K + j] * beta_s[j];
    resid[r] = y[r] - s;
  }
}

// ---------------------------------------------------------------------------------------
// K22
// ---------------------------------------------------------------------------------------
constexpr int COV_ROWS = 64;

__global__ __launch_bounds__(256) void ewma_factor_cov_kernel(
    const double* __restrict__ fr, int K, const int64_t* __restrict__ ends, int obs,
    const double* __restrict__ w_cor, const double* __restrict__ w_var, double scale,
    double* __restrict__ F, double* __restrict__ cor_out, double* __restrict__ var_out,
    int nan_cor) {
  __shared__ double Xs[COV_ROWS][ZS];
  __shared__ double sw[2][COV_ROWS];
  __shared__ double mu[2][KP];
  __shared__ double red[2][8][KP];
  __shared__ double C[2][KP][KP + 1];
  __shared__ double scr[8];
  const int bi = blockIdx.x;
  const int64_t e = ends[bi];
  const int tl = (int)min<int64_t>((int64_t)obs, e);
  const int64_t s0 = e - tl;
  const double* wc = w_cor + (obs - tl);
  const double* wv = w_var + (obs - tl);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;

  // weight normalisers: sum w and sum (w / sum w)^2 for both kinds
  double sc = 0.0, sv = 0.0;
  for (int k = t; k < tl; k += 256) {
    sc += wc[k];
    sv += wv[k];
  }
  sc = block_sum(sc, scr);
  sv = block_sum(sv, scr);
  double qc = 0.0, qv = 0.0;
  for (int k = t; k < tl; k += 256) {
    const double a = wc[k] / sc, b = wv[k] / sv;
    qc += a * a;
    qv += b * b;
  }
  qc = block_sum(qc, scr);
  qv = block_sum(qv, scr);

  // weighted means: thread (column c = t & 31, row phase g = t >> 5)
  {
    const int c = t & 31, g = t >> 5;
    double mc = 0.0, mv = 0.0;
    if (c < K) {
      for (int k = g; k < tl; k += 8) {
        const double x = fr[(s0 + k) * K + c];
        mc += (wc[k] / sc) * x;
        mv += (wv[k] / sv) * x;
      }
    }
    red[0][g][c] = mc;
    red[1][g][c] = mv;
    __syncthreads();
    if (t < 2 * KP) {
      const int kind = t / KP, cc = t % KP;
      double m = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) m += red[kind][q][cc];
      mu[kind][cc] = m;
    }
  }
  __syncthreads();

  // centred weighted Gram matrices: wave w -> kind (w >> 1), tile row (w & 1), both tile cols
  const int kind = w >> 1, ti = (w & 1) * 16;
  double4_t acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
  for (int r0 = 0; r0 < tl; r0 += COV_ROWS) {
    for (int q = t; q < COV_ROWS * KP; q += 256) {
      const int i = q / KP, c = q % KP;
      const int k = r0 + i;
      Xs[i][c] = (k < tl && c < K) ? fr[(s0 + k) * K + c] : 0.0;
    }
    if (t < 2 * COV_ROWS) {
      const int kk = t / COV_ROWS, i = t % COV_ROWS;
      const int k = r0 + i;
      sw[kk][i] = (k < tl) ? sqrt((kk == 0 ? wc[k] / sc : wv[k] / sv)) : 0.0;
    }
    __syncthreads();
    const double* m = mu[kind];
#pragma unroll 4
    for (int k = 0; k < COV_ROWS; k += 4) {
      const int row = k + (lane >> 4), col = lane & 15;
      const double s = sw[kind][row];
      const double av = (Xs[row][ti + col] - m[ti + col]) * s;
      const double b0 = (Xs[row][col] - m[col]) * s;
      const double b1 = (Xs[row][16 + col] - m[16 + col]) * s;
      acc0 = mfma_f64_16x16x4(av, b0, acc0);
      acc1 = mfma_f64_16x16x4(av, b1, acc1);
    }
    __syncthreads();
  }
  const double den = 1.0 / (1.0 - (kind == 0 ? qc : qv));
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ti + PFML_F64_CROW(lane, r), j = lane & 15;
    C[kind][i][j] = acc0[r] * den;
    C[kind][i][16 + j] = acc1[r] * den;
  }
  __syncthreads();
  for (int q = t; q < K * K; q += 256) {
    const int i = q / K, j = q % K;
    // a factor with no exposure in the window (an industry without members: its daily OLS
    // coefficient is the pinv's zero) has variance 0.  nan_cor (compat mode): cov / (sd sd')
    // as weighted_cor_wt divides (General_functions.py:827), 0 / 0 = NaN off the diagonal,
    // which poisons that month's Sigma as it does the reference's; corrected mode: those
    // correlations are 0, so F carries 0 there (the reference's pinv mostly leaves ~1e-16
    // noise instead of an exact zero, i.e. F ~ 1e-32)
    const double dn = sqrt(C[0][i][i]) * sqrt(C[0][j][j]);
    const double cor = (i == j) ? 1.0 : ((nan_cor || dn > 0.0) ? C[0][i][j] / dn : 0.0);
    const double sdi = sqrt(C[1][i][i]), sdj = sqrt(C[1][j][j]);
    const int64_t o = (int64_t)bi * K * K + q;
    F[o] = sdi * cor * sdj * scale;
    if (cor_out) cor_out[o] = cor;
    if (var_out) var_out[o] = C[1][i][j];
  }
}

// ---------------------------------------------------------------------------------------
// K23
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void compose_scan(double& A, double& B, int lane) {
  // inclusive scan of affine maps v -> A v + B in lane order (earlier lanes applied first)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double Ae = __shfl_up(A, o, 64);
    const double Be = __shfl_up(B, o, 64);
    if (lane >= o) {
      B = A * Be + B;
      A = A * Ae;
    }
  }
}

__global__ __launch_bounds__(256) void ewma_vol_kernel(const double* __restrict__ x,
                                                       const int64_t* __restrict__ gs,
                                                       int64_t ng, double lam, int start,
                                                       double* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= ng) return;                       // wave-uniform
  const int lane = threadIdx.x & 63;
  const int64_t a = gs[g], b = gs[g + 1], n = b - a;
  const double nan = __builtin_nan("");
  const int64_t lim = (n > start) ? start : n;
  for (int64_t i = lane; i < lim; i += 64) out[a + i] = nan;
  if (n <= start) return;
  double ss = 0.0, cnt = 0.0;
  for (int64_t i = lane; i < start; i += 64) {
    const double v = x[a + i];
    if (!__builtin_isnan(v)) {
      ss += v * v;
      cnt += 1.0;
    }
  }
  ss = wave_sum(ss);
  cnt = wave_sum(cnt);
  if (cnt <= 1.0) {
    for (int64_t i = start + lane; i < n; i += 64) out[a + i] = nan;
    return;
  }
  double carry = ss / (cnt - 1.0);
  if (lane == 0) out[a + start] = sqrt(carry);
  const double one_m = 1.0 - lam;
  for (int64_t i0 = start + 1; i0 < n; i0 += 64) {
    const int64_t i = i0 + lane;
    double A = 1.0, B = 0.0;
    if (i < n) {
      const double xp = x[a + i - 1];
      if (!__builtin_isnan(xp)) {
        A = lam;
        B = one_m * xp * xp;
      }
    }
    compose_scan(A, B, lane);
    const double v = A * carry + B;
    if (i < n) out[a + i] = sqrt(v);
    carry = __shfl(v, 63, 64);
  }
}

}  // namespace

extern "C" int pfml_risk_max_factors() { return KP - 1; }

extern "C" hipError_t pfml_daily_ols(const double* X, const double* y, const int64_t* off,
                                     int ndays, int K, double* coef, double* resid, int* status,
                                     hipStream_t st) {
  if (K < 1 || K > KP - 1) return hipErrorInvalidValue;
  if (ndays <= 0) return hipSuccess;
  hipLaunchKernelGGL(daily_ols_kernel, dim3(ndays), dim3(256), 0, st, X, y, off, K, coef, resid,
                     status);
  return hipGetLastError();
}

extern "C" hipError_t pfml_ewma_factor_cov(const double* fr, int K, const int64_t* ends, int nb,
                                           int obs, const double* w_cor, const double* w_var,
                                           double scale, double* F, double* cor_out,
                                           double* var_out, int nan_cor, hipStream_t st) {
  if (K < 1 || K > KP) return hipErrorInvalidValue;
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(ewma_factor_cov_kernel, dim3(nb), dim3(256), 0, st, fr, K, ends, obs, w_cor,
                     w_var, scale, F, cor_out, var_out, nan_cor);
  return hipGetLastError();
}

extern "C" hipError_t pfml_ewma_vol(const double* x, const int64_t* gs, int64_t ng, double lam,
                                    int start, double* out, hipStream_t st) {
  if (ng <= 0) return hipSuccess;
  const int64_t blocks = (ng + 3) / 4;
  hipLaunchKernelGGL(ewma_vol_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, gs, ng, lam,
                     start, out);
  return hipGetLastError();
}
