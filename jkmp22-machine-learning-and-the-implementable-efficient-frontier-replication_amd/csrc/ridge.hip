// Ridge hyper-parameter grid, eq. (26):  beta_l = (Dbar_p + l I)^-1 rbar_p  for every l.
//
// Reference: PFML_Search_Coef.py:124-137 runs np.linalg.solve (an O(n^3) LU) 101 times per
// (g, year, p).  All 101 systems share Dbar_p, so this kernel factors Dbar_p ONCE with a
// Householder tridiagonalisation  Dbar = Q T Q^T  (4/3 n^3 flops), after which every lambda
// costs a tridiagonal solve (O(n)) plus its share of the back-transform Q y (O(n^2)):
//
//     beta_l = Q (T + l I)^-1 Q^T rbar
//
// One 1024-thread workgroup owns one (g, year, p) cell; the n x n working copy lives in
// global memory (L2-resident: 2.1 MB at n = 513) and every Householder step makes ONE fused
// read+write pass over the trailing matrix that applies the previous step's rank-2 update
// and, in the same sweep, forms the next step's symmetric mat-vec (the standard sytd2
// formulation needs two passes).  The tridiagonal systems use Gaussian elimination with
// partial pivoting (as LAPACK dgtsv) so lambda = 0 on an indefinite/singular-ish Dbar behaves
// like the reference's pivoted LU rather than failing.
#include "common.h"

namespace {

constexpr int NMAX = 1024;      // largest p+1 supported (p_max = 512 -> 513)
constexpr int NT = 1024;        // threads per workgroup
constexpr int NW = NT / 64;

struct CellDesc {
  int64_t src;      // offset (doubles) of the running-sum matrix S_D for this cell
  int64_t rsrc;     // offset of the running-sum vector S_r
  int64_t work;     // offset of this cell's workspace
  int64_t out;      // offset of beta output [L][ldo]
  int n;            // p + 1
  double scale;     // 1 / T  (the reference divides both sums by n months)
};

__global__ __launch_bounds__(NT) void ridge_tridiag_kernel(
    const double* __restrict__ SD, int64_t ldS, const double* __restrict__ Sr,
    const CellDesc* __restrict__ cells, const double* __restrict__ lvec, int L,
    double* __restrict__ work, double* __restrict__ beta_out, int64_t ldo) {
  __shared__ double v[NMAX], vp[NMAX], wp[NMAX], pk[NMAX], z[NMAX];
  __shared__ double dd[NMAX], ee[NMAX], tau[NMAX];
  __shared__ double red[NW * 2];
  __shared__ double bcast[4];
  __shared__ double part[8][128];

  const CellDesc cd = cells[blockIdx.x];
  const int n = cd.n;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  double* A = work + cd.work;                 // n x n, ld n
  double* Y = A + (int64_t)n * n;             // n x L  ([i][l])
  double* Ua = Y + (int64_t)n * L;            // pivoted-LU of T + lI, per lambda, [i][l]
  double* Ub = Ua + (int64_t)n * L;
  double* Uc = Ub + (int64_t)n * L;
  double* Uy = Uc + (int64_t)n * L;
  const double* S = SD + cd.src;
  const double sc = cd.scale;

  // ---- load scaled copy + rhs ---------------------------------------------------------
  for (int64_t e = t; e < (int64_t)n * n; e += NT) {
    const int i = (int)(e / n), j = (int)(e % n);
    A[e] = S[(int64_t)i * ldS + j] * sc;
  }
  for (int i = t; i < n; i += NT) {
    z[i] = Sr[cd.rsrc + i] * sc;
    vp[i] = 0.0;
    wp[i] = 0.0;
    v[i] = 0.0;
  }
  __syncthreads();

  // block reduction of two values at once
  auto bsum2 = [&](double a, double b, double& ra, double& rb) {
    a = wave_sum(a);
    b = wave_sum(b);
    if (lane == 0) { red[wid] = a; red[NW + wid] = b; }
    __syncthreads();
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) { sa += red[q]; sb += red[NW + q]; }
    ra = sa;
    rb = sb;
    __syncthreads();
  };

  for (int k = 0; k + 2 < n; ++k) {
    // (1) column k with the previous rank-2 update applied:  c_i, i >= k   (stored into pk)
    const double vpk = vp[k], wpk = wp[k];
    for (int i = k + t; i < n; i += NT)
      pk[i] = A[(int64_t)i * n + k] - vp[i] * wpk - wp[i] * vpk;
    __syncthreads();
    // (2) Householder vector from x = c[k+1:]
    double x2 = 0.0;
    for (int i = k + 2 + t; i < n; i += NT) x2 += pk[i] * pk[i];
    double xnorm2, dummy;
    bsum2(x2, 0.0, xnorm2, dummy);
    const double alpha = pk[k + 1];
    double tk, ek, scal;
    if (xnorm2 == 0.0) {
      tk = 0.0; ek = alpha; scal = 0.0;
    } else {
      const double bet = -copysign(sqrt(alpha * alpha + xnorm2), alpha);
      tk = (bet - alpha) / bet;
      scal = 1.0 / (alpha - bet);
      ek = bet;
    }
    if (t == 0) { dd[k] = pk[k]; ee[k] = ek; tau[k] = tk; }
    for (int i = k + 1 + t; i < n; i += NT) {
      const double vi = (i == k + 1) ? 1.0 : pk[i] * scal;
      v[i] = vi;
      A[(int64_t)i * n + k] = vi;              // keep the reflector for the back-transform
    }
    __syncthreads();
    // (3) fused pass: A22 -= vp wp^T + wp vp^T ; pk_i = sum_j A22_ij v_j   (i, j >= k+1)
    for (int i = k + 1 + wid; i < n; i += NW) {
      const double vpi = vp[i], wpi = wp[i];
      double* row = A + (int64_t)i * n;
      double acc = 0.0;
      for (int j = k + 1 + lane; j < n; j += 64) {
        const double a = row[j] - vpi * wp[j] - wpi * vp[j];
        row[j] = a;
        acc += a * v[j];
      }
      acc = wave_sum(acc);
      if (lane == 0) pk[i] = tk * acc;
    }
    __syncthreads();
    // (4) w = p - (tau/2)(p.v) v ;  z <- H_k z
    double pv = 0.0, vz = 0.0;
    for (int i = k + 1 + t; i < n; i += NT) { pv += pk[i] * v[i]; vz += v[i] * z[i]; }
    double spv, svz;
    bsum2(pv, vz, spv, svz);
    const double half = 0.5 * tk * spv;
    for (int i = k + 1 + t; i < n; i += NT) {
      wp[i] = pk[i] - half * v[i];
      vp[i] = v[i];
      z[i] -= tk * svz * v[i];
    }
    if (t == 0) { vp[k] = 0.0; wp[k] = 0.0; }
    __syncthreads();
  }
  // trailing 2 x 2 (or smaller) block
  if (t == 0) {
    if (n >= 2) {
      const int a = n - 2, b = n - 1;
      const double Aaa = A[(int64_t)a * n + a] - 2.0 * vp[a] * wp[a];
      const double Aba = A[(int64_t)b * n + a] - vp[b] * wp[a] - wp[b] * vp[a];
      const double Abb = A[(int64_t)b * n + b] - 2.0 * vp[b] * wp[b];
      dd[a] = Aaa; ee[a] = Aba; dd[b] = Abb;
    } else {
      dd[0] = A[0];
    }
  }
  __syncthreads();

  // ---- tridiagonal solves: one thread per lambda (GE with partial pivoting) -------------
  if (t < L) {
    const int l = t;
    const double lam = lvec[l];
    double a = dd[0] + lam, b = (n > 1) ? ee[0] : 0.0, c = 0.0, y = z[0];
    for (int i = 0; i + 1 < n; ++i) {
      const double lo = ee[i];
      const double dn = dd[i + 1] + lam;
      const double up = (i + 2 < n) ? ee[i + 1] : 0.0;
      const double zn = z[i + 1];
      double na, nb, ny;
      if (fabs(a) >= fabs(lo)) {
        const double m = (a != 0.0) ? lo / a : 0.0;
        Ua[(int64_t)i * L + l] = a; Ub[(int64_t)i * L + l] = b; Uc[(int64_t)i * L + l] = c;
        Uy[(int64_t)i * L + l] = y;
        na = dn - m * b; nb = up - m * c; ny = zn - m * y;
      } else {
        const double m = a / lo;
        Ua[(int64_t)i * L + l] = lo; Ub[(int64_t)i * L + l] = dn; Uc[(int64_t)i * L + l] = up;
        Uy[(int64_t)i * L + l] = zn;
        na = b - m * dn; nb = c - m * up; ny = y - m * zn;
      }
      a = na; b = nb; c = 0.0; y = ny;
    }
    double x1 = y / a, x2 = 0.0;
    Y[(int64_t)(n - 1) * L + l] = x1;
    for (int i = n - 2; i >= 0; --i) {
      const double xi = (Uy[(int64_t)i * L + l] - Ub[(int64_t)i * L + l] * x1 -
                         Uc[(int64_t)i * L + l] * x2) / Ua[(int64_t)i * L + l];
      Y[(int64_t)i * L + l] = xi;
      x2 = x1;
      x1 = xi;
    }
  }
  __syncthreads();

  // ---- back-transform  Y <- H_0 H_1 ... H_{n-3} Y --------------------------------------
  const int lcol = t & 127, prt = t >> 7;   // 8 row-partitions x 128 lambda columns
  for (int k = n - 3; k >= 0; --k) {
    for (int i = k + 1 + t; i < n; i += NT) v[i] = A[(int64_t)i * n + k];
    __syncthreads();
    double s = 0.0;
    if (lcol < L)
      for (int i = k + 1 + prt; i < n; i += 8) s += v[i] * Y[(int64_t)i * L + lcol];
    part[prt][lcol] = s;
    __syncthreads();
    if (lcol < L) {
      double tot = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) tot += part[q][lcol];
      const double f = tau[k] * tot;
      for (int i = k + 1 + prt; i < n; i += 8) Y[(int64_t)i * L + lcol] -= f * v[i];
    }
    __syncthreads();
  }
  // ---- write beta_l (lambda-major, ld ldo) ---------------------------------------------
  double* out = beta_out + cd.out;
  for (int64_t e = t; e < (int64_t)L * n; e += NT) {
    const int l = (int)(e / n), i = (int)(e % n);
    out[(int64_t)l * ldo + i] = Y[(int64_t)i * L + l];
  }
}

}  // namespace

extern "C" int64_t pfml_ridge_work_doubles(int n, int L) {
  return (int64_t)n * n + 5LL * n * L;
}

extern "C" hipError_t pfml_ridge_grid(const double* SD, int64_t ldS, const double* Sr,
                                      const void* cells, int ncells, const double* lvec, int L,
                                      double* work, double* beta_out, int64_t ldo,
                                      hipStream_t st) {
  if (ncells <= 0) return hipSuccess;
  if (L > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ridge_tridiag_kernel, dim3(ncells), dim3(NT), 0, st, SD, ldS, Sr,
                     static_cast<const CellDesc*>(cells), lvec, L, work, beta_out, ldo);
  return hipGetLastError();
}

extern "C" int pfml_ridge_cell_desc_size() { return (int)sizeof(CellDesc); }
extern "C" int pfml_ridge_nmax() { return NMAX; }
