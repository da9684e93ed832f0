// Ridge hyper-parameter grid, eq. (26), band path:  beta_l = (Dbar + l I)^-1 rbar  for all l.
//
// Reference: PFML_Search_Coef.py:124-137 (np.linalg.solve per lambda).  The tridiagonal path
// (ridge.hip) factors Dbar = Q T Q^T with one Householder reflector at a time; every reflector
// needs a full mat-vec over the trailing matrix, i.e. ~n^3/3 doubles streamed per cell through
// ONE CU, and that stream (not the flops) bounds it.  This path reduces Dbar to BAND form
// instead (bandwidth BB = 16, the two-sided blocked Householder of the first stage of a
// two-stage symmetric eigensolver):
//
//     Dbar = Q B Q^T,   Q = Q_0 Q_1 ... Q_{np-1},   Q_p = I - V_p T_p V_p^T  (compact WY)
//
// per panel p (16 columns) the trailing matrix is read once for X = A22 V T and read+written
// once for the rank-32 update A22 -= V W^T + W V^T, both on v_mfma_f64_16x16x4 with V, W
// resident in LDS: 16x fewer passes over the trailing matrix than one pass per reflector.
// Then every lambda is an independent banded Cholesky solve (B + l I) y = Q^T rbar (one wave
// per lambda, register window with DPP broadcasts, O(n BB^2)), and beta = Q y is a blocked-WY back-transform
// (MFMA, Y chunk of 16 lambdas resident in registers).
//
//   kernel 1  band_coop_kernel               K workgroups per cell (1..16, chosen per launch),
//                                            bitwise independent of K
//   kernel 2  ridge_band_solve_kernel        4 lambdas per wave (16-lane DPP rows)
//   kernel 3  ridge_band_backtransform_kernel one 512-thread workgroup per (cell, 16 lambdas)
//
// A non-positive Cholesky pivot (Dbar + l I not numerically SPD, e.g. l = 0 on a singular
// Dbar) marks that lambda's y NaN; kernel 2b re-solves exactly those systems in the band
// domain by LU with partial pivoting (np.linalg.solve semantics) before the back-transform.
#include "common.h"
#include "ridge_desc.h"
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int BB = 16;              // bandwidth = panel width = MFMA tile
constexpr int LS = BB + 1;          // LDS row stride (bank spread for column-wise reads)
constexpr int BMP = 512;            // max panel rows m = n - r0  (n <= BNMAX)
constexpr int BNMAX = BMP + BB;     // 528 >= p_max + 1
constexpr int NTR = 512;            // reduce kernel: 8 waves
constexpr int NWR = NTR / 64;
constexpr int TBR = 4;              // trailing-update tiles per wave per pass
constexpr int NTB = 512;            // back-transform kernel: 8 waves
constexpr int NWB = NTB / 64;
constexpr int LC = 16;              // lambdas per back-transform workgroup

// Per-cell workspace layout (doubles).  A has room for the padded npad x npad matrix
// (npad = n rounded up to 16).
__host__ __device__ __forceinline__ int band_npad(int n) { return (n + BB - 1) & ~(BB - 1); }

struct BandWork {
  double *A, *LB, *z, *T, *Yt, *Lf, *F;
  __device__ BandWork(double* w, int n, int L) {
    const int np = (n + BB - 1) / BB;
    const int npad = band_npad(n);
    A = w;                                   // working matrix (V_p / R_p stored below)
    LB = A + (int64_t)npad * npad;           // n x LS lower band: LB[r][s] = B[r][r-16+s]
    z = LB + (int64_t)n * LS;                // Q^T rbar
    T = z + n;                               // np x 16 x 16 compact-WY T_p
    Yt = T + (int64_t)np * BB * BB;          // L x n   solutions y_l, then beta_l
    // banded Cholesky factors: L x n x 16 sub-diagonal entries (one 128-byte line per row,
    // the base rounded up to 16 doubles: every row is written whole by one store
    // instruction), then L x n inverse diagonals
    Lf = w + ((((Yt - w) + (int64_t)L * n) + 15) & ~(int64_t)15);
    F = Lf + (int64_t)L * n * LS;            // cooperative hand-off scratch (CoopWork)
  }
};

// DPP helpers (gfx950: row_newbcast broadcasts one lane of each 16-lane row).
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// (row_newbcast reads a valid source lane for every lane, so "old" is never used)
template <int SEL>
__device__ __forceinline__ double row_bcast(double v) {   // lane SEL of each 16-lane row
  // one v_mov_b64_dpp (64-bit DPP supports row_newbcast on gfx90a+/gfx950)
  const long s = __builtin_bit_cast(long, v);
  const long r = __builtin_amdgcn_update_dpp(s, s, 0x150 + SEL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, r);
}

// w += bcast_SEL(src) * m  as ONE v_fmac_f64_dpp (row_newbcast on the DPP source).  The
// first use after `src` is written must follow a VALU write by 2 wait states: FIRST adds them.
template <int SEL, bool FIRST>
__device__ __forceinline__ void fmac_bcast(double& w, double src, double m) {
  if constexpr (FIRST)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(w) : "v"(src), "v"(m), "i"(SEL));
  else
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(w) : "v"(src), "v"(m), "i"(SEL));
}

// w -= bcast_SEL(src) * m  (the DPP source negated by the instruction's neg modifier: no
// separate negation of src)
template <int SEL, bool FIRST>
__device__ __forceinline__ void fnmac_bcast(double& w, double src, double m) {
  if constexpr (FIRST)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(w) : "v"(src), "v"(m), "i"(SEL));
  else
    asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(w) : "v"(src), "v"(m), "i"(SEL));
}

// 1/sqrt(x) with ONE Newton step on v_rsq_f64 (~2^-46 relative: the banded Cholesky's pivots,
// far below the factorisation's own n eps backward error)
__device__ __forceinline__ double rsqrt1_f64(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return y * fma(-0.5 * x * y, y, 1.5);
}

template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// 1/sqrt(x) to full fp64 accuracy: v_rsq_f64 refined by Newton steps, a short dependent
// chain in place of the IEEE sqrt and divide sequences on the banded Cholesky's pivot path.
// Measured on MI355X over x in 1e-30 .. 1e30 (tools/micro/rsq_acc.hip): the seed is good to
// ~2^-24 relative, two steps give <= 2 ulp of the IEEE 1/sqrt, a third step changes nothing
// (still 2 ulp), so two steps.
__device__ __forceinline__ double rsqrt_f64(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
#pragma unroll
  for (int it = 0; it < 2; ++it) y = y * fma(-h * y, y, 1.5);
  return y;
}

// 1/x to full fp64 accuracy: v_rcp_f64 refined by Newton steps (e = 1 - x y, y += y e); two
// steps are correctly rounded on every measured x (rsq_acc.hip), as three were.
__device__ __forceinline__ double rcp_f64(double x) {
  double y = __builtin_amdgcn_rcp(x);
#pragma unroll
  for (int it = 0; it < 2; ++it) y = fma(y, fma(-x, y, 1.0), y);
  return y;
}

// w[U + s] = LDS row at byte address `base` (s = 0 .. LS-1) in the lanes U, U+16, U+32, U+48
// (the pivot lane of each 16-lane row): 17 ds_read_b64 straight into the window registers
// under an exec mask set and restored INSIDE the one asm statement (no branch, and "+v": the
// other lanes keep their values, so no merge copies), and NO wait: the caller overlaps the
// loads with independent work and then calls lds_row_wait<U>, which waits for them and ties
// the same registers, so no read of w[U..U+16] can be scheduled between the two.  (Written in
// plain C++ the compiler issued the loads into temporaries, waited for them at once and merged
// them with 14 masked moves: the LDS latency sat on every step.)
// `pv` (the pivot, unchanged) is tied through the asm so that the rsq chain that consumes it
// is scheduled after the loads are issued.
template <int U>
__device__ __forceinline__ void lds_row_issue(double* w, unsigned base, double& pv) {
  static_assert(LS == 17, "17 loads");
  const unsigned long long mask = 0x0001000100010001ULL << U;
  unsigned long long saved;
  // ("memory": the stores into the staged rows are only read here)
  asm volatile(
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[mk]\n\t"
      "ds_read_b64 %[w0], %[a] offset:0\n\t"
      "ds_read_b64 %[w1], %[a] offset:8\n\t"
      "ds_read_b64 %[w2], %[a] offset:16\n\t"
      "ds_read_b64 %[w3], %[a] offset:24\n\t"
      "ds_read_b64 %[w4], %[a] offset:32\n\t"
      "ds_read_b64 %[w5], %[a] offset:40\n\t"
      "ds_read_b64 %[w6], %[a] offset:48\n\t"
      "ds_read_b64 %[w7], %[a] offset:56\n\t"
      "ds_read_b64 %[w8], %[a] offset:64\n\t"
      "ds_read_b64 %[w9], %[a] offset:72\n\t"
      "ds_read_b64 %[w10], %[a] offset:80\n\t"
      "ds_read_b64 %[w11], %[a] offset:88\n\t"
      "ds_read_b64 %[w12], %[a] offset:96\n\t"
      "ds_read_b64 %[w13], %[a] offset:104\n\t"
      "ds_read_b64 %[w14], %[a] offset:112\n\t"
      "ds_read_b64 %[w15], %[a] offset:120\n\t"
      "ds_read_b64 %[w16], %[a] offset:128\n\t"
      "s_mov_b64 exec, %[sv]"
      : [sv] "=&s"(saved), [pv] "+v"(pv), [w0] "+v"(w[U + 0]), [w1] "+v"(w[U + 1]), [w2] "+v"(w[U + 2]), [w3] "+v"(w[U + 3]), [w4] "+v"(w[U + 4]), [w5] "+v"(w[U + 5]), [w6] "+v"(w[U + 6]), [w7] "+v"(w[U + 7]), [w8] "+v"(w[U + 8]), [w9] "+v"(w[U + 9]), [w10] "+v"(w[U + 10]), [w11] "+v"(w[U + 11]), [w12] "+v"(w[U + 12]), [w13] "+v"(w[U + 13]), [w14] "+v"(w[U + 14]), [w15] "+v"(w[U + 15]), [w16] "+v"(w[U + 16])
      : [a] "v"(base), [mk] "s"(mask)
      : "memory");
}

// (`dep`, unchanged, ties the wait after the value the caller computes under the loads)
template <int U>
__device__ __forceinline__ void lds_row_wait(double* w, double& dep) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(dep), "+v"(w[U]), "+v"(w[U + 1]), "+v"(w[U + 2]), "+v"(w[U + 3]), "+v"(w[U + 4]),
                 "+v"(w[U + 5]), "+v"(w[U + 6]), "+v"(w[U + 7]), "+v"(w[U + 8]),
                 "+v"(w[U + 9]), "+v"(w[U + 10]), "+v"(w[U + 11]), "+v"(w[U + 12]),
                 "+v"(w[U + 13]), "+v"(w[U + 14]), "+v"(w[U + 15]), "+v"(w[U + 16]));
}

// (64-bit DPP supports only row_newbcast, so the butterfly levels are 32-bit DPP moves)
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_mov<0xB1>(v);      // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);      // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);     // row_half_mirror
  v += dpp_mov<0x140>(v);     // row_mirror
  return v;
}

// Sum of v over lanes {l, l^16, l^32, l^48} (the 4 row groups of a wave), with the gfx950
// VALU lane swaps instead of two ds_bpermute round trips.
__device__ __forceinline__ double rowgroup_sum(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  v = __hiloint2double((int)h16[0], (int)l16[0]) + __hiloint2double((int)h16[1], (int)l16[1]);
  const int lo2 = __double2loint(v), hi2 = __double2hiint(v);
  const auto l32 = __builtin_amdgcn_permlane32_swap(lo2, lo2, false, false);
  const auto h32 = __builtin_amdgcn_permlane32_swap(hi2, hi2, false, false);
  return __hiloint2double((int)h32[0], (int)l32[0]) + __hiloint2double((int)h32[1], (int)l32[1]);
}

// ---------------------------------------------------------------------------------------
// kernel 1: band reduction of one cell.
// ---------------------------------------------------------------------------------------
// X = U^-1 for upper U given by columns (lane c16: uc[i] = U[i][c16]) and di[i] = 1 / U[i][i];
// x[i] = X[i][c16].  Only entries above the diagonal of uc are read.
__device__ __forceinline__ void triu_inv16(const double (&uc)[BB], const double (&di)[BB],
                                           double (&x)[BB], int c16) {
  // right-looking: row k of X is final once the rows below it are; its update of the rows
  // above is 16 independent accumulations (back-to-back FMAs, no dependent chain)
  double acc[BB];
#pragma unroll
  for (int i = 0; i < BB; ++i) acc[i] = 0.0;
  static_for<0, BB>([&](auto KK) {
    constexpr int k = BB - 1 - decltype(KK)::value;
    x[k] = ((c16 == k) ? 1.0 + acc[k] : acc[k]) * di[k];
    const double nxk = -x[k];
    static_for<0, k>([&](auto I) {
      constexpr int i = decltype(I)::value;
      fmac_bcast<k, true>(acc[i], uc[i], nxk);     // acc[i] -= U[i][k] X[k][c16]
    });
  });
}

// P1 + P2 + T of one panel, by one NTR-thread workgroup: the m x 16 panel below the band
// (columns r0.. of rows k0..k0+15 of the symmetric A) is QR-factored by Householder in
// registers; V (unit lower trapezoid) -> Vs, V and R -> A's panel columns, the compact-WY T
// (dlarft) -> Ts and Tglob.  Ends with a barrier.  `redf` needs 2 x 256 + 32 doubles.
// `n` is A's leading dimension.  `Pn`: the panel is read from this LDS image (Pn[i][c] = panel
// row i, column c; it may alias Vs) instead of A's mirror row.
// (A CholeskyQR2 form with Householder reconstruction measured 45-60 % slower per panel,
// profiles/r04_qr_bench_dpp.jsonl, and was removed.)
__device__ __forceinline__ void band_panel_hh(double* __restrict__ A, int n, int k0, int r0,
                                              int m, double (*Vs)[LS], double (*Gs)[LS],
                                              double* redf, double (*Ts)[LS], double* taus,
                                              double* __restrict__ Tglob, long long* tk,
                                              const double (*Pn)[LS]) {
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int cq = t & 15, rg = t >> 4;
  const int c16 = lane & 15, g4 = lane >> 4;
  // ---- P1: thread (rg, cq) loads rows i = rg + 32 q (q < 16) of panel column cq straight
  //      into registers (row k0+cq of the symmetric A; all 16 loads in flight at once)
  double a[16];
  if (Pn != nullptr) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = rg + 32 * q;
      a[q] = (i < m) ? Pn[i][cq] : 0.0;
    }
  } else {
    const double* src = A + (int64_t)(k0 + cq) * n + r0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = rg + 32 * q;
      a[q] = (i < m) ? src[i] : 0.0;
    }
  }
  if (tk) tk[0] = (long long)__builtin_amdgcn_s_memtime();
  // ---- P2: Householder QR of the m x 16 panel in REGISTERS: column j reaches the 16 lanes
  //      of a row group by row_newbcast DPP, fused into the FMA that consumes it
  //      (v_fmac_f64_dpp); one barrier per column (cross-wave sums, ping-pong buffers).
  //      A finished column keeps its Householder vector UNSCALED below the diagonal (u = the
  //      column at its own step; v = scal u): its scal is applied once, when V is written, and
  //      the dlarft dots of later steps carry it as one factor - so every element costs two
  //      fp64 operations per step (its share of the dots and its update), not five.
  double tau_r[BB];
  double myscal = 0.0;                           // scal of this lane's column once finished
  static_for<0, BB>([&](auto J) {
    constexpr int j = decltype(J)::value;
    const int par = j & 1;
    // (tk: per-column sub-phases of thread 0's wave, accumulated in tk[2..4]: own work before
    // the barrier, barrier wait, reductions + pivot chain + update after it)
    const long long tc0 = tk ? (long long)__builtin_amdgcn_s_memtime() : 0;
    double s1p[4] = {0.0, 0.0, 0.0, 0.0};
    // Only row group q = 0 (rows < 32) meets the diagonal; groups of four row groups at or
    // beyond m are all-zero and skipped (one wave-uniform branch per four).  Four partial
    // sums break the FMA chain.
#pragma unroll
    for (int q4 = 0; q4 < 16; q4 += 4) {
      if (q4 > 0 && 32 * q4 >= m) continue;
#pragma unroll
      for (int q = q4; q < q4 + 4; ++q) {
        const int i = rg + 32 * q;
        const double mq = (q > 0 || i > j) ? a[q] : 0.0;       // rows below the diagonal
        // (DPP source a[q]: only a[0] can have been written by a plain VALU op just before -
        // the diagonal fix-up of the last column; every other a[q] was last written by this
        // asm sequence >= 2 instructions earlier, so only q = 0 needs the 2 wait states)
        if (q == 0) fmac_bcast<j, true>(s1p[q & 3], a[q], mq);  // += x_j[i] a_cq[i]
        else fmac_bcast<j, false>(s1p[q & 3], a[q], mq);
      }
    }
    // sum over the wave's 4 row groups (lanes l, l^16, l^32, l^48): VALU lane swaps
    const double s1 = rowgroup_sum((s1p[0] + s1p[1]) + (s1p[2] + s1p[3]));
    if (lane < 16) redf[par * 256 + wid * 16 + lane] = s1;
    if (rg == j) redf[512 + par * 16 + cq] = a[0];       // row j (q = 0)
    long long tc1 = 0;
    if (tk) {
      tc1 = (long long)__builtin_amdgcn_s_memtime();
      tk[2] += tc1 - tc0;
    }
    __syncthreads();
    if (tk) {
      const long long tc2 = (long long)__builtin_amdgcn_s_memtime();
      tk[3] += tc2 - tc1;
      tk[5] = tc2;
    }
    // the wave partials summed as a depth-3 tree (not an 8-deep chain), and the column's
    // scalars below without a branch, so the dc sum overlaps the rsq / rcp chain instead of
    // following it (the compiler kept every instruction after a data-dependent branch behind it)
    static_assert(NWR == 8, "tree sum of 8 wave partials");
    double xs[NWR], ds[NWR];
#pragma unroll
    for (int w = 0; w < NWR; ++w) {
      xs[w] = redf[par * 256 + w * 16 + j];
      ds[w] = redf[par * 256 + w * 16 + cq];
    }
    const double xn2 = ((xs[0] + xs[1]) + (xs[2] + xs[3])) + ((xs[4] + xs[5]) + (xs[6] + xs[7]));
    const double dc = ((ds[0] + ds[1]) + (ds[2] + ds[3])) + ((ds[4] + ds[5]) + (ds[6] + ds[7]));
    const double alpha = redf[512 + par * 16 + j];
    const double vjc = redf[512 + par * 16 + cq];
    // beta = -sign(alpha) ||x||, tau = 1 + |alpha| / ||x||, 1 / (alpha - beta) =
    // sign(alpha) / (|alpha| + ||x||): one rsq and one rcp chain (Newton-refined) instead of
    // the IEEE sqrt and two divide sequences on the per-column critical path.  xn2 = 0 (nothing
    // below the diagonal): tau = 0, beta = alpha, scal = 0 (the chains run on a dummy 1).
    const bool zc = xn2 == 0.0;
    const double nrm2 = zc ? 1.0 : fma(alpha, alpha, xn2);
    const double rn = rsqrt_f64(nrm2);
    const double nrm = nrm2 * rn;
    const double beta = zc ? alpha : -copysign(nrm, alpha);
    const double tau = zc ? 0.0 : fma(fabs(alpha), rn, 1.0);
    const double scal = zc ? 0.0 : copysign(rcp_f64(fabs(alpha) + nrm), alpha);
    // v_j' a_cq = a_cq[j] + scal sum_{i > j} x_j[i] a_cq[i] = vjc + scal dc: for cq > j the
    // update coefficient wc = tau (...), for a finished column cq < j (unscaled u_cq, factor
    // myscal) the dlarft dot G[cq][j] = v_cq' v_j = myscal (...): G = V'V comes free
    const double gcj = vjc + scal * dc;
    const double wc = tau * gcj;
    if (t < j) Gs[t][j] = myscal * gcj;          // (t < 16: row group 0, cq = t)
    tau_r[j] = tau;
    const bool upd = cq > j, own = cq == j;
    if (own) myscal = scal;
    // columns cq > j: a[i] -= v_j[i] wc = scal x_j[i] wc below the diagonal, a[j] -= wc on
    // it; column j: beta on the diagonal, u = x below it (scaled later); cq < j: unchanged
    const double nsw = upd ? -(scal * wc) : 0.0;
#pragma unroll
    for (int q4 = 0; q4 < 16; q4 += 4) {
      if (q4 > 0 && 32 * q4 >= m) continue;
#pragma unroll
      for (int q = q4; q < q4 + 4; ++q) {
        const int i = rg + 32 * q;
        if (q == 0) {
          const double ns0 = (i > j) ? nsw : 0.0;
          fmac_bcast<j, true>(a[0], a[0], ns0);
          if (i == j) a[0] = upd ? a[0] - wc : (own ? beta : a[0]);
        } else {
          fmac_bcast<j, false>(a[q], a[q], nsw);
        }
      }
    }
    if (t == 0) taus[j] = tau;
    if (tk) tk[4] += (long long)__builtin_amdgcn_s_memtime() - tk[5];
  });
  // explicit V -> Vs (MFMA operand); V (strictly lower) and R (upper) -> A's panel columns
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = rg + 32 * q;
    const double v = a[q] * myscal;
    Vs[i][cq] = (i > cq) ? v : ((i == cq && i < m) ? 1.0 : 0.0);
    if (i < m) A[(int64_t)(r0 + i) * n + k0 + cq] = (i > cq) ? v : a[q];
  }
  __syncthreads();
  if (tk) tk[1] = (long long)__builtin_amdgcn_s_memtime();
  // ---- T of the compact WY form: T^-1 = diag(1 / tau) + striu(V'V) (Puglisi; Joffrain,
  //      Low, Quintana-Orti, van de Geijn, "Accumulating Householder transformations,
  //      revisited", 2006), inverted in registers by every wave (lane c16: column c16 of U,
  //      1 / U_kk = tau_k - a zero tau gives a zero row and column of T, as dlarft does)
  {
    double uc[BB], tc[BB];
#pragma unroll
    for (int i = 0; i < BB; ++i) uc[i] = (i < c16) ? Gs[i][c16] : 0.0;
    triu_inv16(uc, tau_r, tc, c16);
    if (wid == 0 && g4 == 0) {
#pragma unroll
      for (int i = 0; i < BB; ++i) Ts[i][c16] = tc[i];
    }
  }
  __syncthreads();
  if (t < BB * BB) Tglob[t] = Ts[t / BB][t % BB];
}

// ---------------------------------------------------------------------------------------
// kernel 1, cooperative form (band_mode 4, the production form): K workgroups per cell in
// ONE launch, K chosen per cell by the host (ops/ridge.py::coop_plan) so that a launch fills
// the chip whether it holds 106 big cells (one GPU) or 13 (one rank of eight).  The results
// are BITWISE independent of K: every value has one producer whose arithmetic does not
// depend on which workgroup runs it, and every cross-block sum runs over per-block partials in
// a fixed block order.  So a 1-GPU and an N-GPU grid search pick the same hyper-parameters
// (PFML_hp_reals.py:118-122 dense rank, PFML_best_hps.py:275 first rank).
//
// Work units are 16-row blocks of the trailing matrix A22, of which only the LOWER block
// triangle (diagonal tiles whole) is stored: the update writes no mirror tiles and the X phase
// reads column block I above its first row from row block I (dsytrd 'L' semantics: the
// input's upper triangle is never read).  Per panel p:
//
//   B  every WG   U = V_p T_p (LDS), X_I = A22 U for the blocks I it owns in the X phase (the
//                 QR WG the last x0(nI, K) blocks, a cost-model split; the others the rest
//                 round-robin), partials V_I' X_I and V_I' z_I per block
//   C  every WG   P = sum_I V_I' X_I and V'z in block order, M = T' P, z_I -= V_I T' V'z,
//                 W_I = X_I - V_I M / 2 for its X blocks
//   D  QR WG      look-ahead: the tiles (I, 0) of A22 ARE panel p+1; it applies update p to
//                 them in registers and factors panel p+1 (band_panel_hh) while
//      others     apply A22 -= V W' + W V' to their update blocks, tiles (I, J), 1 <= J <= I
//                 (tile (0, 0): the diagonal band block)
//
// With K = 1 the one workgroup runs D's update first, then the look-ahead panel: the same
// operations in the same order.  Hand-offs between the workgroups of a cell
// (cdna_hip_programming.md Guideline 16): every handed-off byte is stored write-through (sc1:
// 8- and 16-byte buffer stores through descriptors on the cell's workspace), every storing
// wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier behind which one lane adds to
// the cell's arrival counter; consumers poll that counter relaxed and read the small payloads
// (V, T, W, partials, z) with sc1 loads; the matrix reads of the X phase follow one agent-scope
// acquire per panel.  Spins are bounded (spin_max polls, pfml_coop_set_spin_max): a timeout
// sets the cell's error word, every later wait of the workgroup returns at once and the launch
// drains (never a hang); the back-transform then writes NaN betas for that cell, so the grid
// search's non-finite-cell recovery (models/search.py recompute_cells, the reference's
// np.linalg.solve per lambda) replaces them, and the host counts the timed-out cells from the
// error words of every launch (ops/ridge.py coop_errors: COUNTERS ridge.coop_timeouts).
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int COOP_SYNC = 32;               // u32 words of sync state per cell (128 B)
constexpr unsigned COOP_SPIN_MAX = 1u << 22;   // default poll bound (~1 s of s_sleep 1)
unsigned g_coop_spin_max = COOP_SPIN_MAX;      // host-side: lowered by tests to force timeouts

// hand-off scratch of one cell (in BandWork's F region: 2 npad x 16 + 256 + 33 x 272 doubles)
struct CoopWork {
  double *Vg, *Wg, *Tg, *Pg, *Pzg;
  __device__ CoopWork(double* f, int npad) {
    Vg = f;                                  // V_p rows 0..m-1 (published by the QR WG)
    Wg = Vg + (int64_t)npad * BB;            // W_p rows (every WG its X blocks)
    Tg = Wg + (int64_t)npad * BB;            // T_p
    Pg = Tg + BB * BB;                       // per block V_I' X_I  [33][256]
    Pzg = Pg + (BNMAX / BB) * BB * BB;       // per block V_I' z_I  [33][16]
  }
};

struct CoopSync {
  gu32* ctr;
  gu32* err;
  int K;
  unsigned epoch;
  unsigned spin_max;
  // Every thread of the workgroup calls it; returns with the cell's K workgroups past the
  // same point.  acquire: one agent-scope acquire behind the poll (plain loads of other
  // workgroups' matrix tiles follow).
  __device__ __forceinline__ void sync(bool acquire, int* err_s) {
    ++epoch;
    if (K == 1) {
      __syncthreads();
      return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its sc1 stores are out
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)K * epoch;
      unsigned spins = 0;
      bool bad = *err_s != 0;
      while (!bad && __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins >= spin_max) {
          bad = true;
          *err_s = 1;
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (acquire) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
  }
};

// One k-chunk (NV x 8 rows of A22 from k) of the X phase for the NQ blocks of a wave, the
// first NB of which lie entirely BELOW the chunk (their first row <= k) and the rest entirely
// above it.  Lane (c16, g4) takes the k pair kk, kk + 1 (kk = k + 8 v + 2 g4) into two MFMAs (the
// k order inside the 16 x 16 x 4 steps is permuted, the same for every block and every K):
// above a block the pair is ONE 16-byte load along row i of the lower triangle (the 16 lanes of
// a k-group read 16 rows: half the load instructions of one 8-byte load per k), below it two
// row loads (coalesced along the block's 16 columns).  No per-element branch: with one the
// compiler made both paths exec-masked and waited for each load's predecessor (WAW).
template <int NQ, int NB, int NV>
__device__ __forceinline__ void coop_x_chunk(const double* __restrict__ A, int lda, int r0, int m,
                                             int k, const int (&col)[NQ], int c16, int g4,
                                             const double (*__restrict__ Us)[LS],
                                             double4_t (&X)[4]) {
  typedef double d2v __attribute__((ext_vector_type(2)));   // 16-B aligned: one dwordx4 load
  double a0[NV][NQ], a1[NV][NQ], b0[NV], b1[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int kk = k + 8 * v + 2 * g4;
    static_for<0, NQ>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      if constexpr (q < NB) {
        a0[v][q] = A[(int64_t)(r0 + min(kk, m - 1)) * lda + r0 + col[q]];
        a1[v][q] = A[(int64_t)(r0 + min(kk + 1, m - 1)) * lda + r0 + col[q]];
      } else {
        const d2v x = *reinterpret_cast<const d2v*>(A + (int64_t)(r0 + col[q]) * lda + r0 + kk);
        a0[v][q] = x.x;
        a1[v][q] = x.y;
      }
    });
    // (rows >= m of U are zero; the clamp keeps a last chunk inside Us)
    b0[v] = Us[min(kk, BMP - 1)][c16];
    b1[v] = Us[min(kk + 1, BMP - 1)][c16];
  }
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      X[q] = mfma_f64_16x16x4(a0[v][q], b0[v], X[q]);
      X[q] = mfma_f64_16x16x4(a1[v][q], b1[v], X[q]);
    }
}

// X_I += A22[k][I cols] U[k][:] for the NQ blocks blk[] of this wave (increasing).  Only the
// LOWER triangle of A22 is kept (the update writes no mirror tiles): element (kk, i) of column
// block I is A[kk][i] for rows kk at or below the block's first row and A[i][kk] above it - the
// same value a mirrored copy held.  The first rows of a wave's blocks are equal mod 32 (its
// blocks are 8 K' apart), so 32-row chunks aligned to them (after a 16-row head when they are
// 16 mod 32) never straddle one: each chunk is one coop_x_chunk<NQ, NB> with NB uniform.
template <int NQ>
__device__ __forceinline__ void coop_x_accum(const double* __restrict__ A, int lda, int r0,
                                             int m, const int (&blk)[4], int c16, int g4,
                                             const double (*__restrict__ Us)[LS],
                                             double4_t (&X)[4]) {
  int col[NQ], top[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    col[q] = min(blk[q] * 16 + c16, m - 1);
    top[q] = blk[q] * 16;
  }
  auto chunk = [&](int k, auto NV) {
    int nb = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) nb += (top[q] <= k) ? 1 : 0;
    static_for<0, NQ + 1>([&](auto B) {
      if (nb == decltype(B)::value)
        coop_x_chunk<NQ, decltype(B)::value, decltype(NV)::value>(A, lda, r0, m, k, col, c16,
                                                                 g4, Us, X);
    });
  };
  int k = 0;
  if (top[0] & 16) {
    chunk(0, std::integral_constant<int, 2>{});
    k = 16;
  }
  for (; k < m; k += 32) chunk(k, std::integral_constant<int, 4>{});
}

// Trailing-update rows of each wave at K = 1, per number of live row blocks nI: row I holds
// the tiles J = 1..I (row 0: the diagonal band tile), i.e. max(1, ceil(I / TBR)) chunks of TBR
// tiles, and the rows go to the waves longest-first, each to the least-loaded wave (LPT).  The
// fixed snake (w, 15 - w, 16 + w, 31 - w) balanced only nI = 32: as the panels advance, the
// rows >= nI it drops are the long ones of the low waves, and the K = 1 update waited up to 2x
// on its slowest wave (wave 0 idle ~14 % of a cell's cycles at the barrier after the update).
// Which wave updates a tile does not change its arithmetic: the same bits.
constexpr int UPD_RMAX = 8;
constexpr int UPD_NI = BNMAX / BB + 2;
struct UpdRows {
  signed char r[UPD_NI][NWR][UPD_RMAX];
};
constexpr UpdRows make_upd_rows() {
  UpdRows t{};
  for (int nI = 0; nI < UPD_NI; ++nI) {
    int load[NWR] = {}, cnt[NWR] = {};
    for (int w = 0; w < NWR; ++w)
      for (int k = 0; k < UPD_RMAX; ++k) t.r[nI][w][k] = -1;
    for (int I = nI - 1; I >= 0; --I) {
      const int c = I == 0 ? 1 : (I + TBR - 1) / TBR;
      int best = -1;
      for (int w = 0; w < NWR; ++w)
        if (cnt[w] < UPD_RMAX && (best < 0 || load[w] < load[best])) best = w;
      t.r[nI][best][cnt[best]++] = (signed char)I;
      load[best] += c;
    }
  }
  return t;
}
__constant__ UpdRows kUpdRows = make_upd_rows();

template <bool TIMED>
__global__ __launch_bounds__(NTR) void band_coop_kernel(
    const double* __restrict__ SD, int64_t ldS, const double* __restrict__ Sr,
    const RidgeCellDesc* __restrict__ cells, int L, double* __restrict__ work,
    const int* __restrict__ wgmap, unsigned* __restrict__ syncw, long long* __restrict__ tim,
    unsigned spin_max) {
  __shared__ double Vs[BMP][LS];       // V_p (rows >= m zero); the QR WG: panel p+1, V_{p+1}
  __shared__ double Ws[BMP][LS];       // U = V T, then W
  __shared__ double red[NWR][BB * BB]; // QR scratch, canonical sums, update transposes
  __shared__ double Ts[BB][LS];
  __shared__ double taus[BB];
  __shared__ double zts[BB];
  __shared__ int err_s;

  const int code = wgmap[blockIdx.x];
  const int cell = code >> 8, w = (code >> 4) & 15, K = (code & 15) + 1;
  const RidgeCellDesc cd = cells[cell];
  const int n = cd.n;
  const int lda = band_npad(n), nb = lda / BB;
  const int npan = (n - 1) / BB;                 // panels: k0 = 16 p with k0 + 16 < n
  const int t_ = threadIdx.x, lane_ = t_ & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t_ >> 6);
  BandWork bw(work + cd.work, n, L);
  CoopWork cw(bw.F, lda);
  double* __restrict__ A = bw.A;
  CoopSync cs{(gu32*)(syncw + (int64_t)cell * COOP_SYNC),
              (gu32*)(syncw + (int64_t)cell * COOP_SYNC + 1), K, 0u, spin_max};
  const bool qwg = (w == 0);
  const int Ku = K > 1 ? K - 1 : 1;            // update workgroups: all but the QR one
  const int wu = K > 1 ? w - 1 : 0;            // (-1: the QR workgroup when K > 1)
  // 16-byte write-through stores of the matrix tiles through a buffer descriptor on A (a
  // masked store gets an offset past the range and is dropped by the range check)
  const unsigned abytes = (unsigned)lda * (unsigned)lda * 8u;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(A, 0, (int)abytes, 0x00020000);
  auto st2 = [&](unsigned off, bool ok, double x, double y) {
    const double2 v = make_double2(x, y);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsA,
                                           ok ? off : abytes, 0, 16);
  };
  // the hand-off words (V, T, W, partials, z) through a descriptor on the cell's workspace:
  // write-through (sc1) 8-byte buffer stores and sc1 buffer loads (not atomics: a loop's loads
  // are all in flight before the first wait)
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc(A, 0, 0x7ffffff0, 0x00020000);
  auto ldw = [&](const double* p) -> double {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                          rsW, (unsigned)((p - A) * 8), 0, 16));
  };
  auto stw = [&](double* p, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rsW,
                                          (unsigned)((p - A) * 8), 0, 16);
  };
  long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long tlast = 0;
#define COOP_TMARK(ph)                                                   \
  if (TIMED && threadIdx.x == 0) {                                       \
    const long long now = (long long)__builtin_amdgcn_s_memtime();       \
    tacc[ph] += now - tlast;                                             \
    tlast = now;                                                         \
  }
  if (t_ == 0) err_s = 0;

  // ---- A = S * scale (the lower block triangle incl. the diagonal blocks, zero padding),
  //      z = r * scale: row blocks gb = w (mod K)
  {
    const double* S = SD + cd.src;
    const double sc = cd.scale;
    for (int gb = w; gb < nb; gb += K) {
      const int wc = 8 * (gb + 1);                 // column pairs through the diagonal block
      for (int e = t_; e < BB * wc; e += NTR) {
        const int i = 16 * gb + e / wc, j = 2 * (e % wc);
        const double* srow = S + (int64_t)min(i, n - 1) * ldS;
        const double x = (i < n && j < n) ? srow[j] * sc : 0.0;
        const double y = (i < n && j + 1 < n) ? srow[j + 1] * sc : 0.0;
        st2((unsigned)((i * lda + j) * 8), true, x, y);
      }
      if (t_ < BB && 16 * gb + t_ < n) stw(bw.z + 16 * gb + t_, Sr[cd.rsrc + 16 * gb + t_] * sc);
    }
  }
  cs.sync(true, &err_s);
  if (TIMED && threadIdx.x == 0) tlast = (long long)__builtin_amdgcn_s_memtime();

  // ---- panel 0 (the QR workgroup): column block 0, rows 16.., then publish V_0, T_0
  auto publish_vt = [&](int mp) {
    for (int e = t_; e < mp * BB; e += NTR) stw(cw.Vg + e, Vs[e / BB][e % BB]);
    if (t_ < BB * BB) stw(cw.Tg + t_, Ts[t_ / BB][t_ % BB]);
  };
  if (npan > 0 && qwg) {
    const int m0 = n - BB;
    for (int e = t_; e < BMP * BB; e += NTR) {
      const int i = e / BB, c = e % BB;
      Vs[i][c] = (i < m0) ? A[(int64_t)(BB + i) * lda + c] : 0.0;
    }
    __syncthreads();
    band_panel_hh(A, lda, 0, BB, m0, Vs, Ws, &red[0][0], Ts, taus, bw.T, nullptr, Vs);
    if (K > 1) publish_vt(m0);
  }
  if (npan > 0) cs.sync(false, &err_s);
  COOP_TMARK(0)

  for (int p = 0; p < npan; ++p) {
    const int k0 = p * BB, r0 = k0 + BB, m = n - r0;
    const int nI = (m + 15) >> 4;
    int t = t_, lane = lane_;
    asm volatile("" : "+v"(t), "+v"(lane));
    const int c16 = lane & 15, g4 = lane >> 4;
    // ---- B: V_p, T_p (the other workgroups load the published copy), U = V T -> Ws
    if (!qwg) {
      double v[BMP * BB / NTR];
#pragma unroll
      for (int u = 0; u < BMP * BB / NTR; ++u) v[u] = ldw(cw.Vg + min(t + NTR * u, m * BB - 1));
      const double tv = ldw(cw.Tg + (t & (BB * BB - 1)));
#pragma unroll
      for (int u = 0; u < BMP * BB / NTR; ++u) {
        const int e = t + NTR * u, i = e / BB;
        Vs[i][e % BB] = (i < m) ? v[u] : 0.0;
      }
      if (t < BB * BB) Ts[t / BB][t % BB] = tv;
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < BMP / 16 / NWR; ++q) {
      const int i0 = (wid + NWR * q) * 16;
      double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = mfma_f64_16x16x4(Vs[i0 + c16][4 * r + g4], Ts[4 * r + g4][c16], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) Ws[i0 + g4 + 4 * r][c16] = acc[r];
    }
    __syncthreads();
    COOP_TMARK(1)
    // X blocks of this workgroup.  The QR workgroup (w = 0) also factors the next panel and
    // the others also apply the update, so the X blocks are split to balance the two: w = 0
    // takes the last x0 blocks, the K - 1 others the rest round-robin, with x0 from a cost
    // model of one panel calibrated on the MI355X phase timings (tools/bench_ridge.py
    // --timing; cycles: X 197 per block per block row, update 174 per 16 x 16 tile, panel QR
    // 30000 + 550 per block row) - large panels (update-heavy) give w = 0 about half the X
    // blocks, small ones (QR-latency-bound) none.  Which workgroup computes a block does not
    // change its arithmetic, so the betas stay bitwise independent of K.
    int x0 = nI;
    if (K > 1) {
      const float fn = (float)nI;
      const float upd = 174.0f * fn * (fn + 1.0f) * 0.5f, xs = 197.0f * fn;
      const float qr = 30000.0f + 550.0f * fn;
      const float xq = (upd + xs * fn - (float)(K - 1) * qr) / ((float)K * xs);
      x0 = min(nI, max(0, (int)(xq + 0.5f)));
    }
    int blk[4];
    int nq = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = wid + NWR * q;
      blk[q] = qwg ? nI - x0 + k : (w - 1) + (K - 1) * k;
      nq += (qwg ? k < x0 : blk[q] < nI - x0) ? 1 : 0;
    }
    double4_t X[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) X[q] = double4_t{0.0, 0.0, 0.0, 0.0};
    switch (nq) {
      case 1: coop_x_accum<1>(A, lda, r0, m, blk, c16, g4, Ws, X); break;
      case 2: coop_x_accum<2>(A, lda, r0, m, blk, c16, g4, Ws, X); break;
      case 3: coop_x_accum<3>(A, lda, r0, m, blk, c16, g4, Ws, X); break;
      case 4: coop_x_accum<4>(A, lda, r0, m, blk, c16, g4, Ws, X); break;
      default: break;
    }
    // per-block partials V_I' X_I and V_I' z_I (z as column 0 of the B operand).  With one
    // workgroup per cell (K = 1) they stay on the CU: U is dead once every wave's X is done, so
    // they go to the LDS of Ws (32 blocks x 272 doubles = exactly its 512 x 17), and W later
    // straight to Ws - no global round trip of partials and W per panel.  (Same values, same
    // summation order: bitwise the same betas as K > 1.)
    double* const Pl = &Ws[0][0];
    if (K == 1) __syncthreads();                   // every wave's reads of U are done
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < nq) {
        const int i0 = 16 * blk[q];
        double4_t Pp = {0.0, 0.0, 0.0, 0.0}, Pz = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i0 + 4 * r + g4;
          const double va = Vs[row][c16];
          Pp = mfma_f64_16x16x4(va, X[q][r], Pp);
          const double zl = ldw(bw.z + r0 + min(row, m - 1));
          const double zb = (c16 == 0 && row < m) ? zl : 0.0;
          Pz = mfma_f64_16x16x4(va, zb, Pz);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (K == 1) {
            Pl[blk[q] * (BB * BB + BB) + (g4 + 4 * r) * BB + c16] = Pp[r];
            if (c16 == 0) Pl[blk[q] * (BB * BB + BB) + BB * BB + g4 + 4 * r] = Pz[r];
          } else {
            stw(cw.Pg + (int64_t)blk[q] * (BB * BB) + (g4 + 4 * r) * BB + c16, Pp[r]);
            if (c16 == 0) stw(cw.Pzg + blk[q] * BB + g4 + 4 * r, Pz[r]);
          }
        }
      }
    }
    COOP_TMARK(2)
    cs.sync(false, &err_s);
    COOP_TMARK(3)
    // ---- C: canonical sums (block order), M = T' P, z and W of the X blocks
    if (t < BB * BB + BB) {
      // (all nI partials in flight, then summed in block order)
      const bool isP = t < BB * BB;
      constexpr int NB = BNMAX / BB;
      double v[NB];
      if (K == 1) {
#pragma unroll
        for (int I = 0; I < NB; ++I) v[I] = Pl[min(I, nI - 1) * (BB * BB + BB) + t];
      } else {
        const double* base = isP ? cw.Pg + t : cw.Pzg + (t - BB * BB);
        const int stride = isP ? BB * BB : BB;
#pragma unroll
        for (int I = 0; I < NB; ++I) v[I] = ldw(base + min(I, nI - 1) * stride);
      }
      double s = 0.0;
#pragma unroll
      for (int I = 0; I < NB; ++I) s = (I < nI) ? s + v[I] : s;
      if (isP) red[0][t] = s;
      else red[1][t - BB * BB] = s;
    }
    __syncthreads();
    if (t < BB) {
      double s = 0.0;
      for (int a = 0; a <= t; ++a) s = fma(Ts[a][t], red[1][a], s);
      zts[t] = s;
    }
    double4_t Mm = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r)
      Mm = mfma_f64_16x16x4(Ts[4 * r + g4][c16], red[0][(4 * r + g4) * BB + c16], Mm);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < nq) {
        const int i0 = 16 * blk[q];
        if (lane < BB && i0 + lane < m) {
          const int i = i0 + lane;
          double s = 0.0;
#pragma unroll
          for (int c = 0; c < BB; ++c) s = fma(Vs[i][c], zts[c], s);
          stw(bw.z + r0 + i, ldw(bw.z + r0 + i) - s);
        }
        double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = mfma_f64_16x16x4(Vs[i0 + c16][4 * r + g4], Mm[r], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + g4 + 4 * r;
          const double wv = (i < m) ? X[q][r] - 0.5 * acc[r] : 0.0;
          if (K == 1) Ws[i][c16] = wv;               // (the partials were read before the
          else stw(cw.Wg + i * BB + c16, wv);        // barriers above)
        }
      }
    }
    COOP_TMARK(4)
    cs.sync(false, &err_s);
    COOP_TMARK(3)
    // ---- D: W -> Ws (K = 1: already there); update (update workgroups) / look-ahead panel
    //      p+1 (QR workgroup)
    if (K > 1) {
      double v[BMP * BB / NTR];
#pragma unroll
      for (int u = 0; u < BMP * BB / NTR; ++u) v[u] = ldw(cw.Wg + min(t + NTR * u, nI * BB * BB - 1));
#pragma unroll
      for (int u = 0; u < BMP * BB / NTR; ++u) {
        const int e = t + NTR * u;
        if (e < nI * BB * BB) Ws[e / BB][e % BB] = v[u];
      }
    }
    __syncthreads();
    auto update = [&]() {
      // rows I = first_u + pos Ku (pos: snake over the waves), tiles J = (I ? 1 : 0) .. I,
      // TBR tiles per chunk, next chunk's tiles loaded before this chunk's MFMAs (the
      // one-workgroup kernel's trailing loop; stores through the buffer descriptor)
      const int first_u = ((wu - (p + 1)) % Ku + Ku) % Ku;
      // this workgroup's rows first_u + u Ku (u < nu) go to its waves by the LPT table of nu
      // rows (kUpdRows: K = 1 exactly; K > 1 the costs ceil((first_u + u Ku) / TBR) grow
      // linearly in u as the table's do).  A row >= nI ends the wave's list.
      constexpr int RR = UPD_RMAX;
      const int nu = (first_u < nI) ? (nI - first_u + Ku - 1) / Ku : 0;
      auto row_of = [&](int rr) {
        const int r = (rr < UPD_RMAX) ? (int)kUpdRows.r[nu][wid][rr] : -1;
        return r < 0 ? nI : first_u + r * Ku;
      };
      double4_t nxt[TBR];
      auto fetch = [&](int I, int J0) {
#pragma unroll
        for (int u = 0; u < TBR; ++u) {
          const int J = J0 + u;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * I + g4 + 4 * r, jj = 16 * J + c16;
            nxt[u][r] = A[(int64_t)(r0 + min(i, m - 1)) * lda + r0 + min(jj, m - 1)];
          }
        }
      };
      int rr = 0, I = row_of(0);
      while (rr < RR && I >= nI) I = row_of(++rr);
      if (rr >= RR) I = nI;
      int J0 = (I == 0) ? 0 : 1;
      auto advance = [&]() {
        J0 += TBR;
        if (J0 > I) {
          do I = row_of(++rr);
          while (rr < RR && I >= nI);
          if (rr >= RR) I = nI;
          J0 = (I == 0) ? 0 : 1;
        }
      };
      fetch(I, J0);
      double* tw = &red[0][0] + wid * (BB * BB);
      double4_t acc[TBR];
#pragma unroll
      for (int u = 0; u < TBR; ++u) acc[u] = nxt[u];
#pragma unroll
      for (int u = 0; u < TBR; ++u) asm volatile("" ::"v"(acc[u]));
      int ci = I, cj = J0;
      advance();
      while (ci < nI) {
        fetch(I, J0);
        double aV[4], aW[4], bW[TBR][4], bV[TBR][4];
        const int ia = 16 * ci + c16;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          aV[s] = -Vs[ia][4 * s + g4];
          aW[s] = -Ws[ia][4 * s + g4];
        }
#pragma unroll
        for (int u = 0; u < TBR; ++u) {
          const int jb = 16 * min(cj + u, ci) + c16;
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            bW[u][s] = Ws[jb][4 * s + g4];
            bV[u][s] = Vs[jb][4 * s + g4];
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int u = 0; u < TBR; ++u) acc[u] = mfma_f64_16x16x4(aV[s], bW[u][s], acc[u]);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int u = 0; u < TBR; ++u) acc[u] = mfma_f64_16x16x4(aW[s], bV[u][s], acc[u]);
#pragma unroll
        for (int u = 0; u < TBR; ++u) {
          const int J = cj + u;
          const bool live = J <= ci;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = g4 + 4 * r;
            tw[row * BB + (c16 ^ (row & ~1))] = acc[u][r];
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          {
            const int pr = lane >> 3, pc = 2 * (lane & 7);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int row = pr + 8 * h;
              const double2 v = *reinterpret_cast<const double2*>(&tw[row * BB + (pc ^ (row & ~1))]);
              st2((unsigned)(((r0 + 16 * ci + row) * lda + r0 + 16 * J + pc) * 8), live, v.x, v.y);
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#pragma unroll
        for (int u = 0; u < TBR; ++u) asm volatile("" ::"v"(acc[u]));
#pragma unroll
        for (int u = 0; u < TBR; ++u) acc[u] = nxt[u];
        ci = I;
        cj = J0;
        advance();
      }
    };
    // the old tiles (I, 0) of the look-ahead panel, loaded before the update's stores are
    // issued (a load behind write-through stores waits for them: one vmcnt counter)
    double4_t pt[4];
    auto lookahead_load = [&]() {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int I = 1 + wid + NWR * q;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          pt[q][r] = A[(int64_t)(r0 + min(16 * min(I, nI - 1) + g4 + 4 * r, m - 1)) * lda + r0 + c16];
      }
    };
    auto lookahead = [&]() {
      // panel p+1 = tiles (I, 0), I >= 1, of A22 after update p (computed here, never stored
      // by the update), into Vs rows 16 (I - 1) .., then its QR (V_{p+1} -> Vs, T -> Ts)
      const int m1 = m - BB;
      double bW0[4], bV0[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bW0[s] = Ws[c16][4 * s + g4];
        bV0[s] = Vs[c16][4 * s + g4];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int I = 1 + wid + NWR * q;
        if (I < nI) {
          double aV[4], aW[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            aV[s] = -Vs[16 * I + c16][4 * s + g4];
            aW[s] = -Ws[16 * I + c16][4 * s + g4];
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) pt[q] = mfma_f64_16x16x4(aV[s], bW0[s], pt[q]);
#pragma unroll
          for (int s = 0; s < 4; ++s) pt[q] = mfma_f64_16x16x4(aW[s], bV0[s], pt[q]);
        }
      }
      __syncthreads();                             // every V_p / W_p read is done
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int I = 1 + wid + NWR * q;
        if (I < nI) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * I + g4 + 4 * r;     // A22 row; panel row i - 16
            Vs[i - BB][c16] = (i < m) ? pt[q][r] : 0.0;
          }
        }
      }
      for (int e = t + 16 * (nI - 1) * BB; e < BMP * BB; e += NTR) Vs[e / BB][e % BB] = 0.0;
      __syncthreads();
      band_panel_hh(A, lda, k0 + BB, r0 + BB, m1, Vs, Ws, &red[0][0], Ts, taus,
                    bw.T + (int64_t)(p + 1) * BB * BB, nullptr, Vs);
      if (K > 1) publish_vt(m1);
    };
    if (K == 1) {
      if (p + 1 < npan) lookahead_load();
      update();
      COOP_TMARK(5)
      __syncthreads();
      COOP_TMARK(3)                                  // (timing: wave 0 waiting for the update)
      if (p + 1 < npan) lookahead();
      COOP_TMARK(6)
    } else if (qwg) {
      if (p + 1 < npan) {
        lookahead_load();
        lookahead();
      }
      COOP_TMARK(6)
    } else {
      update();
      COOP_TMARK(5)
    }
    cs.sync(true, &err_s);
    COOP_TMARK(7)
  }
  if (TIMED && threadIdx.x == 0 && w < 2)
    for (int q = 0; q < 8; ++q) tim[(int64_t)cell * 16 + w * 8 + q] = tacc[q];
#undef COOP_TMARK
  // ---- row-major lower band (the QR workgroup: it wrote the R blocks itself)
  if (qwg) {
    for (int e = t_; e < n * LS; e += NTR) {
      const int r = e / LS, c = r - BB + e % LS;
      bw.LB[e] = (c >= 0) ? A[(int64_t)r * lda + c] : 0.0;
    }
  }
}

// ---------------------------------------------------------------------------------------
// kernel 2: banded Cholesky solves, 4 lambdas per wave (one 16-lane DPP row each).
//
// Lane p of a row holds the band row r (r = p mod 16) of the 16-row window j+1..j+16 (the
// retiring pivot lane takes row j+16 in the same step), columns j..j+16 in 17 registers
// (slot k <-> column j+k, shifted one slot per step).  Every cross-lane value is a
// row_newbcast DPP move, and 4 independent solves share each instruction.  The entering rows
// (the same for the workgroup's 16 lambdas) are staged in LDS one block ahead and read by the
// pivot lane straight into its window (exec-masked ds_reads in flight during the pivot's rsq
// chain; measured 543 / 860 us vs 593 / 928 us for the big / small cells of the headline step
// with a 17-register row prefetch and VALU moves).  Slots right of a row's diagonal hold
// garbage that is never read.
// ---------------------------------------------------------------------------------------
constexpr int NTS = 256;      // 4 waves x 4 rows = 16 lambdas per workgroup

// 158 VGPRs: 3 waves per SIMD (the entering rows come from LDS, not a register prefetch).
__global__ __launch_bounds__(NTS, 3) void ridge_band_solve_kernel(
    const RidgeCellDesc* __restrict__ cells, const double* __restrict__ lvec, int L,
    double* __restrict__ work, long long* __restrict__ tim, int ncells,
    int* __restrict__ lu_count) {
  const long long t_start = (long long)__builtin_amdgcn_s_memtime();
  // the repair list count of kernel 2b starts at zero (no separate fill launch)
  if (lu_count != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *lu_count = 0;
  const int nb = (L + 15) / 16;
  const int cell = blockIdx.x / nb;
  const RidgeCellDesc cd = cells[cell];
  const int n = cd.n;
  const int p = threadIdx.x & 15;
  const int l = (blockIdx.x % nb) * 16 + (threadIdx.x >> 4);
  const bool lv = l < L;
  const int lc = lv ? l : L - 1;                 // padding rows redo the last lambda
  BandWork bw(work + cd.work, n, L);
  const double lam = lvec[lc];
  double* Lrow = bw.Lf + (int64_t)lc * n * BB;   // row j: l_{j+1..j+16, j}
  double* Linv = bw.Lf + (int64_t)L * n * BB + (int64_t)lc * n;
  double* yl = bw.Yt + (int64_t)lc * n;
  const double* LB = bw.LB;                      // row-major band: LB[r][s] = B[r][r-16+s]
  const double* z = bw.z;

  // w: 32 slots; within a 16-step block at phase u, slot u + k <-> column j + k (k <= 16), so
  // the window never shifts inside a block (one 16-slot move per block).  Rows >= n are
  // identity rows, so every block is a full, branch-free 16 steps.  The band rows entering
  // during a block are the same for all 16 lambdas of the workgroup: they are staged in LDS one
  // block ahead (double buffer, one barrier per block) and each lane reads its row at the
  // block start, instead of a second 17-register prefetch per lane (occupancy: VGPRs).
  __shared__ double LBs[2][BB][LS];
  // LDS byte offset of LBs (the low word of its flat address)
  const unsigned lbs_base = (unsigned)reinterpret_cast<uintptr_t>(&LBs[0][0][0]);
  const int npad = (n + 15) & ~15;
  double w[2 * BB];
  auto stage_rows = [&](int r0s, int buf) {       // rows r0s .. r0s + 15 -> LBs[buf]
    for (int e = threadIdx.x; e < BB * LS; e += NTS) {
      const int r = r0s + e / LS, s = e % LS;
      LBs[buf][e / LS][s] = (r < n) ? LB[(int64_t)r * LS + s] : (s == BB ? 1.0 : 0.0);
    }
  };
  // the same in two halves: the global loads at a block's start into two registers per thread
  // (BB * LS = 272 <= 2 NTS), the LDS stores at its end, so the loads' latency is spent under
  // the block's 16 steps instead of in front of them
  static_assert(BB * LS <= 2 * NTS, "two staged doubles per thread");
  double st[2];
  auto load_rows = [&](int r0s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = threadIdx.x + h * NTS;
      const int r = r0s + e / LS, s = e % LS;
      st[h] = (e < BB * LS && r < n) ? LB[(int64_t)r * LS + s] : (s == BB ? 1.0 : 0.0);
    }
  };
  auto store_rows = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = threadIdx.x + h * NTS;
      if (e < BB * LS) LBs[buf][e / LS][e % LS] = st[h];
    }
  };
  // window at j = 0: lane p holds row p, slot k <-> column k
#pragma unroll
  for (int k = 0; k < 2 * BB; ++k)
    w[k] = (k <= p && p < n) ? LB[(int64_t)p * LS + BB - p + k] + (k == p ? lam : 0.0)
                             : (k == p ? 1.0 : 0.0);
  double zr = (p < n) ? z[p] : 0.0;
  stage_rows(BB, 0);                               // block 0's entering rows 16..31
  double znx = (p + BB < n) ? z[p + BB] : 0.0;
  bool ok = true;
  __syncthreads();

  // every prologue load (window, z) done here: otherwise the compiler's wait for the first
  // in-loop use of zr is a vmcnt(0) at the top of EVERY block, which also drains the block's
  // own staging loads issued just before it
  __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0)
  // One 16-step block.  CHECK (the last block only): rows >= n are identity rows and store
  // nothing.  Elsewhere the stores need no condition: a padding lane (lambda >= L) redoes
  // lambda L-1 bit for bit, so its stores repeat the same values; 1 / l_jj and y_j are kept by
  // the pivot lane and stored once per block (16 lanes, one line) instead of per step.
  auto fwd_block = [&](int j0, auto CHECK) {
    constexpr bool chk = decltype(CHECK)::value;
    const int sb = (j0 >> 4) & 1;
    // this block's entering row for lane p (row j0 + 16 + p, taken at step p), then the NEXT
    // block's rows to the other buffer
    const double lam_in = (j0 + BB + p < n) ? lam : 0.0;   // diagonal shift of the entering row
    load_rows(j0 + 2 * BB);                        // -> LBs[sb ^ 1] at the block's end
    const double znx2 = (j0 + 2 * BB + p < n) ? z[j0 + 2 * BB + p] : 0.0;
    double myinv = 0.0, myy = 0.0;
    static_for<0, 16>([&](auto U) {
      constexpr int u = decltype(U)::value;
      const int j = j0 + u;
      const bool pl = (p == u);                  // pivot lane: holds row j, takes row j+16
      double piv = row_bcast<u>(w[u]);
      const double zpiv = row_bcast<u>(zr);      // (read before the pivot lane's zr changes)
      // LDS reads straight into the pivot lane's window, in flight during the pivot's rsq chain
      lds_row_issue<u>(w, lbs_base + (unsigned)(sb * BB * LS + u * LS) * 8u, piv);
      ok = ok && (piv > 0.0);
      double inv = rsqrt1_f64(piv);
      lds_row_wait<u>(w, inv);
      const double yj = zpiv * inv;
      if (pl) {
        w[u + BB] += lam_in;
        zr = znx;
        myinv = inv;
        myy = yj;
      }
      const double lval = w[u] * inv;            // l_i, i = (p - u) mod 16, pivot lane: i = 16
      if (!chk || j < n) Lrow[(int64_t)j * BB + (pl ? BB - 1 : ((p - u) & 15) - 1)] = lval;
      zr -= lval * yj;
      static_for<1, LS>([&](auto K) {
        constexpr int k = decltype(K)::value;
        fnmac_bcast<(u + k) & 15, k == 1>(w[u + k], lval, lval);   // w -= l_k * l_i
      });
    });
    if (!chk || j0 + p < n) {
      Linv[j0 + p] = myinv;
      yl[j0 + p] = myy;
    }
#pragma unroll
    for (int s = 0; s < BB; ++s) w[s] = w[s + BB];
    znx = znx2;
    store_rows(sb ^ 1);
    __syncthreads();                               // next block's rows staged; this buffer free
  };
  for (int j0 = 0; j0 < npad - 16; j0 += 16) fwd_block(j0, std::false_type{});
  fwd_block(npad - 16, std::true_type{});
  // back substitution L^T x = y, x overwrites y.  Lane (j+i) mod 16 holds x_{j+i} (xr); every
  // lane also holds the last two x (x1 = x_{j+1}, x2 = x_{j+2}).  Step j only waits on
  //     x_j = ((y_j - P_j) - l_{j+2,j} x2 - l_{j+1,j} x1) / l_jj,
  // P_j = sum_{i=3..16} l_{j+i,j} x_{j+i} being reduced over the row two steps earlier (its x
  // are all known then), so the 16-lane sum is off the step-to-step chain (two fmas and a mul
  // on it instead of a product, four DPP add levels, a subtract and a mul).  The factor data of
  // a block's 16 steps come in two halves of 8, each loaded one half ahead.
  __syncthreads();
  const long long t_mid = (long long)__builtin_amdgcn_s_memtime();
  struct Half {
    double pl[8], iv[8], yv[8];
  };
  // step s of the block at jb: j = jb - s, u = j & 15 = 15 - s; lane p's factor entry
  // l_{j+i,j}, i = (p - u) & 15 (0 -> 16).  CHECK (the first block only): rows >= n are
  // identity rows (l = 0, 1 / l_jj = 1, y = 0).  Elsewhere every row is < n and the loads are
  // branch-free (a row < 0, prefetched past the end, is clamped and never used): with a branch
  // per load the compiler waited for ALL loads (the prefetch included) at the first use.
  auto load_half = [&](int jb, auto S0, auto CHECK, Half& h) {
    constexpr int s0 = decltype(S0)::value;
    static_for<0, 8>([&](auto V) {
      constexpr int v = decltype(V)::value;
      constexpr int u = 15 - s0 - v;
      const int j = jb - s0 - v;
      const int i = (p - u) & 15;
      if constexpr (decltype(CHECK)::value) {
        const bool in = j < n;
        h.pl[v] = in ? Lrow[(int64_t)j * BB + (i == 0 ? BB - 1 : i - 1)] : 0.0;
        h.iv[v] = in ? Linv[j] : 1.0;
        h.yv[v] = in ? yl[j] : 0.0;
      } else {
        const int jc = max(j, 0);
        h.pl[v] = Lrow[(int64_t)jc * BB + (i == 0 ? BB - 1 : i - 1)];
        h.iv[v] = Linv[jc];
        h.yv[v] = yl[jc];
      }
    });
  };
  double xr = 0.0, x1 = 0.0, x2 = 0.0;
  double Pq[2] = {0.0, 0.0}, L1q[2] = {0.0, 0.0}, L2q[2] = {0.0, 0.0};
  // the row of step s + 2 (phase u' = u - 2, factor entries pl): its P from xr before step s's
  // update, its two critical coefficients broadcast from lanes u' + 1, u' + 2
  auto prep = [&](auto UP, double pl) {
    constexpr int up = decltype(UP)::value & 15;
    const int i = (p - up) & 15;
    const double pm = (i == 1 || i == 2) ? 0.0 : pl;
    Pq[0] = Pq[1];
    L1q[0] = L1q[1];
    L2q[0] = L2q[1];
    Pq[1] = row16_sum(pm * xr);
    L1q[1] = row_bcast<(up + 1) & 15>(pl);
    L2q[1] = row_bcast<(up + 2) & 15>(pl);
  };
  auto step = [&](double yv, double iv) {
    const double t = fma(-L2q[0], x2, yv - Pq[0]);
    const double xj = fma(-L1q[0], x1, t) * iv;
    x2 = x1;
    x1 = xj;
    return xj;
  };
  auto store_half = [&](int jb, int s0) {   // lanes u of the half hold their x in xr
    const int j = jb - (15 - p);
    if (lv && j < n && 15 - p >= s0 && 15 - p < s0 + 8) yl[j] = ok ? xr : __builtin_nan("");
  };
  using I0 = std::integral_constant<int, 0>;
  using I8 = std::integral_constant<int, 8>;
  Half A, B;
  load_half(npad - 1, I0{}, std::true_type{}, A);
  // the first two rows' P, l (rows >= n: zero factor, so zero from xr = 0 anyway)
  {
    Pq[1] = 0.0;
    L1q[1] = row_bcast<0>(A.pl[0]);   // u = 15: lanes 0, 1
    L2q[1] = row_bcast<1>(A.pl[0]);
    Pq[0] = Pq[1]; L1q[0] = L1q[1]; L2q[0] = L2q[1];
    Pq[1] = 0.0;
    L1q[1] = row_bcast<15>(A.pl[1]);  // u = 14: lanes 15, 0
    L2q[1] = row_bcast<0>(A.pl[1]);
  }
  auto block = [&](int jb, auto FIRST) {
    load_half(jb, I8{}, FIRST, B);
    static_for<0, 8>([&](auto V) {
      constexpr int v = decltype(V)::value;
      constexpr int u = 15 - v;
      const double xj = step(A.yv[v], A.iv[v]);
      if constexpr (v + 2 < 8) prep(std::integral_constant<int, u - 2>{}, A.pl[v + 2]);
      else prep(std::integral_constant<int, u - 2>{}, B.pl[v - 6]);
      xr = (p == u) ? xj : xr;
    });
    store_half(jb, 0);
    load_half(jb - 16, I0{}, std::false_type{}, A);
    static_for<0, 8>([&](auto V) {
      constexpr int v = decltype(V)::value;
      constexpr int u = 7 - v;
      const double xj = step(B.yv[v], B.iv[v]);
      if constexpr (v + 2 < 8) prep(std::integral_constant<int, u - 2 + 16>{}, B.pl[v + 2]);
      else prep(std::integral_constant<int, u - 2 + 16>{}, A.pl[v - 6]);
      xr = (p == u) ? xj : xr;
    });
    store_half(jb, 8);
  };
  block(npad - 1, std::true_type{});
  for (int jb = npad - 17; jb >= 0; jb -= 16) block(jb, std::false_type{});
  if (tim != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {   // debug: wave 0 of block 0
    const long long t_end = (long long)__builtin_amdgcn_s_memtime();
    tim[(int64_t)ncells * 8 + 0] = t_mid - t_start;
    tim[(int64_t)ncells * 8 + 1] = t_end - t_mid;
  }
}

// ---------------------------------------------------------------------------------------
// kernel 2b: the lambdas whose banded Cholesky failed (Dbar + l I not numerically SPD: l = 0
// on a rank-deficient Dbar, PFML_Search_Coef.py:131-133 / General_functions.py:81) are
// re-solved IN THE BAND DOMAIN by LU with partial pivoting (the LAPACK dgbtf2 pivot order) on
// (B + l I) y = z, before the back-transform turns y into beta = Q y.  Q is orthogonal, so this
// is a backward-stable solve of (Dbar + l I) beta = rbar, the system np.linalg.solve sees, at
// O(n BB^2) per system instead of the O(n^3) dense pivoted LU it replaces.
//
//   band_lu_flag_kernel  one thread per (cell, lambda): a NaN-marked y appends it to a list
//   ridge_band_lu_kernel LU_WG one-wave workgroups walk the list.  Window of the 17 live rows
//                        (slot = row mod 17) x 33 columns (slot = column mod 33: with
//                        pivoting U has upper bandwidth 2 BB) in LDS; the pivot row goes to
//                        an LDS copy of U, then 16 x 32 lanes eliminate and the row 17 below
//                        enters the freed slot (its loads issued two steps ahead).  Back substitution from LDS, y written back.
//                        An exactly zero pivot (singular: the reference raises LinAlgError)
//                        leaves the NaN.
// ---------------------------------------------------------------------------------------
constexpr int LR = BB + 1;          // live rows of the pivoting window
constexpr int UW = 2 * BB + 1;      // U row width (upper bandwidth 2 BB after pivoting)
constexpr int LU_WG = 128;

__global__ __launch_bounds__(256) void band_lu_flag_kernel(const RidgeCellDesc* __restrict__ cells,
                                                           int ncells, int L,
                                                           double* __restrict__ work,
                                                           int* __restrict__ list,
                                                           int* __restrict__ count, int cap) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ncells * L) return;
  const int c = e / L, l = e % L;
  const RidgeCellDesc cd = cells[c];
  const BandWork bw(work + cd.work, cd.n, L);
  const double y0 = bw.Yt[(int64_t)l * cd.n];
  if (y0 != y0) {
    const int slot = atomicAdd(count, 1);
    if (slot < cap) list[slot] = e;
  }
}

__global__ __launch_bounds__(64) void ridge_band_lu_kernel(
    const RidgeCellDesc* __restrict__ cells, const double* __restrict__ lvec, int L,
    double* __restrict__ work, const int* __restrict__ list, const int* __restrict__ count,
    int cap) {
  __shared__ double Us[BNMAX][UW];    // U rows: Us[k][c] = U[k][k + c]
  __shared__ double ys[BNMAX];        // L^-1 z, then y
  __shared__ double W[LR][UW];        // live rows k..k+16, columns k..k+32 (both mod-indexed)
  __shared__ double Z[LR];
  const int total = min(*count, cap);
  const int lane = threadIdx.x;
  for (int q = blockIdx.x; q < total; q += gridDim.x) {
    const int e = list[q];
    const RidgeCellDesc cd = cells[e / L];
    const int l = e % L, n = cd.n;
    BandWork bw(work + cd.work, n, L);
    const double lam = lvec[l];
    const double* __restrict__ LB = bw.LB;
    // B(r, c) + lam delta_rc for |r - c| <= BB (symmetric band, lower half stored)
    auto band = [&](int r, int c) -> double {
      if (r >= n || c >= n || c < 0 || abs(r - c) > BB) return 0.0;
      const int hi = max(r, c), lo = min(r, c);
      return LB[(int64_t)hi * LS + lo - hi + BB] + (r == c ? lam : 0.0);
    };
    for (int x = lane; x < LR * UW; x += 64) W[x / UW][x % UW] = band(x / UW, x % UW);
    if (lane < LR) Z[lane] = lane < n ? bw.z[lane] : 0.0;
    __syncthreads();
    // entering rows prefetched two steps ahead (their global loads overlap two steps of
    // elimination instead of stalling each step): the k loop is unrolled by two with one
    // register pair per parity, loads are unconditional (clamped) and the masks are applied
    // where the values are used - a select right after a load, a load under a branch or a
    // register copy would each wait for the load at once
    auto fetch = [&](int k, double& ev, double& zv) {
      const int r = k + LR, c = k + 1 + lane;
      const int hi = max(r, c), lo = min(r, c);
      ev = LB[(int64_t)min(hi, n - 1) * LS + max(0, min(BB, lo - hi + BB))];
      zv = bw.z[min(r, n - 1)];
    };
    // one elimination step; false on an exactly zero / NaN pivot
    auto step = [&](int k, double& ev, double& zv) -> bool {
      const int ks = k % LR, kc = k % UW;
      // pivot: first max |W[k + i][k]|, i = 0..16 (idamax order)
      double a = (lane < LR && k + lane < n) ? fabs(W[(k + lane) % LR][kc]) : -1.0;
      int ia = lane;
#pragma unroll
      for (int off = 16; off > 0; off >>= 1) {
        const double oa = __shfl_xor(a, off, 32);
        const int oi = __shfl_xor(ia, off, 32);
        if (oa > a || (oa == a && oi < ia)) { a = oa; ia = oi; }
      }
      const int ip = __shfl(ia, 0);
      if (ip != 0) {
        const int ps = (k + ip) % LR;
        if (lane < UW) {
          const double t0 = W[ks][lane];
          W[ks][lane] = W[ps][lane];
          W[ps][lane] = t0;
        }
        if (lane == 0) {
          const double t0 = Z[ks];
          Z[ks] = Z[ps];
          Z[ps] = t0;
        }
      }
      __syncthreads();
      const double piv = W[ks][kc];
      if (piv == 0.0 || piv != piv) return false;
      const double rp = 1.0 / piv;
      const double zk = Z[ks];
      if (lane < UW) Us[k][lane] = W[ks][(k + lane) % UW];
      if (lane == 0) ys[k] = zk;
      // eliminate rows k+1..k+16, columns k+1..k+32: lane -> column 1 + (lane & 31), rows
      // 1 + (lane >> 5) + 2 t
      const int c = 1 + (lane & 31);
      const double uc = W[ks][(k + c) % UW];
      double zm = 0.0;
      if (lane < BB && k + 1 + lane < n) zm = W[(k + 1 + lane) % LR][kc] * rp;
#pragma unroll
      for (int t = 0; t < BB / 2; ++t) {
        const int i = 1 + (lane >> 5) + 2 * t;
        if (k + i < n) {
          const int rs = (k + i) % LR;
          const double m = W[rs][kc] * rp;
          W[rs][(k + c) % UW] -= m * uc;
        }
      }
      if (lane < BB && k + 1 + lane < n) Z[(k + 1 + lane) % LR] -= zm * zk;
      __syncthreads();
      // row k + 17 enters the pivot row's slot (columns k+1 .. k+33); the other rows' column
      // k slot becomes column k + 33, zero for them
      const int r = k + LR, col = k + 1 + lane;
      if (lane < UW)
        W[ks][col % UW] = (r < n && col < n) ? ev + (r == col ? lam : 0.0) : 0.0;
      if (lane < BB) W[(k + 1 + lane) % LR][kc] = 0.0;
      if (lane == 0) Z[ks] = r < n ? zv : 0.0;
      fetch(k + 2, ev, zv);
      __syncthreads();
      return true;
    };
    double eA, zA, eB, zB;
    fetch(0, eA, zA);
    fetch(1, eB, zB);
    bool singular = false;
    for (int k = 0; k < n; k += 2) {
      if (!step(k, eA, zA)) { singular = true; break; }
      if (k + 1 < n && !step(k + 1, eB, zB)) { singular = true; break; }
    }
    if (!singular) {
      for (int k = n - 1; k >= 0; --k) {
        double s = (lane >= 1 && lane < UW && k + lane < n) ? Us[k][lane] * ys[k + lane] : 0.0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) ys[k] = (ys[k] - s) / Us[k][0];
        __syncthreads();
      }
      double* __restrict__ yl = bw.Yt + (int64_t)l * n;
      for (int j = lane; j < n; j += 64) yl[j] = ys[j];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// kernel 3: beta = Q y, blocked WY, one workgroup per (cell, chunk of LC = 16 lambdas).
//
// The chunk's Y (n x 16) lives in REGISTERS: wave w owns the 16-row blocks b = w + 8 q, one
// double4 per block in the MFMA C layout (row 16 b + g4 + 4 r, lambda c16) - which is also
// the B-operand layout of P = V^T Y, so Y never round-trips through LDS.  Per panel
// (backwards) each wave holds V_p of its live blocks (b > p) in A-operand order, loaded one
// panel AHEAD (the loads of panel p-1 are in flight while panel p computes); the 8 partial P
// meet in LDS (ping-pong buffers: one barrier per panel), every wave forms M = T P itself,
// re-reads its V blocks transposed through a wave-private LDS image (no barrier) and updates
// Y_b -= V_b M.
// ---------------------------------------------------------------------------------------
// Row-block capacity per wave of the production shape (n <= BNMAX, 8 waves).  Cells of small n
// take narrower instances (NWT waves x NBT blocks, ridge_band_bt_launch): their LDS (the
// wave-private V images and the partial-P ping-pong) shrinks with the instance, so two or three
// workgroups share a CU instead of one, and fewer waves idle (n = 65 has 5 row blocks).
constexpr int NBW = (BNMAX / 16 + NWB - 1) / NWB;   // row blocks per wave

template <int NWT, int NBT>
__global__ __launch_bounds__(NWT * 64) void ridge_band_backtransform_kernel(
    const RidgeCellDesc* __restrict__ cells, int cell0, int ncells, int L, double* __restrict__ work,
    double* __restrict__ beta_out, int64_t ldo, const unsigned* __restrict__ syncw) {
  __shared__ double red[2][NWT][BB * BB];
  __shared__ double Vw[NWT][NBT][BB][LS];         // wave-private V_b images (transpose)
  // (the chunks of a cell are adjacent in dispatch order, so they run together and share
  // the cell's V panels through the caches; an XCD-grouped order measured slower)
  const int nch = (L + LC - 1) / LC;
  if ((int)blockIdx.x >= ncells * nch) return;
  const int cell = cell0 + (int)blockIdx.x / nch, ch = blockIdx.x % nch;
  const RidgeCellDesc cd = cells[cell];
  const int n = cd.n;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, g4 = lane >> 4;
  BandWork bw(work + cd.work, n, L);
  const double* __restrict__ A = bw.A;
  const int l0 = ch * LC;
  const bool lok = c16 < min(LC, L - l0);
  const int nb = (n + 15) >> 4;
  const double* __restrict__ yc = bw.Yt + (int64_t)(l0 + (lok ? c16 : 0)) * n;
  {   // padding columns [n, ldo) of this chunk's lambda rows are zero (no fill by the caller)
    const int lc = min(LC, L - l0), pad = (int)(ldo - n);
    double* __restrict__ o = beta_out + cd.out + (int64_t)l0 * ldo + n;
    for (int e = threadIdx.x; e < lc * pad; e += NWT * 64) o[(int64_t)(e / pad) * ldo + e % pad] = 0.0;
  }
  // a cell whose cooperative reduction timed out (its error word, CoopSync) gets NaN betas:
  // the grid search's non-finite-cell recovery then recomputes it (never silent garbage)
  const bool failed = syncw != nullptr && syncw[(int64_t)cell * COOP_SYNC + 1] != 0u;
  double4_t Y[NBT];
#pragma unroll
  for (int q = 0; q < NBT; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * (wid + NWT * q) + g4 + 4 * r;
      Y[q][r] = (lok && i < n) ? (failed ? __builtin_nan("") : yc[i]) : 0.0;
    }
  // va[q][r] = V_p[16 b - r0 + 4 r + g4][c16] for the live blocks b = wid + 8 q of panel p
  const int lda = band_npad(n);                   // A's leading dimension (padded)
  double vn[NBT][4], tn[4];
  // Branch-free loads (the row clamped into the panel: dead blocks and rows past m read a
  // valid, cached element) and the unit-lower-triangular mask applied where the panel is
  // used: with the loads under conditions and the mask right after them, the compiler waited
  // for every V load of the prefetch as soon as it was issued.
  auto fetch = [&](int p) {
    const int k0 = p * BB, r0 = k0 + BB, m = n - r0;
    const double* Ap = A + (int64_t)r0 * lda + k0; // &V_p[0][0] (wave-uniform)
#pragma unroll
    for (int q = 0; q < NBT; ++q) {
      const int b = wid + NWT * q;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * b - r0 + 4 * r + g4;
        const int ic = min(max(i, 0), m - 1);
        vn[q][r] = Ap[(int64_t)ic * lda + c16];
      }
    }
    const double* Tp = bw.T + (int64_t)p * BB * BB;
#pragma unroll
    for (int r = 0; r < 4; ++r) tn[r] = Tp[c16 * BB + 4 * r + g4];
  };
  const int np = (n - 1) / BB;    // panels: k0 = 16 p with k0 + 16 < n
  if (np > 0) fetch(np - 1);
  for (int p = np - 1; p >= 0; --p) {
    double (*rp)[BB * BB] = red[p & 1];
    double va[NBT][4], tv[4];
    {
      const int m = n - (p * BB + BB);
#pragma unroll
      for (int q = 0; q < NBT; ++q) {
        const int b = wid + NWT * q;
        const bool live = b > p && b < nb;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * (b - p - 1) + 4 * r + g4;
          va[q][r] = (live && i < m && i >= c16) ? (i == c16 ? 1.0 : vn[q][r]) : 0.0;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) tv[r] = tn[r];
    if (p > 0) fetch(p - 1);                        // next panel's V in flight from here on
    // P_w = sum over live blocks of V_b^T Y_b; V_b also to the wave's LDS image
    double4_t Pp[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};   // two MFMA chains
#pragma unroll
    for (int q = 0; q < NBT; ++q) {
      const int b = wid + NWT * q;
      if (b > p && b < nb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          Vw[wid][q][4 * r + g4][c16] = va[q][r];
          Pp[r & 1] = mfma_f64_16x16x4(va[q][r], Y[q][r], Pp[r & 1]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) rp[wid][(g4 + 4 * r) * BB + c16] = Pp[0][r] + Pp[1][r];
    __syncthreads();
    // M = T P (every wave)
    double4_t Mm = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double pv = 0.0;
#pragma unroll
      for (int w = 0; w < NWT; ++w) pv += rp[w][(4 * r + g4) * BB + c16];
      Mm = mfma_f64_16x16x4(tv[r], pv, Mm);
    }
    // Y_b -= V_b M   (A operand V_b[c16][4 r + g4] from the wave's own image)
#pragma unroll
    for (int q = 0; q < NBT; ++q) {
      const int b = wid + NWT * q;
      if (b > p && b < nb) {
        double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = mfma_f64_16x16x4(Vw[wid][q][c16][4 * r + g4], Mm[r], acc);
        Y[q] -= acc;
      }
    }
  }
  if (lok) {
    double* __restrict__ out = beta_out + cd.out + (int64_t)(l0 + c16) * ldo;
#pragma unroll
    for (int q = 0; q < NBT; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * (wid + NWT * q) + g4 + 4 * r;
        if (i < n) out[i] = Y[q][r];
      }
  }
}

}  // namespace

extern "C" int64_t pfml_ridge_band_work_doubles(int n, int L) {
  const int64_t np = (n + BB - 1) / BB;
  const int64_t npad = band_npad(n);
  // F region: the cooperative hand-off scratch (CoopWork)
  const int64_t coop = 2LL * npad * BB + BB * BB + (int64_t)(BNMAX / BB) * (BB * BB + BB);
  return npad * npad + (int64_t)n * LS + n + np * BB * BB + (int64_t)L * n + 15 +
         (int64_t)L * n * LS + coop;
}

extern "C" int pfml_ridge_band_nmax() { return BNMAX; }

namespace {
// Panel-QR micro-benchmark (tools/bench_qr.py): every workgroup factors its own m x 16 panel
// (row-major in P) `reps` times with band_panel_hh, the band reduction's hot serial step, from
// an LDS image of the panel as the cooperative kernel holds it.  Cycles per factorisation
// (thread 0's s_memtime) -> cyc[block * 8 + ...]: total, load, column loop (incl. V stores),
// G + T, and the column loop's own work / barrier wait / pivot chain + update; V -> Vout,
// T -> Tout; R / V as band_panel_hh stores them land in A's columns 0..15, rows 16.. (lda =
// m + 16).
__global__ __launch_bounds__(NTR) void band_qr_bench_kernel(const double* __restrict__ P, int m,
                                                            int reps,
                                                            double* __restrict__ Aout,
                                                            double* __restrict__ Vout,
                                                            double* __restrict__ Tout,
                                                            long long* __restrict__ cyc) {
  __shared__ double Vs[BMP][LS];
  __shared__ double Gs[BB][LS];
  __shared__ double red[NWR][BB * BB];
  __shared__ double Ts[BB][LS];
  __shared__ double taus[BB];
  const int t = threadIdx.x;
  const int lda = m + BB;
  const double* Pb = P + (int64_t)blockIdx.x * m * BB;
  double* Ab = Aout + (int64_t)blockIdx.x * lda * lda;
  long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = t; e < BMP * BB; e += NTR) {
      const int i = e / BB, c = e % BB;
      Vs[i][c] = (i < m) ? Pb[e] : 0.0;
    }
    __syncthreads();
    long long tk[6] = {0, 0, 0, 0, 0, 0};
    const long long t0 = (long long)__builtin_amdgcn_s_memtime();
    band_panel_hh(Ab, lda, 0, BB, m, Vs, Gs, &red[0][0], Ts, taus,
                  Tout + (int64_t)blockIdx.x * BB * BB, t == 0 ? tk : nullptr, Vs);
    __syncthreads();
    const long long t1 = (long long)__builtin_amdgcn_s_memtime();
    acc[0] += t1 - t0;
    acc[1] += tk[0] - t0;
    acc[2] += tk[1] - tk[0];
    acc[3] += t1 - tk[1];
    acc[4] += tk[2];
    acc[5] += tk[3];
    acc[6] += tk[4];
  }
  for (int e = t; e < m * BB; e += NTR) Vout[(int64_t)blockIdx.x * m * BB + e] = Vs[e / BB][e % BB];
  if (t == 0)
    for (int q = 0; q < 8; ++q) cyc[(int64_t)blockIdx.x * 8 + q] = acc[q] / (reps > 0 ? reps : 1);
}
}  // namespace

extern "C" hipError_t pfml_band_qr_bench(const double* P, int m, int nblocks, int reps,
                                         double* Aout, double* Vout, double* Tout,
                                         long long* cyc, hipStream_t st) {
  if (m < 1 || m > BMP) return hipErrorInvalidValue;
  hipLaunchKernelGGL(band_qr_bench_kernel, dim3(nblocks), dim3(NTR), 0, st, P, m, reps, Aout,
                     Vout, Tout, cyc);
  return hipGetLastError();
}

// Poll bound of the cooperative reduction's hand-off waits for later launches (0: default).
extern "C" void pfml_coop_set_spin_max(unsigned n) { g_coop_spin_max = n ? n : COOP_SPIN_MAX; }

namespace {
// kernel 3 instances by cell size: (waves, row blocks per wave) with 16 NWT NBT >= n
template <int NWT, int NBT>
void bt_one(const RidgeCellDesc* cd, int c0, int nc, int L, double* work, double* beta_out,
            int64_t ldo, const unsigned* syncw, hipStream_t st) {
  const int nch = (L + LC - 1) / LC;
  hipLaunchKernelGGL((ridge_band_backtransform_kernel<NWT, NBT>), dim3(nc * nch), dim3(NWT * 64),
                     0, st, cd, c0, nc, L, work, beta_out, ldo, syncw);
}

int bt_class(int n) { return n <= 96 ? 0 : (n <= 192 ? 1 : (n <= 320 ? 2 : 3)); }

// kernel 3 over a launch's cells: one launch per run of consecutive cells of one instance
// class (the plan orders cells by size, ops/ridge.py ridge_plan, so a grid has one run per
// size class).  n_host: the cells' n in plan order (host copy); nullptr = the 8-wave form for all.
void ridge_band_bt_launch(const RidgeCellDesc* cd, const int* n_host, int ncells, int L,
                          double* work, double* beta_out, int64_t ldo, const unsigned* syncw,
                          hipStream_t st) {
  if (n_host == nullptr) {
    bt_one<NWB, NBW>(cd, 0, ncells, L, work, beta_out, ldo, syncw, st);
    return;
  }
  int c0 = 0;
  while (c0 < ncells) {
    const int k = bt_class(n_host[c0]);
    int c1 = c0 + 1;
    while (c1 < ncells && bt_class(n_host[c1]) == k) ++c1;
    switch (k) {
      case 0: bt_one<2, 3>(cd, c0, c1 - c0, L, work, beta_out, ldo, syncw, st); break;
      case 1: bt_one<4, 3>(cd, c0, c1 - c0, L, work, beta_out, ldo, syncw, st); break;
      case 2: bt_one<4, 5>(cd, c0, c1 - c0, L, work, beta_out, ldo, syncw, st); break;
      default: bt_one<NWB, NBW>(cd, c0, c1 - c0, L, work, beta_out, ldo, syncw, st); break;
    }
    c0 = c1;
  }
}
}  // namespace

extern "C" hipError_t pfml_ridge_band_launch(const double* SD, int64_t ldS, const double* Sr,
                                             const void* cells, int ncells, const double* lvec,
                                             int L, double* work, double* beta_out, int64_t ldo,
                                             long long* tim, int* lu_list, int* lu_count,
                                             int lu_cap, const int* wgmap, int nwg,
                                             unsigned* syncw, const int* n_host,
                                             hipStream_t st) {
  const RidgeCellDesc* cd = static_cast<const RidgeCellDesc*>(cells);
  // the cooperative reduction: nwg workgroups (wgmap: cell << 8 | w << 4 | K - 1), the cells'
  // sync words zeroed on the stream first (a memset node under graph capture)
  if (wgmap == nullptr || syncw == nullptr || nwg <= 0)
    return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(syncw, 0, (size_t)ncells * COOP_SYNC * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  if (tim != nullptr)
    hipLaunchKernelGGL(band_coop_kernel<true>, dim3(nwg), dim3(NTR), 0, st, SD, ldS, Sr, cd, L,
                       work, wgmap, syncw, tim, g_coop_spin_max);
  else
    hipLaunchKernelGGL(band_coop_kernel<false>, dim3(nwg), dim3(NTR), 0, st, SD, ldS, Sr, cd, L,
                       work, wgmap, syncw, tim, g_coop_spin_max);
  // (timing: the cooperative kernel fills 16 slots per cell, the solve's two go after them)
  hipLaunchKernelGGL(ridge_band_solve_kernel, dim3(ncells * ((L + 15) / 16)), dim3(NTS), 0, st,
                     cd, lvec, L, work,
                     tim != nullptr ? tim + (int64_t)ncells * 8 : tim, ncells,
                     lu_count);
  if (lu_count != nullptr) {   // non-SPD lambdas: pivoted banded LU (count zeroed by kernel 2)
    hipLaunchKernelGGL(band_lu_flag_kernel, dim3((ncells * L + 255) / 256), dim3(256), 0, st, cd,
                       ncells, L, work, lu_list, lu_count, lu_cap);
    hipLaunchKernelGGL(ridge_band_lu_kernel, dim3(LU_WG), dim3(64), 0, st, cd, lvec, L, work,
                       lu_list, lu_count, lu_cap);
  }
  const int nch = (L + LC - 1) / LC;
  ridge_band_bt_launch(cd, n_host, ncells, L, work, beta_out, ldo, syncw, st);
  return hipGetLastError();
}
