// Batched, strided fp64 GEMM on CDNA4 matrix cores (v_mfma_f64_16x16x4_f64).
//
//   C[b] = alpha * diag(rs[b]) * op(A[b]) * op(B[b]) * diag(cs[b]) + beta * C[b]
//
// This is the workhorse of the PFML engine: the reference
// runs every one of these products as an OpenBLAS dgemm, often with a dense diagonal matrix
// as one operand (`m @ np.diag(gt)`, `np.diag(1/vol) @ s`, ...).  Here the diagonal factors
// are fused as row/column scales of the epilogue, so they cost O(MN) instead of a GEMM.
//
// Tiling: BM x BN output tile per 256-thread workgroup (4 waves, 2 x 2), BK = 16 staged in
// LDS.  Each operand keeps the layout it has in global memory, so the LDS stores are as
// conflict-free as the coalesced global loads: an operand contiguous along k (A not
// transposed, B transposed) is stored [row][k] with a row stride of 18 doubles (the 16 rows x
// 2 k of one ds_read_b64 group then hit 32 distinct bank pairs), one contiguous along its
// row/column index is stored [k][index] with a 16-double pad (stride = 32 banks mod 64).
// Each wave owns a (BM/2) x (BN/2) sub-tile = (BM/32) x (BN/32) MFMA 16x16 accumulators.
// Double-buffered LDS: the global loads of K-step t+1 are issued into registers before the
// MFMAs of step t.
#include "common.h"

namespace {

constexpr int BK = 16;
constexpr int PAD = 16;      // [k][index] layouts
constexpr int KS = BK + 2;   // [index][k] layouts: row stride in doubles

template <bool TA, bool TB, int BM, int BN>
__global__ __launch_bounds__(256) void dgemm_kernel(
    int M, int N, int K, double alpha,
    const double* __restrict__ A, int64_t lda, int64_t sA,
    const double* __restrict__ B, int64_t ldb, int64_t sB,
    double beta, double* __restrict__ C, int64_t ldc, int64_t sC,
    const double* __restrict__ rs, int64_t srs,
    const double* __restrict__ cs, int64_t scs) {
  constexpr int TM = BM / 32, TN = BN / 32;         // MFMA tiles per wave (M, N)
  constexpr int LA = BM * BK / 256, LB = BN * BK / 256;  // elements loaded per thread
  // A: TA ? [k][i] : [i][k];  B: TB ? [j][k] : [k][j]   (flat, see the header)
  constexpr int ASZ = TA ? BK * (BM + PAD) : BM * KS;
  constexpr int BSZ = TB ? BN * KS : BK * (BN + PAD);
  __shared__ double As[2][ASZ];
  __shared__ double Bs[2][BSZ];
  auto aidx = [](int i, int k) { return TA ? k * (BM + PAD) + i : i * KS + k; };
  auto bidx = [](int k, int j) { return TB ? j * KS + k : k * (BN + PAD) + j; };

  const int b = blockIdx.y;
  A += (int64_t)b * sA;
  B += (int64_t)b * sB;
  C += (int64_t)b * sC;
  const int tiles_n = (N + BN - 1) / BN;
  const int tile = blockIdx.x;
  const int bm = (tile / tiles_n) * BM, bn = (tile % tiles_n) * BN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;

  double4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = double4_t{0.0, 0.0, 0.0, 0.0};

  double ra[LA], rb[LB];
  // global -> registers for the K-step starting at k0
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int e = t + q * 256;
      int i, k;
      if (TA) { k = e / BM; i = e % BM; }            // A stored K x M: contiguous along i
      else    { i = e / BK; k = e % BK; }            // A stored M x K: contiguous along k
      const int gi = bm + i, gk = k0 + k;
      double v = 0.0;
      if (gi < M && gk < K) v = TA ? A[(int64_t)gk * lda + gi] : A[(int64_t)gi * lda + gk];
      ra[q] = v;
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int e = t + q * 256;
      int j, k;
      if (TB) { j = e / BK; k = e % BK; }            // B stored N x K: contiguous along k
      else    { k = e / BN; j = e % BN; }            // B stored K x N: contiguous along j
      const int gj = bn + j, gk = k0 + k;
      double v = 0.0;
      if (gj < N && gk < K) v = TB ? B[(int64_t)gj * ldb + gk] : B[(int64_t)gk * ldb + gj];
      rb[q] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int e = t + q * 256;
      int i, k;
      if (TA) { k = e / BM; i = e % BM; } else { i = e / BK; k = e % BK; }
      As[buf][aidx(i, k)] = ra[q];
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int e = t + q * 256;
      int j, k;
      if (TB) { j = e / BK; k = e % BK; } else { k = e / BN; j = e % BN; }
      Bs[buf][bidx(k, j)] = rb[q];
    }
  };

  const int nk = (K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    const int cur = s & 1;
    if (s + 1 < nk) load((s + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      double a[TM], bb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[cur][aidx(wm * (BM / 2) + i * 16 + (lane & 15), kk + (lane >> 4))];
#pragma unroll
      for (int j = 0; j < TN; ++j) bb[j] = Bs[cur][bidx(kk + (lane >> 4), wn * (BN / 2) + j * 16 + (lane & 15))];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_f64_16x16x4(a[i], bb[j], acc[i][j]);
    }
    if (s + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  const double* rsb = rs ? rs + (int64_t)b * srs : nullptr;
  const double* csb = cs ? cs + (int64_t)b * scs : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = bm + wm * (BM / 2) + i * 16 + PFML_F64_CROW(lane, r);
        const int gj = bn + wn * (BN / 2) + j * 16 + (lane & 15);
        if (gi < M && gj < N) {
          double v = alpha * acc[i][j][r];
          if (rsb) v *= rsb[gi];
          if (csb) v *= csb[gj];
          double* cp = C + (int64_t)gi * ldc + gj;
          if (beta != 0.0) v += beta * (*cp);
          *cp = v;
        }
      }
}

template <int BM, int BN>
hipError_t launch(int ta, int tb, int M, int N, int K, int batch, double alpha,
                  const double* A, int64_t lda, int64_t sA, const double* B, int64_t ldb,
                  int64_t sB, double beta, double* C, int64_t ldc, int64_t sC,
                  const double* rs, int64_t srs, const double* cs, int64_t scs,
                  hipStream_t st) {
  dim3 grid(((M + BM - 1) / BM) * ((N + BN - 1) / BN), batch);
  dim3 block(256);
#define PFML_GEMM_CASE(TA_, TB_)                                                            \
  hipLaunchKernelGGL((dgemm_kernel<TA_, TB_, BM, BN>), grid, block, 0, st, M, N, K, alpha, A, \
                     lda, sA, B, ldb, sB, beta, C, ldc, sC, rs, srs, cs, scs)
  if (!ta && !tb) PFML_GEMM_CASE(false, false);
  else if (!ta && tb) PFML_GEMM_CASE(false, true);
  else if (ta && !tb) PFML_GEMM_CASE(true, false);
  else PFML_GEMM_CASE(true, true);
#undef PFML_GEMM_CASE
  return hipGetLastError();
}

}  // namespace

extern "C" hipError_t pfml_dgemm(int ta, int tb, int M, int N, int K, int batch, double alpha,
                                 const double* A, int64_t lda, int64_t sA,
                                 const double* B, int64_t ldb, int64_t sB, double beta,
                                 double* C, int64_t ldc, int64_t sC,
                                 const double* rs, int64_t srs, const double* cs, int64_t scs,
                                 hipStream_t st) {
  if (M <= 0 || N <= 0 || batch <= 0) return hipSuccess;
  // Large problems: 128 x 128 tiles (4 x 4 accumulators per wave); small: 64 x 64 so that a
  // batch of ~500 x 500 matrices still gives >> 256 workgroups.
  const long tiles128 = (long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  if (tiles128 >= 512)
    return launch<128, 128>(ta, tb, M, N, K, batch, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc,
                            sC, rs, srs, cs, scs, st);
  return launch<64, 64>(ta, tb, M, N, K, batch, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC,
                        rs, srs, cs, scs, st);
}
