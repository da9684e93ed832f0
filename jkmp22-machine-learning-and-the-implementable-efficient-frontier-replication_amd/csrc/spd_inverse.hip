// Batched in-place inverse of symmetric positive definite matrices by blocked Gauss-Jordan
// elimination without pivoting (the 10 fixed-point inversions of m_func,
// General_functions.py:959-960, plus the Denman-Beavers square-root iterations that replace
// scipy.linalg.sqrtm, :956).
//
// For block column k (width NB):
//     P      = A_kk^-1                          (pivot block, Gauss-Jordan in LDS)
//     A_kj  <- P A_kj            (j != k)       row panel
//     A_ij  <- A_ij - A_ik A_kj  (i, j != k)    rank-NB trailing update (fp64 MFMA)
//     A_ik  <- -A_ik P           (i != k)       column panel
//     A_kk  <- P
// SPD pivots are Schur-complement diagonals (positive), so no pivoting is needed; a
// non-positive or non-finite pivot sets the matrix's status flag and the host falls back to
// a pivoted LU inverse for that matrix only.
//
// Kernels per block step (all batched over matrices): pivot+row panel (one workgroup per
// matrix and column tile), trailing update with the column panel fused in the same launch
// (workgroups owning column k's tiles apply -A_ik P instead of the update).
#include "common.h"

namespace {

constexpr int NB = 32;

// ---- step 1: invert the NB x NB pivot block of every matrix in LDS; write P to a side buffer
__global__ __launch_bounds__(256) void gj_pivot_kernel(double* __restrict__ A, int n, int64_t lda,
                                                        int64_t sA, int k0, int nb,
                                                        double* __restrict__ Pbuf,
                                                        int* __restrict__ status) {
  __shared__ double P[NB][NB + 1];
  const int b = blockIdx.x;
  double* Ab = A + (int64_t)b * sA;
  const int t = threadIdx.x;
  for (int e = t; e < nb * nb; e += 256) {
    const int i = e / nb, j = e % nb;
    P[i][j] = Ab[(int64_t)(k0 + i) * lda + k0 + j];
  }
  __syncthreads();
  // unblocked Gauss-Jordan on the nb x nb block (in place)
  for (int p = 0; p < nb; ++p) {
    const double piv = P[p][p];
    __syncthreads();
    if (!(piv > 0.0) || !isfinite(piv)) {
      if (t == 0) status[b] = 1;
    }
    const double inv = 1.0 / piv;
    // row p scaled, column p updated; thread handles element (i, j)
    for (int e = t; e < nb * nb; e += 256) {
      const int i = e / nb, j = e % nb;
      if (i != p && j != p) P[i][j] -= P[i][p] * P[p][j] * inv;
    }
    __syncthreads();
    for (int e = t; e < nb; e += 256) {
      if (e != p) {
        P[p][e] *= inv;
        P[e][p] *= -inv;
      }
    }
    if (t == 0) P[p][p] = inv;
    __syncthreads();
  }
  double* Pb = Pbuf + (int64_t)b * NB * NB;
  for (int e = t; e < nb * nb; e += 256) {
    const int i = e / nb, j = e % nb;
    Pb[i * NB + j] = P[i][j];
  }
}

// ---- step 2: row panel  R_kj = P A_kj  (written to Rbuf, width n), A_kj keeps old values
__global__ __launch_bounds__(256) void gj_rowpanel_kernel(const double* __restrict__ A, int n,
                                                           int64_t lda, int64_t sA, int k0, int nb,
                                                           const double* __restrict__ Pbuf,
                                                           double* __restrict__ Rbuf) {
  __shared__ double P[NB][NB + 1];
  const int b = blockIdx.y;
  const double* Ab = A + (int64_t)b * sA;
  const int t = threadIdx.x;
  // the full NB x NB tile: entries beyond nb must read as 0 (the product below runs over all
  // NB columns, and 0 * uninitialised LDS can be NaN)
  for (int e = t; e < NB * NB; e += 256) {
    const int i = e / NB, q = e % NB;
    P[i][q] = (i < nb && q < nb) ? Pbuf[(int64_t)b * NB * NB + i * NB + q] : 0.0;
  }
  __syncthreads();
  const int j = blockIdx.x * 256 + t;
  if (j >= n) return;
  double col[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) col[q] = (q < nb) ? Ab[(int64_t)(k0 + q) * lda + j] : 0.0;
  double* Rb = Rbuf + (int64_t)b * NB * n;
#pragma unroll 4
  for (int i = 0; i < nb; ++i) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NB; ++q) s += P[i][q] * col[q];
    Rb[(int64_t)i * n + j] = s;
  }
}

// ---- step 3: trailing update + column panel, 64 x 64 tiles on fp64 MFMA.
// For output tile (I, J):
//   J not in block k, I not in block k: A_IJ -= A_Ik R_kJ       (A_Ik = OLD column panel)
//   J not in block k, I in block k   : A_kJ  = R_kJ
//   J in block k, I not in block k   : A_Ik  = -A_Ik P          (OLD A_Ik)
//   J in block k, I in block k       : A_kk  = P
// Tiles that read the old column panel must not race with tiles that overwrite it: the
// column-panel tiles (J in block k) first stash A_Ik in LDS and every other tile reads the
// column panel from the snapshot Cbuf taken by gj_snapshot_kernel.
__global__ __launch_bounds__(256) void gj_snapshot_kernel(const double* __restrict__ A, int n,
                                                           int64_t lda, int64_t sA, int k0, int nb,
                                                           double* __restrict__ Cbuf) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double* Ab = A + (int64_t)b * sA + (int64_t)i * lda + k0;
  double* Cb = Cbuf + (int64_t)b * n * NB + (int64_t)i * NB;
#pragma unroll
  for (int q = 0; q < NB; ++q) Cb[q] = (q < nb) ? Ab[q] : 0.0;
}

__global__ __launch_bounds__(256) void gj_update_kernel(double* __restrict__ A, int n, int64_t lda,
                                                         int64_t sA, int k0, int nb,
                                                         const double* __restrict__ Pbuf,
                                                         const double* __restrict__ Rbuf,
                                                         const double* __restrict__ Cbuf) {
  constexpr int BT = 64;
  __shared__ double Cs[NB][BT + 16];     // column panel tile, k-major: Cs[q][i]
  __shared__ double Rs[NB][BT + 16];     // row panel tile: Rs[q][j]
  const int b = blockIdx.y;
  double* Ab = A + (int64_t)b * sA;
  const double* Pb = Pbuf + (int64_t)b * NB * NB;
  const double* Rb = Rbuf + (int64_t)b * NB * n;
  const double* Cb = Cbuf + (int64_t)b * n * NB;
  const int tiles = (n + BT - 1) / BT;
  const int I0 = (blockIdx.x / tiles) * BT, J0 = (blockIdx.x % tiles) * BT;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  // load column panel rows I0.. (old values) and row panel cols J0..
  for (int e = t; e < BT * NB; e += 256) {
    const int i = e / NB, q = e % NB;
    Cs[q][i] = (I0 + i < n && q < nb) ? Cb[(int64_t)(I0 + i) * NB + q] : 0.0;
  }
  for (int e = t; e < NB * BT; e += 256) {
    const int q = e / BT, j = e % BT;
    Rs[q][j] = (J0 + j < n && q < nb) ? Rb[(int64_t)q * n + J0 + j] : 0.0;
  }
  __syncthreads();
  double4_t acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = double4_t{0.0, 0.0, 0.0, 0.0};
  // rank-NB product for the whole tile (columns of block k simply ignore it)
#pragma unroll
  for (int q = 0; q < NB; q += 4) {
    double a[2], bb[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) a[x] = Cs[q + (lane >> 4)][wm * 32 + x * 16 + (lane & 15)];
#pragma unroll
    for (int y = 0; y < 2; ++y) bb[y] = Rs[q + (lane >> 4)][wn * 32 + y * 16 + (lane & 15)];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = mfma_f64_16x16x4(a[x], bb[y], acc[x][y]);
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = I0 + wm * 32 + x * 16 + PFML_F64_CROW(lane, r);
        const int j = J0 + wn * 32 + y * 16 + (lane & 15);
        if (i >= n || j >= n) continue;
        const bool ik = (i >= k0 && i < k0 + nb), jk = (j >= k0 && j < k0 + nb);
        double* p = Ab + (int64_t)i * lda + j;
        if (!ik && !jk) {
          *p -= acc[x][y][r];
        } else if (ik && !jk) {
          *p = Rb[(int64_t)(i - k0) * n + j];
        } else if (!ik && jk) {
          double s = 0.0;
          for (int q = 0; q < nb; ++q) s += Cb[(int64_t)i * NB + q] * Pb[q * NB + (j - k0)];
          *p = -s;
        } else {
          *p = Pb[(i - k0) * NB + (j - k0)];
        }
      }
}

}  // namespace

extern "C" int64_t pfml_spd_inverse_work_doubles(int n, int batch) {
  return (int64_t)batch * (NB * NB + 2LL * NB * n);
}

// In-place inverse of `batch` SPD matrices (n x n, leading dim lda, batch stride sA).
// work: pfml_spd_inverse_work_doubles(n, batch) doubles; status: batch ints (set to 1 when a
// non-positive pivot was met; caller zero-initialises).
extern "C" hipError_t pfml_spd_inverse(double* A, int n, int64_t lda, int64_t sA, int batch,
                                       double* work, int* status, hipStream_t st) {
  if (n <= 0 || batch <= 0) return hipSuccess;
  double* Pbuf = work;
  double* Rbuf = Pbuf + (int64_t)batch * NB * NB;
  double* Cbuf = Rbuf + (int64_t)batch * NB * n;
  const int tiles = (n + 63) / 64;
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int nb = (n - k0 < NB) ? (n - k0) : NB;
    hipLaunchKernelGGL(gj_pivot_kernel, dim3(batch), dim3(256), 0, st, A, n, lda, sA, k0, nb,
                       Pbuf, status);
    hipLaunchKernelGGL(gj_rowpanel_kernel, dim3((n + 255) / 256, batch), dim3(256), 0, st, A, n,
                       lda, sA, k0, nb, Pbuf, Rbuf);
    hipLaunchKernelGGL(gj_snapshot_kernel, dim3((n + 255) / 256, batch), dim3(256), 0, st, A, n,
                       lda, sA, k0, nb, Cbuf);
    hipLaunchKernelGGL(gj_update_kernel, dim3(tiles * tiles, batch), dim3(256), 0, st, A, n, lda,
                       sA, k0, nb, Pbuf, Rbuf, Cbuf);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Leaves of the recursive Schur-complement inverse (the production form for n >= 160, host
// orchestration in ops/linalg.py::_spd_inverse_recursive: every off-diagonal product one
// fused GEMM, csrc/gemm_f64.hip).  (Blocked Gauss-Jordan forms with 64- / 128-wide pivot
// blocks and a fused sign-symmetric form measured 2.1 / 3.0 / 2.4x slower on [256, 490, 490],
// profiles/r02_inverse_variants_v2.json, and were removed.)
namespace {
constexpr int NBL = 64;

// Register-resident 64 x 64 Gauss-Jordan inverse (no pivoting: SPD blocks), 4 pivots per
// barrier.  An LDS form that re-reads and re-writes the whole block at every pivot was
// LDS-bandwidth bound (~80 us per batch of 256 blocks) and a one-pivot register form is
// bound by its 64 barrier + divide round trips (~50 us).  Here each of the 256 threads keeps a
// 4 x 4 sub-block in registers; pivot block q (4 pivots) is exactly thread row / column block
// q, so the owners publish whole register tiles to a double-buffered LDS line
// (one barrier per step, no second barrier: the buffer written at step q + 2 is rewritten
// only after every thread has passed step q + 1's barrier, i.e. finished reading it).  Frame
// entries past nb hold the identity, so partial blocks need no special case.  ``src``: the
// block (global or LDS, leading dimension ld); the inverse is left in a (thread (rb, cb) =
// (t >> 4, t & 15): rows 4 rb.., columns 4 cb..).  Every thread of the block must call it.
struct GjLds {
  double rowb[2][4][64], colb[2][64][4];
};

// 1 / x as v_rcp_f64 + two Newton steps (correctly rounded on every x measured by
// tools/micro/rsq_acc.hip, as the IEEE divide): a 5-instruction dependent chain in place of
// the divide's ~10 (div_scale, rcp, Newton, div_fmas, div_fixup) on every pivot - the pivot
// chain is what bounds a Gauss-Jordan step (profiles/r05_spd_node_phase_cycles.jsonl)
__device__ __forceinline__ double gj_rcp(double x) {
  double y = __builtin_amdgcn_rcp(x);
#pragma unroll
  for (int it = 0; it < 2; ++it) y = fma(y, fma(-x, y, 1.0), y);
  return y;
}

__device__ __forceinline__ bool gj64(const double* src, int64_t ld, int nb, double (&a)[4][4],
                                     GjLds& sh) {
  const int t = threadIdx.x;
  const int rb = t >> 4, cb = t & 15;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * rb + u, j = 4 * cb + v;
      a[u][v] = src[(int64_t)min(i, nb - 1) * ld + min(j, nb - 1)];
    }
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * rb + u, j = 4 * cb + v;
      if (!(i < nb && j < nb)) a[u][v] = (i == j) ? 1.0 : 0.0;
    }
  bool bad = false;
  const int nq = (nb + 3) >> 2;
  for (int q = 0; q < nq; ++q) {
    const int buf = q & 1;
    if (rb == q) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int v = 0; v < 4; ++v) sh.rowb[buf][r][4 * cb + v] = a[r][v];
    }
    if (cb == q) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) sh.colb[buf][4 * rb + u][c] = a[u][c];
    }
    __syncthreads();
    // The 4 pivots of the block, replayed as SCALAR Gauss-Jordan steps on the thread's local
    // 8 x 8 view M = [[P, rp], [cp, a]] (P = A_KK, rp = A_K,mycols, cp = A_myrows,K): every
    // entry sees the update sequence of one-pivot-at-a-time GJ (an explicit P^-1 block step
    // amplifies rounding by cond(P) on ill-conditioned Denman-Beavers iterates).  Pivot row
    // scaled first, then one FMA per updated entry: M[r][c] -= M[r][p] (M[p][c] / piv).
    double P[4][4], rp[4][4], cp[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) P[r][c] = sh.rowb[buf][r][4 * q + c];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int v = 0; v < 4; ++v) rp[r][v] = sh.rowb[buf][r][4 * cb + v];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) cp[u][c] = sh.colb[buf][4 * rb + u][c];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const double piv = P[p][p];
      bad |= !(piv > 0.0) || !isfinite(piv);
      const double inv = gj_rcp(piv);
      // pivot row (its final values)
#pragma unroll
      for (int v = 0; v < 4; ++v) rp[p][v] *= inv;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c != p) P[p][c] *= inv;
      // a (rows != p, cols != p: always, the thread's rows / cols are outside K unless it
      // owns the pivot block, whose result is then read from P / rp / cp below)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) a[u][v] = fma(-cp[u][p], rp[p][v], a[u][v]);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r != p)
#pragma unroll
          for (int v = 0; v < 4; ++v) rp[r][v] = fma(-P[r][p], rp[p][v], rp[r][v]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c != p) cp[u][c] = fma(-cp[u][p], P[p][c], cp[u][c]);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (r != p && c != p) P[r][c] = fma(-P[r][p], P[p][c], P[r][c]);
      // pivot column (old values used above)
#pragma unroll
      for (int u = 0; u < 4; ++u) cp[u][p] *= -inv;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r != p) P[r][p] *= -inv;
      P[p][p] = inv;
    }
    const bool inr = rb == q, inc = cb == q;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        a[u][v] = (inr && inc) ? P[u][v] : (inr ? rp[u][v] : (inc ? cp[u][v] : a[u][v]));
  }
  return bad;
}

// Output to any (ld, batch stride): in place (Pout = the block itself) or to a packed buffer.
__global__ __launch_bounds__(256) void spd_leafinv_kernel(const double* __restrict__ A,
                                                          int64_t lda, int64_t sA, int k0,
                                                          int nb, double* Pout, int64_t ldp,
                                                          int64_t sP, int* __restrict__ status,
                                                          int sym) {
  __shared__ GjLds sh;
  const int b = blockIdx.x, t = threadIdx.x;
  const int rb = t >> 4, cb = t & 15;
  double a[4][4];
  const bool bad = gj64(A + (int64_t)b * sA + (int64_t)k0 * lda + k0, lda, nb, a, sh);
  if (t == 0 && bad) status[b] = 1;
  double* Pb = Pout + (int64_t)b * sP;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * rb + u, j = 4 * cb + v;
      if (!(i < nb && j < nb)) continue;
      if (!sym) {
        Pb[(int64_t)i * ldp + j] = a[u][v];
      } else if (i >= j) {             // exactly symmetric output: the lower triangle, mirrored
        Pb[(int64_t)i * ldp + j] = a[u][v];
        Pb[(int64_t)j * ldp + i] = a[u][v];
      }
    }
}

// ---------------------------------------------------------------------------------------
// One whole node of the one-triangle recursive inverse (ops/linalg.py spd_inverse_sym) for
// 64 < nn <= 128, in ONE launch (one workgroup per matrix): the two 64-leaf Gauss-Jordan
// inverses and the node's four products on the MFMA, with every operand in LDS -
//
//     X11 = A11^-1 (GJ),  W = X11 A12,  S = A22 - A21 W (lower tiles, mirrored),
//     X22 = S^-1 (GJ),  X12 = -W X22 (X21 = X12'),  X11 -= X12 W' (lower tiles, mirrored)
//
// instead of 4 GEMM launches + 2 leaf launches per node (the 64-wide GEMMs ran at 5-9 TF/s:
// tile prologue / epilogue and launch bound).  Each product walks k in steps of 4 from 0 with
// zero padding past K and applies the same epilogue expressions as the fused GEMM
// (csrc/gemm_f64.hip: v = -acc + C, v = -acc), and the leaves are the same gj64, so the node is
// bitwise the launch sequence it replaces.  Input block exactly symmetric (A12 = A21' is read
// as A21).  LDS: two 64 x 64 operand images + the GJ lines (~76 KB: two workgroups per CU);
// X11 stays in the GJ registers between its inverse and the final update.
constexpr int NLP = 66;                        // operand image row stride (doubles)

// phase timestamps of workgroup 0 (a build with -DPFML_NODE_TIMING; pfml_node_timing reads
// them): where one node's latency goes, for the small-batch (per-rank) S4
#ifdef PFML_NODE_TIMING
__device__ unsigned long long g_node_ts[16];
#define NODE_TS(k) do { if (blockIdx.x == 0 && threadIdx.x == 0) g_node_ts[k] = clock64(); } while (0)
#else
#define NODE_TS(k) do { } while (0)
#endif

struct NodeLds {
  double u[64][NLP];                           // X11 -> W
  double v[64][NLP];                           // A21 -> S -> X22 -> X12 -> X12 W'
  GjLds gj;
};

// acc[q] (q < nt) = sum_k A(ti[q] * 16 + i, k) B(k, tj[q] * 16 + j), k < K (zero past K);
// fa(i, k) / fb(k, j) read the LDS images (k, i, j in range: the callers clamp / mask)
template <int NT, class FA, class FB>
__device__ __forceinline__ void node_mm(const int (&ti)[NT], const int (&tj)[NT], int nt, int K,
                                        FA fa, FB fb, double4_t (&acc)[NT]) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int q = 0; q < NT; ++q) acc[q] = double4_t{0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < K; k0 += 4) {
    const int k = k0 + lk;
    const bool ok = k < K;
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      if (q < nt) {
        const double av = ok ? fa(ti[q] * 16 + li, k) : 0.0;
        const double bv = ok ? fb(k, tj[q] * 16 + li) : 0.0;
        acc[q] = mfma_f64_16x16x4(av, bv, acc[q]);
      }
    }
  }
}

// Src: the input (the same layout as X; == X in place): A11, A21, A22 are read from it, every
// result is written to X (out of place: no copy of the input first)
__global__ __launch_bounds__(256, 2) void spd_node_sym_kernel(const double* Src, double* X,
                                                             int64_t ld, int64_t sX, int r0,
                                                             int nn, int* __restrict__ status) {
  __shared__ NodeLds L;
  NODE_TS(0);
  const int b = blockIdx.x, t = threadIdx.x;
  const int lane = t & 63, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int rb = t >> 4, cb = t & 15;
  const int m = nn - 64;                       // 1..64
  const int tn = (m + 15) >> 4;                // 16-wide tiles over m
  double* Xb = X + (int64_t)b * sX + (int64_t)r0 * ld + r0;
  double* X21 = Xb + (int64_t)64 * ld;         // rows 64.., columns 0..
  double* X22 = X21 + 64;
  const double* Ab = Src + (int64_t)b * sX + (int64_t)r0 * ld + r0;
  const double* A21 = Ab + (int64_t)64 * ld;
  const double* A22 = A21 + 64;
  // A21 -> v (rows >= m: zero)
  for (int e = t; e < 64 * 64; e += 256) {
    const int i = e >> 6, k = e & 63;
    L.v[i][k] = i < m ? A21[(int64_t)i * ld + k] : 0.0;
  }
  // X11 = A11^-1 (registers), its mirrored image -> u
  double x11[4][4];
  NODE_TS(1);
  bool bad = gj64(Ab, ld, 64, x11, L.gj);
  NODE_TS(2);
#pragma unroll
  for (int uu = 0; uu < 4; ++uu)
#pragma unroll
    for (int vv = 0; vv < 4; ++vv) {
      const int i = 4 * rb + uu, j = 4 * cb + vv;
      if (i >= j) {
        L.u[i][j] = x11[uu][vv];
        L.u[j][i] = x11[uu][vv];
      }
    }
  __syncthreads();
  double4_t acc[4];
  // W = X11 A21' (64 x m): wave w = tile row w, all tn tile columns
  {
    const int ti[4] = {w, w, w, w}, tj[4] = {0, 1, 2, 3};
    node_mm<4>(ti, tj, tn, 64, [&](int i, int k) { return L.u[i][k]; },
               [&](int k, int j) { return L.v[j][k]; }, acc);
  }
  __syncthreads();                             // u (X11) fully read
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < tn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = w * 16 + PFML_F64_CROW(lane, r), j = q * 16 + li;
        L.u[i][j] = j < m ? acc[q][r] : 0.0;  // W (columns >= m: zero)
      }
  __syncthreads();
  NODE_TS(3);
  // S = A22 - A21 W: lower tiles (I >= J) of the tn x tn grid, round-robin over the waves
  {
    int ti[3], tj[3], nt = 0;
    const int nl = tn * (tn + 1) / 2;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int l = w + 4 * q;
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= l) ++I;
      ti[q] = l < nl ? I : 0;
      tj[q] = l < nl ? l - I * (I + 1) / 2 : 0;
      nt += l < nl;
    }
    double4_t sacc[3];
    node_mm<3>(ti, tj, nt, 64, [&](int i, int k) { return L.v[i][k]; },
               [&](int k, int j) { return L.u[k][j]; }, sacc);
    double sv[3][4];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = ti[q] * 16 + PFML_F64_CROW(lane, r), j = tj[q] * 16 + li;
        const double c = (q < nt && i < m && j < m) ? A22[(int64_t)i * ld + j] : 0.0;
        sv[q][r] = -sacc[q][r] + c;
      }
    __syncthreads();                           // v (A21) fully read
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q < nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = ti[q] * 16 + PFML_F64_CROW(lane, r), j = tj[q] * 16 + li;
          if (i < m && j < m && i >= j) {
            L.v[i][j] = sv[q][r];
            L.v[j][i] = sv[q][r];
          }
        }
  }
  __syncthreads();
  NODE_TS(4);
  // X22 = S^-1 -> global (lower, mirrored) and v (its mirrored image, zero outside m x m)
  double x22[4][4];
  bad |= gj64(&L.v[0][0], NLP, m, x22, L.gj);
  NODE_TS(5);
  __syncthreads();                             // every thread has loaded S from v
#pragma unroll
  for (int uu = 0; uu < 4; ++uu)
#pragma unroll
    for (int vv = 0; vv < 4; ++vv) {
      const int i = 4 * rb + uu, j = 4 * cb + vv;
      if (i >= j) {
        const bool in = i < m;
        L.v[i][j] = in ? x22[uu][vv] : 0.0;
        L.v[j][i] = in ? x22[uu][vv] : 0.0;
        if (in) {
          X22[(int64_t)i * ld + j] = x22[uu][vv];
          X22[(int64_t)j * ld + i] = x22[uu][vv];
        }
      }
    }
  if (t == 0 && bad) status[b] = 1;
  __syncthreads();
  NODE_TS(6);
  // X12 = -W X22 (64 x m) -> global X12 and X21 = X12'
  {
    const int ti[4] = {w, w, w, w}, tj[4] = {0, 1, 2, 3};
    node_mm<4>(ti, tj, tn, m, [&](int i, int k) { return L.u[i][k]; },
               [&](int k, int j) { return L.v[k][j]; }, acc);
  }
  __syncthreads();                             // v (X22) fully read
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < tn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = w * 16 + PFML_F64_CROW(lane, r), j = q * 16 + li;
        const double v = -acc[q][r];
        L.v[i][j] = j < m ? v : 0.0;
        if (j < m) {
          Xb[(int64_t)i * ld + 64 + j] = v;
          X21[(int64_t)j * ld + i] = v;
        }
      }
  __syncthreads();
  NODE_TS(7);
  // D = X12 W' on the lower tiles of 64 x 64 (10 tiles), then X11 -= D (lower, mirrored)
  {
    int ti[3], tj[3], nt = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int l = w + 4 * q;
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= l) ++I;
      ti[q] = l < 10 ? I : 0;
      tj[q] = l < 10 ? l - I * (I + 1) / 2 : 0;
      nt += l < 10;
    }
    double4_t dacc[3];
    node_mm<3>(ti, tj, nt, m, [&](int i, int k) { return L.v[i][k]; },
               [&](int k, int j) { return L.u[j][k]; }, dacc);
    __syncthreads();                           // v (X12) and u (W) fully read
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q < nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = ti[q] * 16 + PFML_F64_CROW(lane, r), j = tj[q] * 16 + li;
          L.u[i][j] = dacc[q][r];
        }
  }
  __syncthreads();
  NODE_TS(8);
#pragma unroll
  for (int uu = 0; uu < 4; ++uu)
#pragma unroll
    for (int vv = 0; vv < 4; ++vv) {
      const int i = 4 * rb + uu, j = 4 * cb + vv;
      if (i >= j) {
        const double v = -L.u[i][j] + x11[uu][vv];
        Xb[(int64_t)i * ld + j] = v;
        Xb[(int64_t)j * ld + i] = v;
      }
    }
  NODE_TS(9);
}
}  // namespace

// Inverse of the nb x nb (nb <= 64) diagonal block at (k0, k0) of A written to the block at
// (k0, k0) of P (any leading dims / batch strides; P == A: in place); sym: the lower triangle
// mirrored (an exactly symmetric result for the symmetric recursive form).
extern "C" hipError_t pfml_spd_leafinv_to(const double* A, int64_t lda, int64_t sA, double* P,
                                          int64_t ldp, int64_t sP, int batch, int k0, int nb,
                                          int* status, int sym, hipStream_t st) {
  if (batch <= 0 || nb <= 0) return hipSuccess;
  if (nb > NBL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spd_leafinv_kernel, dim3(batch), dim3(256), 0, st, A, lda, sA, k0, nb,
                     P + (int64_t)k0 * ldp + k0, ldp, sP, status, sym);
  return hipGetLastError();
}

// One-triangle inverse of the nn x nn diagonal block at (r0, r0) of every matrix of Src into
// the same block of X (Src == X: in place), 64 < nn <= 128 (exactly symmetric input and
// output), one launch (spd_node_sym_kernel).
extern "C" hipError_t pfml_spd_node_sym(const double* Src, double* X, int64_t ld, int64_t sX,
                                        int batch, int r0, int nn, int* status,
                                        hipStream_t st) {
  if (batch <= 0) return hipSuccess;
  if (nn <= NBL || nn > 2 * NBL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spd_node_sym_kernel, dim3(batch), dim3(256), 0, st, Src, X, ld, sX, r0, nn,
                     status);
  return hipGetLastError();
}

// the phase timestamps of the last node launch's workgroup 0 (16 values; zeros without
// -DPFML_NODE_TIMING)
extern "C" hipError_t pfml_node_timing(unsigned long long* out) {
#ifdef PFML_NODE_TIMING
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_node_ts), 16 * sizeof(unsigned long long));
#else
  for (int i = 0; i < 16; ++i) out[i] = 0;
  return hipSuccess;
#endif
}
