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
// Large-block variant: the NBL x NBL pivot block (NBL = 128) is inverted in LDS by one
// 1024-thread workgroup per matrix; the row panel, the rank-NBL trailing update and the
// column panel are then plain batched GEMMs on pfml_dgemm (host orchestration in
// ops/linalg.py), so each block step is one MFMA-bound pass over the matrix instead of the
// four bandwidth-bound passes of the NB = 32 kernels above.
namespace {
constexpr int NBL = 64;

template <int NBT>
__global__ __launch_bounds__(256) void spd_blockinv_kernel(const double* __restrict__ A,
                                                            int64_t lda, int64_t sA, int k0,
                                                            int nb, double* __restrict__ Pout,
                                                            int* __restrict__ status) {
  __shared__ double P[NBT][NBT + 1];
  constexpr int EPT = NBT * NBT / 256;            // elements per thread (fixed NBT^2 frame)
  const int b = blockIdx.x;
  const double* Ab = A + (int64_t)b * sA + (int64_t)k0 * lda + k0;
  const int t = threadIdx.x;
  // element u of this thread: (i, j) = (e / NBT, e % NBT), e = t + 256 u; frame entries past
  // nb hold the identity, so the elimination below needs no bounds tests
  {
    double v[EPT];
#pragma unroll
    for (int u = 0; u < EPT; ++u) {            // every load in flight at once
      const int e = t + 256 * u, i = e / NBT, j = e % NBT;
      v[u] = Ab[(int64_t)min(i, nb - 1) * lda + min(j, nb - 1)];
    }
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = t + 256 * u, i = e / NBT, j = e % NBT;
      P[i][j] = (i < nb && j < nb) ? v[u] : (i == j ? 1.0 : 0.0);
    }
  }
  __syncthreads();
  for (int p = 0; p < nb; ++p) {
    // P[p][p], P[i][p], P[p][j] are only rewritten after the next barrier, so reading the
    // pivot needs no barrier of its own
    const double piv = P[p][p];
    if (t == 0 && (!(piv > 0.0) || !isfinite(piv))) status[b] = 1;
    const double inv = 1.0 / piv;
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = t + 256 * u, i = e / NBT, j = e % NBT;
      if (i != p && j != p) P[i][j] -= P[i][p] * P[p][j] * inv;
    }
    __syncthreads();
    if (t < NBT && t != p) {
      P[p][t] *= inv;
      P[t][p] *= -inv;
    }
    if (t == 0) P[p][p] = inv;
    __syncthreads();
  }
  double* Pb = Pout + (int64_t)b * NBT * NBT;
#pragma unroll
  for (int u = 0; u < EPT; ++u) {
    const int e = t + 256 * u, i = e / NBT, j = e % NBT;
    if (i < nb && j < nb) Pb[i * NBT + j] = P[i][j];
  }
}
}  // namespace

extern "C" hipError_t pfml_spd_blockinv128(const double* A, int64_t lda, int64_t sA, int batch,
                                           int k0, int nb, double* Pout, int* status,
                                           hipStream_t st) {
  if (batch <= 0 || nb <= 0) return hipSuccess;
  if (nb > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spd_blockinv_kernel<128>, dim3(batch), dim3(256), 0, st, A, lda, sA, k0, nb,
                     Pout, status);
  return hipGetLastError();
}

namespace {
// Register-resident 64 x 64 Gauss-Jordan inverse (no pivoting: SPD blocks), 4 pivots per
// barrier.  The LDS form above re-reads and re-writes the whole block from LDS at every pivot
// (LDS-bandwidth bound, ~80 us per batch of 256 blocks) and a one-pivot register form is
// bound by its 64 barrier + divide round trips (~50 us).  Here each of the 256 threads keeps a
// 4 x 4 sub-block in registers; pivot block q (4 pivots) is exactly thread row / column block
// q, so the owners publish whole register tiles to a double-buffered LDS line
// (one barrier per step, no second barrier: the buffer written at step q + 2 is rewritten
// only after every thread has passed step q + 1's barrier, i.e. finished reading it).  Frame
// entries past nb hold the identity, so partial blocks need no special case.  Output to any
// (ld, batch stride): in place (Pout = the block itself) or to a packed buffer.
__global__ __launch_bounds__(256) void spd_leafinv_kernel(const double* __restrict__ A,
                                                          int64_t lda, int64_t sA, int k0,
                                                          int nb, double* Pout, int64_t ldp,
                                                          int64_t sP, int* __restrict__ status) {
  __shared__ double rowb[2][4][64], colb[2][64][4];
  const int b = blockIdx.x, t = threadIdx.x;
  const int rb = t >> 4, cb = t & 15;
  const double* Ab = A + (int64_t)b * sA + (int64_t)k0 * lda + k0;
  double a[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * rb + u, j = 4 * cb + v;
      a[u][v] = Ab[(int64_t)min(i, nb - 1) * lda + min(j, nb - 1)];
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
        for (int v = 0; v < 4; ++v) rowb[buf][r][4 * cb + v] = a[r][v];
    }
    if (cb == q) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) colb[buf][4 * rb + u][c] = a[u][c];
    }
    __syncthreads();
    // The 4 pivots of the block, replayed as SCALAR Gauss-Jordan steps on the thread's local
    // 8 x 8 view M = [[P, rp], [cp, a]] (P = A_KK, rp = A_K,mycols, cp = A_myrows,K): every
    // entry sees exactly the update sequence, and the expressions, of one-pivot-at-a-time GJ,
    // so the result is bitwise that of the LDS kernel (an explicit P^-1 block step amplifies
    // rounding by cond(P) on ill-conditioned Denman-Beavers iterates).
    double P[4][4], rp[4][4], cp[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) P[r][c] = rowb[buf][r][4 * q + c];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int v = 0; v < 4; ++v) rp[r][v] = rowb[buf][r][4 * cb + v];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) cp[u][c] = colb[buf][4 * rb + u][c];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const double piv = P[p][p];
      bad |= !(piv > 0.0) || !isfinite(piv);
      const double inv = 1.0 / piv;
      // a (rows != p, cols != p: always, the thread's rows / cols are outside K unless it
      // owns the pivot block, whose result is then read from P / rp / cp below)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) a[u][v] -= cp[u][p] * rp[p][v] * inv;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r != p)
#pragma unroll
          for (int v = 0; v < 4; ++v) rp[r][v] -= P[r][p] * rp[p][v] * inv;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c != p) cp[u][c] -= cp[u][p] * P[p][c] * inv;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (r != p && c != p) P[r][c] -= P[r][p] * P[p][c] * inv;
      // pivot row / column scaling (old values of row p / column p used above)
#pragma unroll
      for (int v = 0; v < 4; ++v) rp[p][v] *= inv;
#pragma unroll
      for (int u = 0; u < 4; ++u) cp[u][p] *= -inv;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c != p) {
          P[p][c] *= inv;
          P[c][p] *= -inv;
        }
      P[p][p] = inv;
    }
    const bool inr = rb == q, inc = cb == q;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        a[u][v] = (inr && inc) ? P[u][v] : (inr ? rp[u][v] : (inc ? cp[u][v] : a[u][v]));
  }
  if (t == 0 && bad) status[b] = 1;
  double* Pb = Pout + (int64_t)b * sP;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * rb + u, j = 4 * cb + v;
      if (i < nb && j < nb) Pb[(int64_t)i * ldp + j] = a[u][v];
    }
}
}  // namespace

extern "C" int pfml_spd_block_size() { return NBL; }

extern "C" hipError_t pfml_spd_blockinv(const double* A, int64_t lda, int64_t sA, int batch,
                                        int k0, int nb, double* Pout, int* status,
                                        hipStream_t st) {
  if (batch <= 0 || nb <= 0) return hipSuccess;
  if (nb > NBL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spd_leafinv_kernel, dim3(batch), dim3(256), 0, st, A, lda, sA, k0, nb, Pout,
                     (int64_t)NBL, (int64_t)NBL * NBL, status);
  return hipGetLastError();
}

// Inverse of the nb x nb (nb <= 64) diagonal block at (k0, k0) of A written to the block at
// (k0, k0) of P (any leading dims / batch strides; P == A: in place).
extern "C" hipError_t pfml_spd_leafinv_to(const double* A, int64_t lda, int64_t sA, double* P,
                                          int64_t ldp, int64_t sP, int batch, int k0, int nb,
                                          int* status, hipStream_t st) {
  if (batch <= 0 || nb <= 0) return hipSuccess;
  if (nb > NBL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spd_leafinv_kernel, dim3(batch), dim3(256), 0, st, A, lda, sA, k0, nb,
                     P + (int64_t)k0 * ldp + k0, ldp, sP, status);
  return hipGetLastError();
}

// In-place inverse of the nb x nb (nb <= 64) diagonal block at (k0, k0) of each matrix.
extern "C" hipError_t pfml_spd_leafinv_inplace(double* A, int64_t lda, int64_t sA, int batch,
                                               int k0, int nb, int* status, hipStream_t st) {
  if (batch <= 0 || nb <= 0) return hipSuccess;
  if (nb > NBL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spd_leafinv_kernel, dim3(batch), dim3(256), 0, st, A, lda, sA, k0, nb,
                     A + (int64_t)k0 * lda + k0, lda, sA, status);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Fused symmetric block step (the production path for n >= 160).  For SPD A, blocked
// Gauss-Jordan keeps the working matrix "sign-symmetric": with s_i = -1 on rows of blocks
// already eliminated (i < k0) and +1 elsewhere, A_ij = s_i s_j A_ji.  So the old column
// panel of block K is C = diag(s) W^T with W = A[K, :] (the row panel), and the new column
// panel -C P is -diag(s) R^T with R = P W.  One step is then three launches:
//   spd_blockinv_kernel   P = A_KK^-1                                  (LDS Gauss-Jordan)
//   gjs_prep_kernel        W = A[K, :] (snapshot), R = P W              (MFMA, one 64-col tile)
//   gjs_update_kernel      every 64 x 64 tile of A, one read-modify-write:
//        i, j outside K : A_ij -= s_i sum_k W_ki R_kj                  (MFMA, rank nb)
//        i in K, j out  : A_ij  = R_(i-k0) j
//        i out, j in K  : A_ij  = -s_i R_(j-k0) i
//        i, j in K      : A_ij  = P
// instead of the seven (block inverse, three GEMMs, three copies) of the generic form.
namespace {
constexpr int GT = 64;          // tile = block width (NBL)
constexpr int GK = 16;          // k chunk streamed through LDS
constexpr int GS = GT + 16;     // [k][idx] LDS row stride (MFMA fragment reads conflict-free)

// C_tile += op(X)[:, k-chunk] * Y[k-chunk, :] for a 64 x 64 tile, operands staged [k][idx]
// in 16-deep chunks (20 KB of LDS: several workgroups per CU hide each other's latency).
// Loads of chunk c+1 are issued before the MFMAs of chunk c; the mask / sign is applied at
// the LDS store (after the MFMAs), so the loads stay in flight across them.
template <typename PtrX, typename PtrY, typename MaskX, typename MaskY>
__device__ __forceinline__ void gjs_tile_mma(double4_t (&acc)[2][2], int nk, PtrX px, PtrY py,
                                             MaskX mx, MaskY my, double (*Xs)[GK][GS],
                                             double (*Ys)[GK][GS]) {
  constexpr int Q = GK * GT / 256;       // 4 elements of each operand per thread per chunk
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1, li = lane & 15, lk = lane >> 4;
  double xv[Q], yv[Q];
  // raw loads from always-valid (clamped) addresses; nothing consumes them before the MFMAs
  auto load = [&](int c) {
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      const int e = t + u * 256, k = c * GK + e / GT, i = e % GT;
      xv[u] = *px(k, i);
      yv[u] = *py(k, i);
    }
  };
  auto store = [&](int c, int buf) {
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      const int e = t + u * 256, k = c * GK + e / GT, i = e % GT;
      Xs[buf][e / GT][i] = xv[u] * mx(k, i);
      Ys[buf][e / GT][i] = yv[u] * my(k, i);
    }
  };
  load(0);
  store(0, 0);
  __syncthreads();
  for (int c = 0; c < nk; ++c) {
    const int cur = c & 1;
    if (c + 1 < nk) load(c + 1);
#pragma unroll
    for (int k = 0; k < GK; k += 4) {
      double a[2], bb[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) a[x] = Xs[cur][k + lk][wm * 32 + x * 16 + li];
#pragma unroll
      for (int y = 0; y < 2; ++y) bb[y] = Ys[cur][k + lk][wn * 32 + y * 16 + li];
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = mfma_f64_16x16x4(a[x], bb[y], acc[x][y]);
    }
    if (c + 1 < nk) store(c + 1, cur ^ 1);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void gjs_prep_kernel(const double* __restrict__ A, int n,
                                                       int64_t sA, int k0, int nb,
                                                       const double* __restrict__ Pbuf,
                                                       double* __restrict__ Wbuf,
                                                       double* __restrict__ Rbuf) {
  __shared__ double Xs[2][GK][GS], Ys[2][GK][GS];
  const int b = blockIdx.y, j0 = blockIdx.x * GT;
  const double* Ab = A + (int64_t)b * sA;
  const double* Pb = Pbuf + (int64_t)b * GT * GT;
  double* Wb = Wbuf + (int64_t)b * GT * n;
  double* Rb = Rbuf + (int64_t)b * GT * n;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1, li = lane & 15;
  // snapshot W = A[K, j0..j0+63] (row panel, coalesced)
  for (int e = t; e < GT * GT; e += 256) {
    const int k = e / GT, j = j0 + e % GT;
    if (k < nb && j < n) Wb[(int64_t)k * n + j] = Ab[(int64_t)(k0 + k) * n + j];
  }
  double4_t acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = double4_t{0.0, 0.0, 0.0, 0.0};
  // R = P W: X operand P^T[k][i] = P[i][k] (P symmetric: read P[k][i]), Y = W[k][j]
  auto px = [&](int k, int i) { return Pb + min(k, nb - 1) * GT + min(i, nb - 1); };
  auto py = [&](int k, int j) {
    return Ab + (int64_t)(k0 + min(k, nb - 1)) * n + min(j0 + j, n - 1);
  };
  auto mx = [&](int k, int i) { return (k < nb && i < nb) ? 1.0 : 0.0; };
  auto my = [&](int k, int j) { return (k < nb && j0 + j < n) ? 1.0 : 0.0; };
  gjs_tile_mma(acc, (nb + GK - 1) / GK, px, py, mx, my, Xs, Ys);
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = wm * 32 + x * 16 + PFML_F64_CROW(lane, r);
        const int j = j0 + wn * 32 + y * 16 + li;
        if (i < nb && j < n) Rb[(int64_t)i * n + j] = acc[x][y][r];
      }
}

__global__ __launch_bounds__(256) void gjs_update_kernel(double* __restrict__ A, int n, int64_t sA,
                                                         int k0, int nb,
                                                         const double* __restrict__ Pbuf,
                                                         const double* __restrict__ Wbuf,
                                                         const double* __restrict__ Rbuf) {
  __shared__ double Xs[2][GK][GS], Ys[2][GK][GS];
  const int tiles = (n + GT - 1) / GT;
  const int b = blockIdx.y;
  const int I0 = (blockIdx.x / tiles) * GT, J0 = (blockIdx.x % tiles) * GT;
  double* Ab = A + (int64_t)b * sA;
  const double* Pb = Pbuf + (int64_t)b * GT * GT;
  const double* Wb = Wbuf + (int64_t)b * GT * n;
  const double* Rb = Rbuf + (int64_t)b * GT * n;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1, li = lane & 15;
  double4_t acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = double4_t{0.0, 0.0, 0.0, 0.0};
  // A_ij -= s_i sum_k W_ki R_kj  (s_i = -1 on rows of eliminated blocks)
  auto px = [&](int k, int i) { return Wb + (int64_t)min(k, nb - 1) * n + min(I0 + i, n - 1); };
  auto py = [&](int k, int j) { return Rb + (int64_t)min(k, nb - 1) * n + min(J0 + j, n - 1); };
  auto mx = [&](int k, int i) {
    const int gi = I0 + i;
    return (k < nb && gi < n) ? (gi < k0 ? -1.0 : 1.0) : 0.0;
  };
  auto my = [&](int k, int j) { return (k < nb && J0 + j < n) ? 1.0 : 0.0; };
  gjs_tile_mma(acc, (nb + GK - 1) / GK, px, py, mx, my, Xs, Ys);
  // epilogue: gather the old values first (one memory latency for the tile), then write
  double old[2][2][4];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = min(I0 + wm * 32 + x * 16 + PFML_F64_CROW(lane, r), n - 1);
        const int j = min(J0 + wn * 32 + y * 16 + li, n - 1);
        old[x][y][r] = Ab[(int64_t)i * n + j];
      }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = I0 + wm * 32 + x * 16 + PFML_F64_CROW(lane, r);
        const int j = J0 + wn * 32 + y * 16 + li;
        if (i >= n || j >= n) continue;
        const bool ik = (i >= k0 && i < k0 + nb), jk = (j >= k0 && j < k0 + nb);
        double v;
        if (!ik && !jk) v = old[x][y][r] - acc[x][y][r];
        else if (ik && !jk) v = Rb[(int64_t)(i - k0) * n + j];
        else if (!ik && jk) v = (i < k0 ? 1.0 : -1.0) * Rb[(int64_t)(j - k0) * n + i];
        else v = Pb[(i - k0) * GT + (j - k0)];
        Ab[(int64_t)i * n + j] = v;
      }
}
}  // namespace

extern "C" int64_t pfml_spd_inverse_sym_work_doubles(int n, int batch) {
  return (int64_t)batch * (GT * GT + 2LL * GT * n);
}

// In-place inverse of `batch` contiguous n x n SPD matrices (batch stride n*n) by the fused
// symmetric block steps above.  status: set to 1 for a matrix that met a non-positive pivot.
extern "C" hipError_t pfml_spd_inverse_sym(double* A, int n, int batch, double* work,
                                           int* status, hipStream_t st) {
  if (n <= 0 || batch <= 0) return hipSuccess;
  const int64_t sA = (int64_t)n * n;
  double* Pbuf = work;
  double* Wbuf = Pbuf + (int64_t)batch * GT * GT;
  double* Rbuf = Wbuf + (int64_t)batch * GT * n;
  const int tiles = (n + GT - 1) / GT;
  for (int k0 = 0; k0 < n; k0 += GT) {
    const int nb = (n - k0 < GT) ? (n - k0) : GT;
    hipLaunchKernelGGL(spd_blockinv_kernel<NBL>, dim3(batch), dim3(256), 0, st, A, (int64_t)n, sA,
                       k0, nb, Pbuf, status);
    hipLaunchKernelGGL(gjs_prep_kernel, dim3(tiles, batch), dim3(256), 0, st, A, n, sA, k0, nb,
                       Pbuf, Wbuf, Rbuf);
    hipLaunchKernelGGL(gjs_update_kernel, dim3(tiles * tiles, batch), dim3(256), 0, st, A, n, sA,
                       k0, nb, Pbuf, Wbuf, Rbuf);
  }
  return hipGetLastError();
}
