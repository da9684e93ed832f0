// Out-of-sample validation utilities (PFML_hp_reals.py:81-102):
//
//     obj[job, l] = r_t^T beta_l - 1/2 beta_l^T D_t beta_l
//
// for every (g, year, p) cell, every one of its 12 validation months t and all 101 lambdas.
// The reference evaluates 513,888 of these quadratic forms one at a time from Python.  Here a
// job = (cell, month); the kernel computes the GEMM  U = D_t[:n,:n] * B  (B = [beta_l], n x L)
// on fp64 MFMA (upper block triangle only: D_t is symmetric) and folds the two reductions
// into the epilogue, so U never leaves registers.
//
// Tail index: n = p + 1 with p a multiple of 64 (65 .. 513), so the last index would cost a
// 16-wide K step of its own in every row tile and a 64-row tile of its own.  When n - 1 is a
// multiple of BK the tiles cover indices 0 .. n-2 only (K loop included); column n-1 enters
// each row's U in the epilogue (one rank-1 term) and row n-1's own term
// b_{n-1} (r_{n-1} - D_{n-1,n-1} b_{n-1} / 2) is added by the reduce kernel: 1 / 5 fewer
// tile-steps at n = 65, 2 / 15 at 129, 5 / 45 at 257, 9 / 153 at 513.
//
// Tile: 64 rows of D x 112 lambda columns (L <= 112) x 1 (or 2) validation months of one cell
// per 256-thread workgroup (3 per CU); each wave owns 16 rows x 7 MFMA 16x16 accumulators per
// month.  Every workgroup writes a deterministic per-row-tile
// partial; a second tiny kernel sums the partials in a fixed order (bitwise reproducible, no
// float atomics).
#include "common.h"
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int BK = 16, NCOL = 112, NTILE = NCOL / 16, BM = 64, NT = 256, NW = NT / 64;
// Months per workgroup (the host's plan decides, ops/ridge.py quad_plan): 1 by default; 2
// (PFML_QUAD_MM=2) lets the two validation months of one tile share the cell's beta, so every
// beta K-tile staged in LDS feeds two D tiles (half the beta traffic, twice the MFMAs per
// barrier) - measured slower on the headline step (5.90 vs 5.78 ms: 2 instead of 3 resident
// workgroups per CU), kept for the A/B.
// Earlier variants measured slower and removed: 128-row tiles (6.76 vs 6.64 ms per step) and
// a prefetch distance of 2 (1.20 vs 1.33 ms), profiles/r02_quad_pf_ab.json.
// Both operands are staged k-contiguous, as they sit in HBM ([row][k] for D, [lambda][k] for
// beta), with a row stride of BK + 2 = 18 doubles: the coalesced global rows are stored
// without bank conflicts, and a fragment read (16 rows x 2 k per 32-lane group) hits 32
// distinct bank pairs.  (A [k][row] image made every staging store a 16-way conflict.)
constexpr int KS = BK + 2;

// indices the tiles cover (n, or n - 1 when the tail index is split off, see above)
__host__ __device__ __forceinline__ int quad_main(int n) {
  return (n > 1 && (n - 1) % 16 == 0) ? n - 1 : n;
}

struct JobDesc {
  int64_t d_off;     // offset of D_t (P x P, ld ldD)
  int64_t r_off;     // offset of r_t
  int64_t b_off;     // offset of beta block [L][ldB]
  int64_t o_off;     // offset of this job's L utilities in obj
  int n;             // p + 1
  int ptile0;        // first partial slot of this job
};

// MM months x 64 rows of D per 256-thread workgroup (4 waves x 16 rows, 7 MFMA 16x16
// accumulators per month).  Global->register prefetch of the next K step while this one is
// computed from LDS (double-buffered), one barrier per K step; the epilogue's cross-wave sums
// reuse the A staging buffer.
template <int MM>
__global__ __launch_bounds__(NT, MM == 1 ? 3 : 2) void quadform_kernel(
    const double* __restrict__ D, int64_t ldD, const double* __restrict__ R,
    const double* __restrict__ Bt, int64_t ldB, const JobDesc* __restrict__ jobs,
    const int* __restrict__ tile_job, int L, double* __restrict__ partial) {
  __shared__ double As[2][MM][BM][KS];
  __shared__ double Bs[2][NCOL][KS];
  static_assert(MM * NW * NCOL <= 2 * MM * BM * KS, "cross-wave sums must fit in the A buffers");
  double (*red)[NW][NCOL] = reinterpret_cast<double (*)[NW][NCOL]>(&As[0][0][0][0]);

  // tile_job[MM * tile + m] = job << 5 | row tile (month m of the tile; the jobs of one tile
  // share the cell, so n and beta; -1 = no second month: the first is recomputed, not
  // stored).  The host lists the tiles longest-first (all row tiles 0, then all 1, ...: the
  // triangular K loop shrinks with the row tile); the partial slot stays ptile0 + rt.
  const int tile = blockIdx.x;
  int jm[MM];
  bool live[MM];
  int rt = 0;
#pragma unroll
  for (int m = 0; m < MM; ++m) {
    const int tj = tile_job[MM * tile + m];
    live[m] = tj >= 0;
    jm[m] = (live[m] ? tj : tile_job[MM * tile]) >> 5;
    if (m == 0) rt = tj & 31;
  }
  const JobDesc jd0 = jobs[jm[0]];
  const int i0 = rt * BM;
  const int nfull = jd0.n;
  const int n = quad_main(nfull);                 // indices of the tiles and their K loop
  const bool tail = n != nfull;
  const double* Dm[MM];
  const double* rm[MM];
#pragma unroll
  for (int m = 0; m < MM; ++m) {
    const JobDesc jd = jobs[jm[m]];
    Dm[m] = D + jd.d_off;
    rm[m] = R + jd.r_off;
  }
  const double* bt = Bt + jd0.b_off;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;

  double4_t acc[MM][NTILE];
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int q = 0; q < NTILE; ++q) acc[m][q] = double4_t{0.0, 0.0, 0.0, 0.0};

  // D_t is symmetric:  b'Db = sum_I b_I'(D_II b_I + 2 sum_{K>I} D_IK b_K).  A row tile I only
  // walks K >= I, with the diagonal block weighted 1/2, so  acc = U_I / 2  and half the
  // flops and D bytes of the full product are spent.
  constexpr int AQ = (BM * BK) / NT;              // D elements per thread per K step per month
  constexpr int BQ = (NCOL * BK + NT - 1) / NT;   // beta elements per thread per K step
  double ra[MM][AQ], rb[BQ];
  // Loads are unconditional (indices clamped into the matrix) and the masking / diagonal
  // weight is applied when the registers are written to LDS: a load under a branch with its
  // use in the same block made the compiler wait for every D element right after issuing it.
  auto gload = [&](int k0) {
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
      for (int q = 0; q < AQ; ++q) {
        const int e = t + q * NT, i = e / BK, k = e % BK;
        ra[m][q] = Dm[m][(int64_t)min(i0 + i, n - 1) * ldD + min(k0 + k, n - 1)];
      }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int e = min(t + q * NT, NCOL * BK - 1), l = e / BK, k = e % BK;
      rb[q] = bt[(int64_t)min(l, L - 1) * ldB + min(k0 + k, n - 1)];
    }
  };
  auto sstore = [&](int buf, int k0) {
    const double wdiag = (k0 < i0 + BM) ? 0.5 : 1.0;
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
      for (int q = 0; q < AQ; ++q) {
        const int e = t + q * NT, i = e / BK, k = e % BK;
        As[buf][m][i][k] = (i0 + i < n && k0 + k < n) ? wdiag * ra[m][q] : 0.0;
      }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int e = t + q * NT, l = e / BK, k = e % BK;
      if (e < NCOL * BK) Bs[buf][l][k] = (l < L && k0 + k < n) ? rb[q] : 0.0;
    }
  };
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      double a[MM];
#pragma unroll
      for (int m = 0; m < MM; ++m) a[m] = As[buf][m][w * 16 + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
      for (int q = 0; q < NTILE; ++q) {
        const double b = Bs[buf][q * 16 + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
        for (int m = 0; m < MM; ++m) acc[m][q] = mfma_f64_16x16x4(a[m], b, acc[m][q]);
      }
    }
  };
  gload(i0);
  sstore(0, i0);
  __syncthreads();
  int buf = 0;
  for (int k0 = i0;;) {
    const bool more = k0 + BK < n;
    if (more) gload(k0 + BK);
    compute(buf);
    if (!more) break;
    sstore(buf ^ 1, k0 + BK);
    __syncthreads();
    k0 += BK;
    buf ^= 1;
  }
  __syncthreads();                            // red reuses As

  // tail column n: U[i][l] += D[i][n] b_l[n] (K block above every row tile: weight 1)
  if (tail) {
#pragma unroll
    for (int q = 0; q < NTILE; ++q) {
      const int l = min(q * 16 + (lane & 15), L - 1);
      const double bt_l = bt[(int64_t)l * ldB + n];
#pragma unroll
      for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int gi = min(i0 + w * 16 + PFML_F64_CROW(lane, rr), n - 1);
          acc[m][q][rr] = fma(Dm[m][(int64_t)gi * ldD + n], bt_l, acc[m][q][rr]);
        }
    }
  }

  // epilogue: sum over this wave's 16 rows of  beta_l[i] * (r_i - 1/2 U[i][l])
#pragma unroll
  for (int q = 0; q < NTILE; ++q) {
    const int l = q * 16 + (lane & 15);
    double b[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int gi = i0 + w * 16 + PFML_F64_CROW(lane, rr);
      b[rr] = (gi < n && l < L) ? bt[(int64_t)l * ldB + gi] : 0.0;
    }
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      double s = 0.0;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int gi = i0 + w * 16 + PFML_F64_CROW(lane, rr);
        if (gi < n && l < L) s += b[rr] * (rm[m][gi] - acc[m][q][rr]);   // acc = U / 2
      }
      // lanes l, l+16, l+32, l+48 share the column
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 16) red[m][w][l] = s;
    }
  }
  __syncthreads();
  if (t < NCOL) {
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      if (!live[m]) continue;
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < NW; ++q) s += red[m][q][t];
      if (t < L) partial[(int64_t)(jobs[jm[m]].ptile0 + rt) * L + t] = s;
    }
  }
}

// Direct-A form.  A wave's D rows are private to it (16 rows per wave, the tile's four waves
// disjoint), so D needs no LDS staging at all: every lane loads its own MFMA A fragments
// straight from global memory into registers, two K steps ahead (a ring of three 4-double
// fragment sets), and only the beta K-tile - shared by the four waves - goes through LDS.
// That takes the D tile's ds_writes, its masking pass and its place in the per-step vmcnt
// wait out of every step; the D stream (from HBM) has two steps to land.
//   k assignment within a 16-deep step: MFMA slice s takes k = k0 + 4c + s for lane group
//   c = lane >> 4, so lane (r, c) reads D[row r][k0 + 4c .. k0 + 4c + 3] - four consecutive
//   doubles of its row per step - and beta's LDS image is read at the same k.
//   beta image: row l (16 doubles = 32 banks), element k at l * 16 + (k ^ g(l)),
//   g(l) = (m & 3) | ((m & 4) << 1), m = (l >> 1) & 7: the fragment reads (16 rows x 2 lane
//   groups per half-wave) hit all 64 banks, the staging writes 2-way at most.
// Same tile grid, partial slots and epilogue as quadform_kernel<1>; the k summation order
// differs (bits differ from that form, same on every rank count).
__device__ __forceinline__ int qd_swz(int l) {
  const int m = (l >> 1) & 7;
  return (m & 3) | ((m & 4) << 1);
}

__global__ __launch_bounds__(NT, 3) void quadform_direct_kernel(
    const double* __restrict__ D, int64_t ldD, const double* __restrict__ R,
    const double* __restrict__ Bt, int64_t ldB, const JobDesc* __restrict__ jobs,
    const int* __restrict__ tile_job, int L, double* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) double Bs[2][NCOL * BK];
  static_assert(NW * NCOL <= 2 * NCOL * BK, "cross-wave sums must fit in the beta buffers");
  double (*red)[NCOL] = reinterpret_cast<double (*)[NCOL]>(&Bs[0][0]);

  const int tile = blockIdx.x;
  const int tj = tile_job[tile];
  const int jm = tj >> 5, rt = tj & 31;
  const JobDesc jd = jobs[jm];
  const int i0 = rt * BM;
  const int nfull = jd.n;
  const int n = quad_main(nfull);
  const bool tail = n != nfull;
  const double* Dm = D + jd.d_off;
  const double* rm = R + jd.r_off;
  const double* bt = Bt + jd.b_off;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int r = lane & 15, c = lane >> 4;
  const int swz = qd_swz(r);                      // g(16 q + r) = g(r)

  double4_t acc[NTILE];
#pragma unroll
  for (int q = 0; q < NTILE; ++q) acc[q] = double4_t{0.0, 0.0, 0.0, 0.0};

  // this lane's D row (clamped: rows past n feed accumulator rows the epilogue drops)
  const double* drow = Dm + (int64_t)min(i0 + w * 16 + r, n - 1) * ldD;
  double da[3][4];                                 // A fragments of steps s, s + 1, s + 2
  auto dload = [&](int slot, int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) da[slot][u] = drow[min(k0 + 4 * c + u, n - 1)];
  };
  constexpr int BQ = (NCOL * BK) / NT;             // 7 beta elements per thread per step
  double rb[BQ];
  auto bload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int e = t + q * NT, l = e / BK, k = e % BK;
      rb[q] = bt[(int64_t)min(l, L - 1) * ldB + min(k0 + k, n - 1)];
    }
  };
  auto bstore = [&](int buf, int k0) {
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int e = t + q * NT, l = e / BK, k = e % BK;
      Bs[buf][l * BK + (k ^ qd_swz(l))] = (l < L && k0 + k < n) ? rb[q] : 0.0;
    }
  };

  const int nst = (n - i0 + BK - 1) / BK;          // K steps of this row tile
  bload(i0);
  dload(0, i0);
  if (nst > 1) dload(1, i0 + BK);
  bstore(0, i0);
  __syncthreads();
  // one K step; SLOT = st % 3 as a compile-time constant (the fragment ring stays in
  // registers: the step loop below is unrolled by three)
  auto step = [&](auto slot_c, int st) -> bool {
    constexpr int cur = decltype(slot_c)::value;
    const int k0 = i0 + st * BK;
    const int buf = st & 1;
    const bool more = st + 1 < nst;
    // beta of the next step first, then D two steps ahead: the end-of-step wait for beta
    // leaves the D loads in flight (vmcnt counts in issue order)
    if (more) bload(k0 + BK);
    if (st + 2 < nst) dload((cur + 2) % 3, k0 + 2 * BK);
    // the diagonal block (k < i0 + 64) weighted 1/2: acc = U / 2 (see quadform_kernel)
    const double wd = (k0 < i0 + BM) ? 0.5 : 1.0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = k0 + 4 * c + s;
      const double a = (k < n) ? wd * da[cur][s] : 0.0;
#pragma unroll
      for (int q = 0; q < NTILE; ++q) {
        const double b = Bs[buf][(q * 16 + r) * BK + ((4 * c + s) ^ swz)];
        acc[q] = mfma_f64_16x16x4(a, b, acc[q]);
      }
    }
    if (!more) return false;
    bstore(buf ^ 1, k0 + BK);
    __syncthreads();
    return true;
  };
  for (int st = 0;; st += 3) {
    if (!step(std::integral_constant<int, 0>{}, st)) break;
    if (!step(std::integral_constant<int, 1>{}, st + 1)) break;
    if (!step(std::integral_constant<int, 2>{}, st + 2)) break;
  }
  __syncthreads();                                 // red reuses Bs

  if (tail) {
#pragma unroll
    for (int q = 0; q < NTILE; ++q) {
      const int l = min(q * 16 + (lane & 15), L - 1);
      const double bt_l = bt[(int64_t)l * ldB + n];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int gi = min(i0 + w * 16 + PFML_F64_CROW(lane, rr), n - 1);
        acc[q][rr] = fma(Dm[(int64_t)gi * ldD + n], bt_l, acc[q][rr]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NTILE; ++q) {
    const int l = q * 16 + (lane & 15);
    double s = 0.0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int gi = i0 + w * 16 + PFML_F64_CROW(lane, rr);
      if (gi < n && l < L) s += bt[(int64_t)l * ldB + gi] * (rm[gi] - acc[q][rr]);
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (lane < 16) red[w][l] = s;
  }
  __syncthreads();
  if (t < L) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += red[q][t];
    partial[(int64_t)(jd.ptile0 + rt) * L + t] = s;
  }
}

__global__ void quadform_reduce_kernel(const double* __restrict__ partial,
                                       const JobDesc* __restrict__ jobs, int njobs, int L,
                                       const double* __restrict__ D, int64_t ldD,
                                       const double* __restrict__ R,
                                       const double* __restrict__ Bt, int64_t ldB,
                                       double* __restrict__ obj) {
  const int j = blockIdx.x;
  const int l = threadIdx.x;
  if (j >= njobs || l >= L) return;
  const JobDesc jd = jobs[j];
  const int n = quad_main(jd.n);
  const int nt = (n + BM - 1) / BM;
  double s = 0.0;
  for (int q = 0; q < nt; ++q) s += partial[(int64_t)(jd.ptile0 + q) * L + l];
  if (n != jd.n) {                              // the tail row's own term
    const double b = Bt[jd.b_off + (int64_t)l * ldB + n];
    s += b * (R[jd.r_off + n] - 0.5 * D[jd.d_off + (int64_t)n * ldD + n] * b);
  }
  obj[jd.o_off + l] = s;
}

}  // namespace

extern "C" int pfml_quadform_job_desc_size() { return (int)sizeof(JobDesc); }
extern "C" int pfml_quadform_rows_per_tile() { return BM; }
extern "C" int pfml_quadform_row_tiles(int n) { return (quad_main(n) + BM - 1) / BM; }

// tile_job: mm (1 or 2; 1 for the direct form, mm = 3) int32 entries per tile.
extern "C" hipError_t pfml_quadform(const double* D, int64_t ldD, const double* R,
                                    const double* Bt, int64_t ldB, const void* jobs, int njobs,
                                    const int* tile_job, int ntiles, int mm, int L,
                                    double* partial, double* obj, hipStream_t st) {
  if (njobs <= 0) return hipSuccess;
  // mm: months per tile (1 / 2); 3 = the direct-A form on the one-month tile list
  if (L > NCOL || mm < 1 || mm > 3) return hipErrorInvalidValue;
  const JobDesc* jd = static_cast<const JobDesc*>(jobs);
  if (mm == 3)
    hipLaunchKernelGGL(quadform_direct_kernel, dim3(ntiles), dim3(NT), 0, st, D, ldD, R, Bt, ldB,
                       jd, tile_job, L, partial);
  else if (mm == 2)
    hipLaunchKernelGGL(quadform_kernel<2>, dim3(ntiles), dim3(NT), 0, st, D, ldD, R, Bt, ldB, jd,
                       tile_job, L, partial);
  else
    hipLaunchKernelGGL(quadform_kernel<1>, dim3(ntiles), dim3(NT), 0, st, D, ldD, R, Bt, ldB, jd,
                       tile_job, L, partial);
  hipLaunchKernelGGL(quadform_reduce_kernel, dim3(njobs), dim3(128), 0, st, partial, jd, njobs, L,
                     D, ldD, R, Bt, ldB, obj);
  return hipGetLastError();
}
