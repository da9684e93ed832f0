// Host-side native runtime for the panel-preparation and risk-model stages.
//
// The reference runs these as pandas group-wise Python loops (the per-id universe state
// machine is an explicit Python for-loop executed twice per id, General_functions.py:621-634;
// the EWMA idiosyncratic vol is a numba @njit kernel, Estimate Covariance Matrix.py:345-386).
// They are sequential per group, touch each row once and are a one-shot cost, so they live in
// C++ on the host (OpenMP over groups) rather than on the GPU; the EWMA scan has a HIP
// counterpart (csrc/risk.hip) used when the daily residual panel is device-resident.
//
// All entry points take rows sorted by (group, time) and a CSR-style group_start array of
// length ngroups + 1.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <numeric>
#include <vector>

extern "C" {

// Universe membership (General_functions.py:507-548): enter on a rising edge of `add`, leave
// on `del`; the first row of every group is never included.
void pfml_investment_universe(const uint8_t* add, const uint8_t* del, const int64_t* gs,
                              int64_t ngroups, uint8_t* out) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t g = 0; g < ngroups; ++g) {
    const int64_t a = gs[g], b = gs[g + 1];
    if (b - a < 2) {
      for (int64_t i = a; i < b; ++i) out[i] = 0;
      continue;
    }
    bool state = false;
    out[a] = 0;
    for (int64_t i = a + 1; i < b; ++i) {
      if (!state && add[i] && !add[i - 1]) state = true;
      else if (state && del[i]) state = false;
      out[i] = state ? 1 : 0;
    }
  }
}

// Rolling sum over `window` rows within each group; NaN until the window is full
// (pandas rolling(window, min_periods=window).sum()).
void pfml_rolling_sum(const double* x, const int64_t* gs, int64_t ngroups, int window,
                      double* out) {
  const double nan = std::numeric_limits<double>::quiet_NaN();
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t g = 0; g < ngroups; ++g) {
    const int64_t a = gs[g], b = gs[g + 1];
    double s = 0.0;
    for (int64_t i = a; i < b; ++i) {
      s += x[i];
      if (i - a >= window) s -= x[i - window];
      out[i] = (i - a + 1 >= window) ? s : nan;
    }
  }
}

// Percentile rank within segments, pandas rank(method="average", pct=True): NaNs stay NaN and
// are excluded from the count; ties get the average of their ordinal ranks; pct = rank / n.
// x is column-major [ncol][nrows]; segments index rows.
void pfml_pct_rank(const double* x, int64_t nrows, int64_t ncol, const int64_t* ss,
                   int64_t nseg, double* out) {
  const double nan = std::numeric_limits<double>::quiet_NaN();
#pragma omp parallel
  {
    std::vector<int64_t> idx;
#pragma omp for collapse(2) schedule(dynamic, 16)
    for (int64_t c = 0; c < ncol; ++c)
      for (int64_t s = 0; s < nseg; ++s) {
        const double* col = x + c * nrows;
        double* oc = out + c * nrows;
        const int64_t a = ss[s], b = ss[s + 1];
        idx.clear();
        for (int64_t i = a; i < b; ++i) {
          if (std::isnan(col[i])) oc[i] = nan;
          else idx.push_back(i);
        }
        std::stable_sort(idx.begin(), idx.end(),
                         [col](int64_t p, int64_t q) { return col[p] < col[q]; });
        const double n = (double)idx.size();
        size_t k = 0;
        while (k < idx.size()) {
          size_t e = k + 1;
          while (e < idx.size() && col[idx[e]] == col[idx[k]]) ++e;
          const double avg = 0.5 * ((double)(k + 1) + (double)e);   // mean of ranks k+1..e
          for (size_t q = k; q < e; ++q) oc[idx[q]] = avg / n;
          k = e;
        }
      }
  }
}

// Percentile ranks of a row-major panel X [nrows, ncol] within segments of a row permutation
// (Prepare_Data.py:324-374: groupby(eom).rank(pct=True) per feature): segment s holds the rows
// perm[ss[s] .. ss[s+1]).  One task per segment gathers its rows once (contiguous row reads),
// ranks every column (average ties / non-NaN count) and writes out[row][c] in the original row
// order - no transposes or reordered copies of the panel.  zero_keep: exact zeros rank 0 (quirk
// Q15); impute (not NaN): NaN ranks take that value.
// Element (r, c) of X / out at r * rs + c * cs (row- or column-major, no reordered copy).
void pfml_pct_rank_rows(const double* X, int64_t nrows, int64_t ncol, int64_t xrs, int64_t xcs,
                        const int64_t* perm, const int64_t* ss, int64_t nseg, int zero_keep,
                        double impute, double* out, int64_t ors, int64_t ocs) {
  (void)nrows;
  const double nan = std::numeric_limits<double>::quiet_NaN();
  const bool imp = !std::isnan(impute);
#pragma omp parallel
  {
    std::vector<double> buf;                       // [ncol][m] column-major segment copy
    std::vector<double> res;
    std::vector<int32_t> idx;
#pragma omp for schedule(dynamic, 4)
    for (int64_t s = 0; s < nseg; ++s) {
      const int64_t a = ss[s], m = ss[s + 1] - a;
      if (m <= 0) continue;
      buf.resize((size_t)(m * ncol));
      res.resize((size_t)(m * ncol));
      for (int64_t i = 0; i < m; ++i) {
        const double* row = X + perm[a + i] * xrs;
        for (int64_t c = 0; c < ncol; ++c) buf[c * m + i] = row[c * xcs];
      }
      for (int64_t c = 0; c < ncol; ++c) {
        const double* col = buf.data() + c * m;
        double* rc = res.data() + c * m;
        idx.clear();
        for (int64_t i = 0; i < m; ++i) {
          if (std::isnan(col[i])) rc[i] = imp ? impute : nan;
          else idx.push_back((int32_t)i);
        }
        std::stable_sort(idx.begin(), idx.end(),
                         [col](int32_t p, int32_t q) { return col[p] < col[q]; });
        const double n = (double)idx.size();
        size_t k = 0;
        while (k < idx.size()) {
          size_t e = k + 1;
          while (e < idx.size() && col[idx[e]] == col[idx[k]]) ++e;
          const double avg = 0.5 * ((double)(k + 1) + (double)e);   // mean of ranks k+1..e
          const double r = (zero_keep && col[idx[k]] == 0.0) ? 0.0 : avg / n;
          for (size_t q = k; q < e; ++q) rc[idx[q]] = r;
          k = e;
        }
      }
      for (int64_t i = 0; i < m; ++i) {
        double* orow = out + perm[a + i] * ors;
        for (int64_t c = 0; c < ncol; ++c) orow[c * ocs] = res[c * m + i];
      }
    }
  }
}

// Zero-mean EWMA volatility (numba ewma_vol, Estimate Covariance Matrix.py:345-386):
// var[start] = sum(x[:start]^2 over non-NaN) / (count - 1); then
// var[i] = lam var[i-1] + (1-lam) x[i-1]^2, carrying var forward over NaN x[i-1].
// Output NaN before `start` and for groups with <= start rows or count <= 1.
void pfml_ewma_vol(const double* x, const int64_t* gs, int64_t ngroups, double lam, int start,
                   double* out) {
  const double nan = std::numeric_limits<double>::quiet_NaN();
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t g = 0; g < ngroups; ++g) {
    const int64_t a = gs[g], b = gs[g + 1], n = b - a;
    for (int64_t i = a; i < b; ++i) out[i] = nan;
    if (n <= start) continue;
    double ss = 0.0;
    int64_t cnt = 0;
    for (int64_t i = a; i < a + start; ++i)
      if (!std::isnan(x[i])) { ss += x[i] * x[i]; ++cnt; }
    if (cnt <= 1) continue;
    double var = ss / (double)(cnt - 1);
    out[a + start] = std::sqrt(var);
    for (int64_t i = a + start + 1; i < b; ++i) {
      const double xp = x[i - 1];
      if (!std::isnan(xp)) var = lam * var + (1.0 - lam) * xp * xp;
      out[i] = std::sqrt(var);
    }
  }
}

// Group boundaries of a sorted key array: gs[0] = 0, gs[k] = first row of group k, gs[ng] = n.
int64_t pfml_group_starts(const int64_t* key, int64_t n, int64_t* gs) {
  int64_t ng = 0;
  for (int64_t i = 0; i < n; ++i)
    if (i == 0 || key[i] != key[i - 1]) gs[ng++] = i;
  gs[ng] = n;
  return ng;
}

// Shift within groups: out[i] = x[i - k] if row i-k is in the same group, else NaN.
void pfml_group_shift(const double* x, const int64_t* gs, int64_t ngroups, int64_t k,
                      double* out) {
  const double nan = std::numeric_limits<double>::quiet_NaN();
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t g = 0; g < ngroups; ++g) {
    const int64_t a = gs[g], b = gs[g + 1];
    for (int64_t i = a; i < b; ++i) {
      const int64_t j = i - k;
      out[i] = (j >= a && j < b) ? x[j] : nan;
    }
  }
}

}  // extern "C"
