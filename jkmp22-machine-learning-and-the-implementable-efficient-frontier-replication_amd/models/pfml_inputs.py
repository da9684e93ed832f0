"""L4 PFML inputs (PFML_Input_Data.py): r_tilde_t, risk_t, tc_t, denom_t of (25) per month.

The reference's hot loop (:318-491, 1.6-2.6 s per month on 8 CPU cores, pandas-bound) becomes
a batched device pipeline over MONTHS (dates are independent given m_t, Sigma_t and the
13-month signal window) and over g (the g-dependent part is only the signal block):

1. RFF features for the whole panel: ONE fused GEMM launch per g whose epilogue writes
   cos / sin of X W (K13) in the interleaved order [constant, cos1, sin1, ...];
2. vol scales sqrt(diag(Sigma_t)) = sqrt(rowsum((X F) o X) + ivol) per Barra row on the
   device, without forming Sigma (:274-307), NaN filled with the month's median (pandas
   semantics: mean of the two middle values), on the device;
3. per batch of months (ragged universes padded block-diagonally):
   * signals: gather the 13 x N x P window, demean RFF columns, unit-norm every column, scale
     rows by 1/vol (K11/K12, :357-391) - stored for lags 0, 11, 12 only; lags 1..10 are
     formed in the epilogue of the Horner step that consumes them from their column
     statistics (a gathered addend: (F[row] - mean) * scale / vol), never stored;
   * Sigma_t = X F X' + diag(ivol) as one GEMM with a diagonal-add epilogue (K1) and
     m_tilde_t (K2/K3, Lemma 1, ops/linalg.m_tilde: fused symmetric passes + SPD inverses, no
     host sync);
   * the aggregation (24) in Horner form over the augmented [S_{t-theta} | I] (K5/K6):
       T_11 = [S_11 | I],  T_theta = [S_theta | I] + (m D_theta) T_{theta+1}
     gives both sum_theta agg_theta S_{t-theta} and sum_theta agg_theta in 11 GEMMs (the
     reference forms 22 N x N products plus 24 N x P products), with both g stacked in the
     column dimension so m and the agg products are shared; the lag-1 sums of omega_l1 follow
     as T_1 + (m D_1 ... m D_11) [S_12 | I], the product carried along the same launches.  Each step is ONE launch of
     the fused GEMM (csrc/gemm_f64.hip): m = diag(a) m_tilde diag(1/a) and D_theta enter as
     row / k scales, S_theta and the identity block as the epilogue addend - no m, m D or
     [S | I] matrix is ever materialised;
   * omega = const^-1 Omega (pivoted LU solve, K7), omega_chg = omega - D_0 omega_l1;
   * r_tilde = omega' r, risk = gamma omega' Sigma omega (Sigma applied in low-rank form),
     tc = w omega_chg' Lambda omega_chg, denom = risk + tc (K8-K10).

Output: ``PfmlReals`` (search.py) + per-month signals signal_t (all in internal feature
order; ``config.interleaved_order`` maps to the reference's feat_all).
"""
from __future__ import annotations

from dataclasses import dataclass

import contextlib
import os

import numpy as np
import pandas as pd
import torch

from ..config import Config, get_features, interleaved_order
from ..data import io
from ..ops import linalg as la
from ..ops.gemm import gemm, gemm_fused, gemm_prec
from ..ops.panel import (date_sums, excl_stats, rff_features, signal_stats,
                         standardize_signals)
from ..utils.dates import month_index, pfml_date_grids
from ..utils.log import COUNTERS, get_logger
from ..utils.trace import range_pop, range_push
from .risk import BarraCov
from .search import PfmlReals

log = get_logger("pfml_inputs")


@dataclass
class Panel:
    """Monthly characteristics panel sorted by (month, id)."""
    mi: np.ndarray
    ids: np.ndarray
    key: np.ndarray           # mi * 10^7 + id, sorted
    valid: np.ndarray
    cols: dict                # name -> float64 array [R]
    feats: np.ndarray         # [R, k] ranked characteristics

    @classmethod
    def from_chars(cls, chars: pd.DataFrame, features: list[str]) -> "Panel":
        mi = month_index(chars["eom"])
        ids = chars["id"].to_numpy(np.int64)
        order = np.lexsort((ids, mi))
        mi, ids = mi[order], ids[order]
        cols = {}
        for c in ("ret_ld1", "tr_ld0", "mu_ld0", "tr_ld1", "lambda", "me"):
            if c in chars:
                cols[c] = chars[c].to_numpy(np.float64)[order]
        feats = np.ascontiguousarray(chars[features].to_numpy(np.float64)[order])
        return cls(mi=mi, ids=ids, key=mi * 10_000_000 + ids,
                   valid=chars["valid"].to_numpy(bool)[order], cols=cols, feats=feats)

    def rows(self, mi: int, ids: np.ndarray) -> np.ndarray:
        k = mi * 10_000_000 + np.asarray(ids, np.int64)
        p = np.searchsorted(self.key, k)
        p = np.clip(p, 0, len(self.key) - 1)
        ok = self.key[p] == k
        return np.where(ok, p, -1)

    def valid_rows(self, mi: int) -> np.ndarray:
        a = np.searchsorted(self.mi, mi, side="left")
        b = np.searchsorted(self.mi, mi, side="right")
        r = np.arange(a, b)
        return r[self.valid[a:b]]


@dataclass
class PfmlInputs:
    reals: PfmlReals
    months: np.ndarray                   # [T] month indices (dates_m2 handled here)
    signal_rows: list                    # per month: panel rows (valid ids at d, id order)
    signal_t: list                       # per g: per month [n_d, P] tensors (device)
    rff_w: np.ndarray                    # [G, k, P/2]
    ids: list                            # per month: ids
    # m_tilde and a = lambda^-1/2 of the months asked for with ``keep_m`` (S9 reuses them:
    # PFML_best_hps.py:185-190 recomputes exactly S4's m_t): {"months", "mt" [K, N, N],
    # "a" [K, N], "n" [K]} in the padded universe width N of the plan
    m_keep: dict | None = None
    # run_plan(defer_checks=True): the device status of the run, checked by finish_inputs
    # ({"mstat": [T] int32 m_func flags, "nsing": singular-const count}); None once checked
    pending: dict | None = None


def _rff_weights(cfg: Config, k: int) -> np.ndarray:
    """W per g.  compat (quirk Q1): the supplied rff_w.csv for every g (g ignored);
    corrected: W_g ~ N(0, g I_k) drawn from seed_no."""
    G, half = len(cfg.g_vec), cfg.p_max // 2
    if cfg.run.compat_mode:
        W = io.read_rff_w(cfg.run.data_dir)
        if W.shape != (k, half):
            raise ValueError(f"rff_w.csv has shape {W.shape}, expected {(k, half)}")
        return np.stack([W] * G)
    rng = np.random.default_rng(cfg.settings["seed_no"])
    Z = rng.standard_normal((k, half))
    return np.stack([Z * np.sqrt(g) for g in cfg.g_vec])


def vol_scales(panel: Panel, barra: BarraCov, months: np.ndarray) -> np.ndarray:
    """sqrt(diag Sigma_t) merged on (id, month), NaN -> cross-sectional median (:274-307)."""
    vol = np.full(len(panel.mi), np.nan)
    for mi in months:
        ids, X, F, iv = barra.slice(mi)
        d = np.einsum("ik,kl,il->i", X, F, X) + iv
        r = panel.rows(mi, ids)
        ok = r >= 0
        vol[r[ok]] = np.sqrt(d[ok])
    # median fill per month over all panel rows of that month
    s = pd.Series(vol)
    med = s.groupby(panel.mi).transform("median")
    return s.fillna(med).to_numpy()


def auto_month_batch(n_stocks: int, gp: int, device, cap: int = 1024) -> int:
    """Months per S4 batch from the memory one month's working set needs (fp64): the
    three stored signal lags (3 N GP; the other ten exist only as column statistics), five Horner buffers of N x (GP + N) plus two N x N blocks, ~8 N x N matrices of
    m_func / Sigma and the (25) scratch.  A device batch takes up to 60 % of free HBM (288 GB on
    MI355X: all 731 months at N = 500 in one batch - 23 ms faster than 256-month batches,
    profiles/r03_s4_batch_cap_ab.json - ~100 at N = 3000), a host batch 25 % of available RAM."""
    cap = int(os.environ.get("PFML_S4_BATCH_CAP", cap))      # (A/B switch)
    per = 8.0 * (3.0 * n_stocks * gp + 6.0 * n_stocks * (gp + n_stocks) + 11.0 * n_stocks ** 2
                 + 2.0 * gp * gp)
    dev = torch.device(device)
    if dev.type == "cuda":
        free, _ = torch.cuda.mem_get_info(dev)
        budget = 0.6 * free
    else:
        try:
            import psutil
            budget = 0.25 * psutil.virtual_memory().available
        except Exception:                                   # pragma: no cover
            budget = 4e9
    return int(max(1, min(cap, budget // per)))


# S4 month batches run on this many streams (PFML_S4_STREAMS; make_s4_plan then splits the
# months into at least that many batches): one batch's latency-bound kernels (SPD inverse
# nodes, LU pivot panels, leaves, the elementwise passes) overlap another's MFMA GEMMs.
# S4+S5+S6 on one MI355X (A/B on one box): 1 stream 357.6, 2: 345.5, 3: 341.4, 4: 340.8 ms
# (profiles/r05_s4_streams_ab.json; 4 hardware queues per process).  1: one stream.
S4_STREAMS = int(os.environ.get("PFML_S4_STREAMS", "3"))
_STREAMS: dict = {}


def _s4_streams(dev, n_batches: int):
    """The side streams of a multi-batch device run (created once per device), or None."""
    if dev.type != "cuda" or S4_STREAMS <= 1 or n_batches <= 1:
        return None
    key = (str(dev), S4_STREAMS)
    if key not in _STREAMS:
        _STREAMS[key] = [torch.cuda.Stream(device=dev) for _ in range(S4_STREAMS)]
        la.CONCURRENT_STREAMS.update(st_.cuda_stream for st_ in _STREAMS[key])
    return _STREAMS[key]


# statistics of lags 1..10 (the Horner steps' gathered addend) from per-date union sums minus
# each month's few excluded rows (csrc/panel.hip date_sums / excl_stats) instead of a gathered
# pass over every (month, lag) tile; PFML_S4_DSTAT=0 takes the direct pass
DSTAT = os.environ.get("PFML_S4_DSTAT", "1") != "0"


def _lag_date_layout(panel: "Panel", grid_months: np.ndarray, months: np.ndarray,
                     idx_raw: list, ns: list, lb: int, R: int):
    """Host layout of the lag 1..10 statistics by differences.  For every date d that a month
    of this plan reads at a lag 1..lb-1: U(d) = the sorted rows at d of the union of the
    universes of the GLOBAL grid months b with 1 <= b - d <= lb - 1 (so a month's statistics
    do not depend on how the months are sharded), and per (month, lag) tile the sorted rows of
    U(d) outside its own universe.  idx_raw: per batch the raw [B, lb + 2, N] panel rows."""
    # (the plan's own months join the grid: a month outside it must still find its rows in U(d))
    own_months = [np.asarray(m, np.int64) for m in months] + [np.zeros(0, np.int64)]
    gm = np.union1d(np.asarray(grid_months, np.int64), np.concatenate(own_months))
    dates = np.unique(np.concatenate([np.asarray(m, np.int64)[:, None] - np.arange(1, lb)[None, :]
                                      for m in months]).ravel()) if len(months) else \
        np.zeros(0, np.int64)
    slot = {int(d): k for k, d in enumerate(dates)}
    urows = []
    for d in dates:
        bs = gm[(gm - d >= 1) & (gm - d <= lb - 1)]
        ids = np.unique(np.concatenate([panel.ids[panel.valid_rows(int(b))] for b in bs]))
        r = panel.rows(int(d), ids)
        urows.append(np.unique(r[r >= 0]))
    ex = []
    for bm, idx, nb in zip(months, idx_raw, ns):
        rows_b, n_b, pos_b = [], [], []
        for bi, b in enumerate(bm):
            for th in range(1, lb):
                u = urows[slot[int(b) - th]]
                own = idx[bi, th, :int(nb[bi])]
                if len(np.setdiff1d(own, u)):
                    raise AssertionError(f"month {b} lag {th}: rows outside the union universe")
                e = np.setdiff1d(u, own, assume_unique=False)
                rows_b.append(e)
                n_b.append(len(e))
                pos_b.append(slot[int(b) - th])
        ex.append((rows_b, n_b, pos_b))
    return dates, urows, ex


def _even(n: int) -> int:
    return n + (n & 1)


@dataclass
class _Batch:
    months: np.ndarray          # [B] month indices
    ns: np.ndarray              # [B] universe sizes
    idx: torch.Tensor           # [B, 13, N] panel rows (pad -> zero row Rpad), device
    mask: torch.Tensor          # [B, N] 1 = real stock
    n_real: torch.Tensor        # [B] int32
    brow: torch.Tensor          # [B, N] Barra row of each stock (pad -> identity row)
    fpos: torch.Tensor          # [B] Barra month position
    lam: torch.Tensor           # [B, N] Kyle's lambda (pad: gamma / w)
    r: torch.Tensor             # [B, N] ret_ld1 (pad 0)
    w: torch.Tensor             # [B] wealth
    rf: torch.Tensor            # [B]
    # lag 1..10 statistics by differences (``DSTAT``): per (month, lag) tile the rows of its
    # date's union universe outside the month's universe, and the date's slot
    ex_rows: torch.Tensor | None = None    # [B * (lb - 1), emax] (first ex_n real)
    ex_n: torch.Tensor | None = None       # [B * (lb - 1)] int32
    ex_dpos: torch.Tensor | None = None    # [B * (lb - 1)] int32


@dataclass
class S4Plan:
    """Everything of an S4 run that is layout, not arithmetic: panel / Barra row indices of
    every month's 13-month window, per-batch padded index tensors, the device copies of the
    raw panel and Barra arrays.  Built once per (data, months, device); ``run_plan`` does all
    the math (RFF, vol scales, standardisation, Sigma, m_func, (24), (25)) on the device."""
    months: np.ndarray
    G: int                      # g values (output)
    Gc: int                     # distinct signal blocks (1 under quirk Q1)
    P: int                      # 2 * (p_max/2) + 1
    Pp: int                     # P padded to even
    N: int                      # padded universe width (even)
    W: np.ndarray               # [G, k, P/2] RFF weights
    same_w: bool
    feats: torch.Tensor         # [R, k] ranked characteristics (device)
    gt: torch.Tensor            # [R+1] (1+tr_ld0)/(1+mu_ld0), pad 1
    vol_rows: torch.Tensor      # [Mv, nv] panel rows of each vol month (pad -> R)
    vol_brow: torch.Tensor      # [Mv, nv] Barra row of each (pad / missing -> -1)
    vol_fpos: torch.Tensor      # [Mv] Barra month position of each vol month
    bX: torch.Tensor            # [Rb+1, K] Barra loadings (+ zero row)
    biv: torch.Tensor           # [Rb+1] idiosyncratic variance (+ 1 for the pad row)
    bF: torch.Tensor            # [Mb, K, K]
    batches: list
    sig_rows: list
    sig_ids: list
    R: int                      # rows of feats (the pad row is R)
    Wd: list | None = None      # device copies of W per distinct signal block (no upload in
                                # run_plan: its launches can be captured in a HIP graph)
    vol_real: torch.Tensor | None = None   # [Mv, nv] slot holds a real panel row (the vol
                                # month's median runs over all of them, whether this plan
                                # keeps a row or not)
    du_rows: torch.Tensor | None = None    # [nd, umax] union-universe rows of each lag date
    du_n: torch.Tensor | None = None       # [nd] int32


def universe_npad(chars: pd.DataFrame, months: np.ndarray) -> int:
    """The padded universe width S4 uses for the month grid ``months`` (dates_m2): S9 pads its
    m_t recompute to the same width, so a recomputed m_tilde is bitwise S4's."""
    panel = Panel.from_chars(chars, [])
    nmax = max((len(panel.valid_rows(int(d))) for d in months), default=1)
    return _even(max(nmax, 2))


def make_s4_plan(cfg: Config, chars: pd.DataFrame, barra: BarraCov, wealth: pd.DataFrame,
                 risk_free: pd.DataFrame, device, months: np.ndarray | None = None,
                 batch: int | None = None) -> S4Plan:
    features = get_features()
    pf = cfg.pf_set
    gamma = float(pf["gamma_rel"])
    lb = int(pf["lb_hor"])
    G, Pm = len(cfg.g_vec), cfg.p_max
    P = Pm + 1
    Pp = _even(P)
    dev = torch.device(device)
    panel = Panel.from_chars(chars, features)
    grids = pfml_date_grids(int(barra.months.min()), lb, cfg.settings["split"]["test_end"],
                            cfg.settings["pf"]["dates"]["start_year"],
                            cfg.settings["pf"]["dates"]["split_years"])
    if months is None:
        months = grids["m2"]
    months = np.asarray(months, np.int64)
    W = _rff_weights(cfg, len(features))
    same_w = all(np.array_equal(W[0], W[g]) for g in range(G))
    Gc = 1 if same_w else G
    R = len(panel.mi)
    wmap = dict(zip(month_index(wealth["eom"]), wealth["wealth"].to_numpy(np.float64)))
    rfmap = dict(zip(month_index(risk_free["eom"]), risk_free["rf"].to_numpy(np.float64)))
    tc_on = bool(cfg.settings["Transaction_Costs"])
    Rb = len(barra.ids)

    # vol-scale months (:274-307): sqrt(diag Sigma) merged on (id, month), median fill
    lbm = grids["lb"]
    if len(months):
        lbm = lbm[(lbm >= months.min() - (lb + 1)) & (lbm <= months.max())]
    else:
        lbm = lbm[:0]
    vr, vb, vf = [], [], []
    for mi in lbm:
        a_, b_ = np.searchsorted(panel.mi, mi, "left"), np.searchsorted(panel.mi, mi, "right")
        rows = np.arange(a_, b_)
        brow = np.full(len(rows), -1, np.int64)
        bp = 0
        try:
            bp = barra.month_pos(int(mi))
            o0, o1 = barra.offsets[bp], barra.offsets[bp + 1]
            pos = np.searchsorted(barra.ids[o0:o1], panel.ids[rows])
            pos = np.clip(pos, 0, max(o1 - o0 - 1, 0))
            hit = (o1 > o0) & (barra.ids[o0:o1][pos] == panel.ids[rows]) if o1 > o0 else \
                np.zeros(len(rows), bool)
            brow = np.where(hit, o0 + pos, -1)
        except KeyError:
            pass
        vr.append(rows)
        vb.append(brow)
        vf.append(bp)
    # padded widths from the WHOLE PFML date grid, not this rank's months: every month's
    # matrices then have one shape on every rank / batch split, so a month's summands are
    # bitwise the same however the months are sharded (canonical N-rank == 1-rank results)
    lb_all = grids["lb"]
    nv = max([int(np.searchsorted(panel.mi, mi, "right") - np.searchsorted(panel.mi, mi, "left"))
              for mi in lb_all] + [len(x) for x in vr] + [1])
    vol_rows = np.full((len(vr), nv), R, np.int64)
    vol_brow = np.full((len(vr), nv), -1, np.int64)
    for i, (x, y) in enumerate(zip(vr, vb)):
        vol_rows[i, :len(x)] = x
        vol_brow[i, :len(y)] = y

    gt_all = np.nan_to_num((1.0 + panel.cols["tr_ld0"]) / (1.0 + panel.cols["mu_ld0"]), nan=1.0)

    T = len(months)
    nmax = max((len(panel.valid_rows(int(d))) for d in np.union1d(grids["m2"], months)),
               default=1)
    Npad = _even(max(nmax, 2))
    bsz = batch or cfg.run.month_batch
    if not bsz or bsz <= 0:
        bsz = auto_month_batch(Npad, Gc * Pp, dev)
        if torch.device(dev).type == "cuda" and S4_STREAMS > 1 and T > 1:
            bsz = min(bsz, -(-T // S4_STREAMS))              # one batch per stream at least
        log.info(f"PFML inputs: {bsz} months per batch (N <= {nmax})")
    batches, sig_rows, sig_ids, idx_raw = [], [], [], []
    for b0 in range(0, T, bsz):
        bm = months[b0: b0 + bsz]
        B = len(bm)
        idx = np.full((B, lb + 2, Npad), R, dtype=np.int64)
        brow = np.full((B, Npad), Rb, dtype=np.int64)
        fpos = np.zeros(B, np.int64)
        lam = np.empty((B, Npad))
        rr = np.zeros((B, Npad))
        ns = np.zeros(B, np.int64)
        for bi, d in enumerate(bm):
            rows_d = panel.valid_rows(int(d))
            ids = panel.ids[rows_d]
            n = len(ids)
            ns[bi] = n
            for th in range(lb + 2):
                r = panel.rows(int(d) - th, ids)
                if np.any(r < 0):
                    raise ValueError(f"month {d}: universe lacks the {th}-month lookback rows")
                idx[bi, th, :n] = r
            bp = barra.month_pos(int(d))
            o0, o1 = barra.offsets[bp], barra.offsets[bp + 1]
            bids = barra.ids[o0:o1]
            pos = np.searchsorted(bids, ids)
            if np.any(pos >= len(bids)) or np.any(bids[np.minimum(pos, len(bids) - 1)] != ids):
                raise KeyError(f"month {d}: valid ids missing from the Barra universe")
            brow[bi, :n] = o0 + pos
            fpos[bi] = bp
            lam[bi] = gamma / float(wmap[int(d)])
            lam[bi, :n] = panel.cols["lambda"][rows_d] if tc_on else 1e-16
            rr[bi, :n] = panel.cols["ret_ld1"][rows_d]
            sig_rows.append(rows_d)
            sig_ids.append(ids)
        mask = (np.arange(Npad)[None, :] < ns[:, None]).astype(np.float64)
        idx_raw.append(idx)
        tt = lambda x, dt=torch.float64: torch.as_tensor(x, dtype=dt, device=dev)  # noqa: E731
        batches.append(_Batch(
            months=bm, ns=ns, idx=tt(idx, torch.int64), mask=tt(mask),
            n_real=tt(ns, torch.int32), brow=tt(brow, torch.int64), fpos=tt(fpos, torch.int64),
            lam=tt(lam), r=tt(rr), w=tt([wmap[int(d)] for d in bm]),
            rf=tt([rfmap[int(d)] for d in bm])))
    # even inner dimensions (a zero factor / a zero feature column - exact zeros in every sum):
    # the GEMMs on them (X F, X' omega, the RFF product) then take the 16-byte-load kernels
    # (+ two spare zero columns: run_plan puts the month's returns into the first, so that the
    # X' omega GEMM of the risk term also yields r_tilde = omega' r as its extra row)
    K = barra.X.shape[1]
    Kp = _even(K)
    bX = np.zeros((barra.X.shape[0] + 1, Kp + 2))
    bX[:-1, :K] = barra.X
    bF = np.zeros((barra.F.shape[0], Kp, Kp))
    bF[:, :K, :K] = barra.F
    biv = np.r_[barra.ivol, 1.0]
    kf = panel.feats.shape[1]
    kfp = _even(kf)
    Wp = [np.zeros((kfp, W[g].shape[1])) for g in range(Gc)]
    for g in range(Gc):
        Wp[g][:kf] = W[g]
    # compaction: only the panel rows this plan's months reference (their lookback rows) keep
    # an RFF feature row, a vol slot and a growth factor - a rank's S4 then scales with its own
    # months instead of paying the RFF GEMM of the whole panel (per-row arithmetic: the same
    # bits); vol months still take their medians over every row of the month
    dl = None
    if DSTAT and dev.type == "cuda" and lb > 1:
        dl = _lag_date_layout(panel, grids["m2"], [b.months for b in batches], idx_raw,
                              [b.ns for b in batches], lb, R)
    used = np.unique(np.concatenate([b.idx.cpu().numpy().ravel() for b in batches]
                                    + ([np.concatenate(dl[1])] if dl and len(dl[1]) else [])
                                    + [np.zeros(0, np.int64)]))
    used = used[used < R]
    Rc = len(used)

    def remap(a):
        pos = np.searchsorted(used, a)
        hit = (a < R) & (pos < Rc) & (used[np.minimum(pos, max(Rc - 1, 0))] == a) if Rc else \
            np.zeros(a.shape, bool)
        return np.where(hit, pos, Rc).astype(np.int64)

    for b in batches:
        b.idx = torch.as_tensor(remap(b.idx.cpu().numpy()), dtype=torch.int64, device=dev)
    du_rows = du_n = None
    if dl is not None:
        dates, urows, ex = dl
        umax = max([len(u) for u in urows] + [1])
        ua = np.full((len(urows), umax), Rc, np.int64)
        for k, u in enumerate(urows):
            ua[k, :len(u)] = remap(u)
        du_rows = torch.as_tensor(ua, device=dev)
        du_n = torch.as_tensor(np.asarray([len(u) for u in urows], np.int32), device=dev)
        for b, (rows_b, n_b, pos_b) in zip(batches, ex):
            emax = max(n_b + [1])
            ea = np.full((len(rows_b), emax), Rc, np.int64)
            for k, e in enumerate(rows_b):
                ea[k, :len(e)] = remap(e)
            b.ex_rows = torch.as_tensor(ea, device=dev)
            b.ex_n = torch.as_tensor(np.asarray(n_b, np.int32), device=dev)
            b.ex_dpos = torch.as_tensor(np.asarray(pos_b, np.int32), device=dev)
    vol_real = vol_rows < R
    vol_rows = remap(vol_rows)
    feats_p = np.zeros((Rc, kfp))
    feats_p[:, :kf] = panel.feats[used]
    return S4Plan(
        months=months, G=G, Gc=Gc, P=P, Pp=Pp, N=Npad, W=W, same_w=same_w,
        feats=torch.as_tensor(feats_p, dtype=torch.float64, device=dev),
        gt=torch.as_tensor(np.r_[gt_all[used], 1.0], dtype=torch.float64, device=dev),
        vol_rows=torch.as_tensor(vol_rows, device=dev),
        vol_real=torch.as_tensor(vol_real, device=dev),
        vol_brow=torch.as_tensor(vol_brow, device=dev),
        vol_fpos=torch.as_tensor(np.asarray(vf, np.int64), device=dev),
        bX=torch.as_tensor(bX, dtype=torch.float64, device=dev),
        biv=torch.as_tensor(biv, dtype=torch.float64, device=dev),
        bF=torch.as_tensor(bF, dtype=torch.float64, device=dev),
        batches=batches, sig_rows=sig_rows, sig_ids=sig_ids, R=Rc,
        Wd=[torch.as_tensor(Wp[g], dtype=torch.float64, device=dev) for g in range(Gc)],
        du_rows=du_rows, du_n=du_n)


def _vol_device(plan: S4Plan) -> torch.Tensor:
    """vol[r] = sqrt(diag Sigma_t)[r] for every panel row r of the vol months, NaN -> the
    month's median (PFML_Input_Data.py:274-307); rows outside those months NaN; pad row 1.
    diag(X F X')_i = sum_k (X F)_ik X_ik: per Barra row, no N x N matrix is formed."""
    dev = plan.feats.device
    vol = torch.full((plan.R + 1,), float("nan"), dtype=torch.float64, device=dev)
    if plan.vol_rows.numel():
        br = plan.vol_brow
        ok = br >= 0
        brc = torch.where(ok, br, torch.zeros_like(br))
        Fm = plan.bF[plan.vol_fpos]                               # one F per vol month
        Xr = plan.bX[brc][..., :Fm.shape[-1]]                     # [Mv, nv, K]
        d = (gemm(Xr, Fm, backend="own") * Xr).sum(-1) + plan.biv[brc]
        v = torch.where(ok, d.sqrt(), torch.full_like(d, float("nan")))
        real = plan.vol_real if plan.vol_real is not None else plan.vol_rows < plan.R
        v = torch.where(real, v, torch.full_like(v, float("nan")))
        # pandas median: mean of the two middle values of the non-NaN entries (torch's
        # nanmedian returns the lower one); NaN sorts last
        sv = torch.sort(v, dim=1).values
        cnt = (~torch.isnan(v)).sum(1, keepdim=True)
        lo = ((cnt - 1).clamp_min(0)) // 2
        hi = cnt // 2
        hi = torch.minimum(hi, (cnt - 1).clamp_min(0))
        med = 0.5 * (sv.gather(1, lo) + sv.gather(1, hi))
        v = torch.where(torch.isnan(v), med.expand_as(v), v)
        # every slot scattered (padding slots all land on the pad row R, reset below): no
        # boolean-mask indexing, whose output size needs a host sync
        vol.scatter_(0, plan.vol_rows.flatten(), v.flatten())
    vol[plan.R:plan.R + 1].fill_(1.0)
    return vol


def run_plan(plan: S4Plan, cfg: Config, keep_risk_tc: bool = False,
             keep_m: np.ndarray | None = None, defer_checks: bool = False,
             inline_repair: bool = False) -> "PfmlInputs":
    """The S4 arithmetic for every month of the plan (device or CPU fp64 oracle).  ``keep_m``:
    months whose m_tilde / a are kept for S9 (``PfmlInputs.m_keep``).

    ``defer_checks``: no host synchronisation at all - the m_func repair flags and the
    singular-const count stay on the device (``PfmlInputs.pending``) and ``finish_inputs``
    checks them once, afterwards - so the whole run can be captured and replayed as one HIP
    graph (bench.py --with-inputs).  Without it the checks run at the end of this call.
    ``inline_repair``: m_func repairs inside each batch's m_tilde (finish_inputs' re-run)."""
    pf = cfg.pf_set
    gamma, mu = float(pf["gamma_rel"]), float(pf["mu"])
    lb = int(pf["lb_hor"])
    G, Gc, P, Pp, N = plan.G, plan.Gc, plan.P, plan.Pp, plan.N
    GP = Gc * Pp
    Wd = GP + N
    dev = plan.feats.device
    prec = cfg.run.precision         # fp64 | fp32 | bf16 | fp8: covariance / RFF / risk GEMMs
    T = len(plan.months)

    # ---- 1. RFF features (K13) and 2. vol scales -----------------------------------------
    range_push("pfml_inputs.rff")
    Wdev = plan.Wd if plan.Wd is not None else [
        torch.nn.functional.pad(torch.as_tensor(plan.W[g], dtype=torch.float64, device=dev),
                                (0, 0, 0, plan.feats.shape[1] - plan.W[g].shape[0]))
        for g in range(Gc)]
    # the gathered addend's feature table: every g block side by side, [R + 1, Gc * Pp], each
    # block written in place by its RFF launch (no concatenation pass)
    Fcat = torch.empty((plan.feats.shape[0] + 1, Gc * Pp), dtype=torch.float64, device=dev)
    rffs = [rff_features(plan.feats, Wdev[g], prec, width=Pp, pad_rows=1,
                         out=Fcat[:, g * Pp:(g + 1) * Pp]) for g in range(Gc)]
    vol = _vol_device(plan)
    # lag 1..10 statistics by differences: every lag date's union sums, once (per g block)
    dsums = None
    if plan.du_rows is not None:
        dsums = [date_sums(rffs[g], plan.du_rows, plan.du_n, P, Pp) for g in range(Gc)]
    range_pop()

    # every (g, month) block is written by exactly one batch below (the batches partition the
    # plan's months): no zero fill of the 3 GB denom stack in front of the batches
    r_out = torch.empty((G, T, P), dtype=torch.float64, device=dev)
    d_out = torch.empty((G, T, P, P), dtype=torch.float64, device=dev)
    risk_out = torch.empty_like(d_out) if keep_risk_tc else None
    tc_out = torch.empty_like(d_out) if keep_risk_tc else None
    signal_t = [[None] * T for _ in range(G)]
    # singular const flags (batch) and the running count (on device), one of each per stream
    nst = max(1, len(_s4_streams(dev, len(plan.batches)) or []))
    sing_all = torch.zeros((nst, 2 * max((len(b.months) for b in plan.batches), default=0)),
                           dtype=torch.int32, device=dev)
    nsing_all = torch.zeros(nst, dtype=torch.int64, device=dev)
    # m_func repair flags of every month (device runs; checked once, by finish_inputs)
    mstat = (torch.zeros(T, dtype=torch.int32, device=dev)
             if dev.type == "cuda" and not inline_repair else None)
    m_keep = None
    # (only an fp64 Sigma is kept: S9's weight recursion is specified in fp64 whatever the S4
    # GEMM precision, config.py run.precision; other precisions leave S9 its own fp64 m_t)
    if keep_m is not None and prec == "fp64":
        km = np.asarray([m for m in plan.months if int(m) in set(int(x) for x in keep_m)],
                        np.int64)
        kpos = {int(m): i for i, m in enumerate(km)}
        mpos = {int(m): i for i, m in enumerate(plan.months)}
        m_keep = {"months": km, "mt": torch.empty((len(km), N, N), dtype=torch.float64,
                                                   device=dev),
                  "a": torch.empty((len(km), N), dtype=torch.float64, device=dev),
                  "n": np.zeros(len(km), np.int64),
                  # the ids (in row order) behind each kept m_tilde: S9 reuses a month's m_t
                  # only for exactly this universe
                  "ids": [np.asarray(plan.sig_ids[mpos[int(m)]], np.int64) for m in km]}
    b0 = 0
    streams = _s4_streams(dev, len(plan.batches))
    if streams:                     # side streams fork from (and below join) the caller's
        for st_ in streams:
            st_.wait_stream(torch.cuda.current_stream(dev))
    for kb, bt in enumerate(plan.batches):
        B = len(bt.months)
        sing = sing_all[kb % len(sing_all)]
        nsing_t = nsing_all[kb % len(nsing_all)]
        ctx = torch.cuda.stream(streams[kb % len(streams)]) if streams else contextlib.nullcontext()
        with ctx:
            range_push("pfml_inputs.batch")
            # signals of every distinct g, written into one [B, 13, N, Gc*Pp] stack
            # signals (K11/K12): lags 0, 11 and 12 materialised (signal_t, T_11's S block, U_0's
            # GEMM operand) into [B, 3, N, Gc*Pp]; lags 1..10 only as per-column means and scales -
            # the Horner steps form (F[row] - mean) * scale / vol in their epilogue (gathered
            # addend), so 10 of the 13 [N, Gc*Pp] signal blocks per month are never stored
            # (lag 0: signal_t and T_0's addend; lag 12: U_0's GEMM operand; lag 11 is written
            # below straight into T_11, pre-scaled by the next step's k-scale)
            S0 = torch.empty((B, 1, N, GP), dtype=torch.float64, device=dev)
            S12 = torch.empty((B, 1, N, GP), dtype=torch.float64, device=dev)
            idx0 = bt.idx[:, :1].contiguous()
            idx12 = bt.idx[:, lb + 1:lb + 2].contiguous()
            for g in range(Gc):
                gs = slice(g * Pp, (g + 1) * Pp)
                standardize_signals(rffs[g], idx0, bt.mask, vol, P=P, out=S0[..., gs],
                                    n_real=bt.n_real)
                standardize_signals(rffs[g], idx12, bt.mask, vol, P=P, out=S12[..., gs],
                                    n_real=bt.n_real)
            stats = torch.empty((B, lb - 1, 2, GP), dtype=torch.float64, device=dev)
            for g in range(Gc):
                if dsums is not None and bt.ex_rows is not None:
                    excl_stats(rffs[g], bt.ex_rows, bt.ex_n, bt.ex_dpos, dsums[g], bt.n_real,
                               P, out=stats[..., g * Pp:(g + 1) * Pp])
                else:
                    signal_stats(rffs[g], bt.idx[:, 1:lb], bt.mask, P,
                                 out=stats[..., g * Pp:(g + 1) * Pp], n_real=bt.n_real)
            # 1 / vol of each lag's rows (0 on padding rows: their standardised signal is 0)
            ivol = torch.where(bt.mask.unsqueeze(1) > 0, 1.0 / vol[bt.idx[:, 1:lb]],
                               torch.zeros((), dtype=torch.float64, device=dev))
            # Barra Sigma = X F X' + diag(ivol) (K1; pad rows: X = 0, ivol = 1 -> identity block)
            Xr = plan.bX[bt.brow]                                       # [B, N, K + 2]
            Fb = plan.bF[bt.fpos]                                       # [B, K, K]
            Kf = Fb.shape[-1]
            Xl = Xr[..., :Kf]                                           # [B, N, K]
            iv = plan.biv[bt.brow]                                      # [B, N]
            XF = gemm(Xl, Fb, backend="own")                             # in-house fp64 MFMA GEMM
            Sigma = torch.empty((B, N, N), dtype=torch.float64, device=dev)
            if prec == "fp64":
                # symmetric mode: the lower triangle mirrored, an exactly symmetric Sigma
                gemm_fused(XF, Xl, Sigma, trans_b=True, diag_col0=0, diag_vec=iv, sym=True)
            else:
                gemm_prec(XF, Xl.contiguous(), prec, trans_b=True, out=Sigma)
                Sigma.diagonal(dim1=1, dim2=2).add_(iv)
            # the returns ride in the first spare column (after Sigma's GEMM, which reads only
            # the K factor columns): X' omega below then carries r_tilde = omega' r as row K
            Xr[..., Kf] = bt.r
            # m = diag(a) m_tilde diag(1/a) (Lemma 1); a and 1/a are folded into the Horner GEMMs
            mt, a = la.m_tilde(Sigma, bt.lam, bt.w, bt.rf, mu, gamma, cfg.run.iterations,
                               mask=bt.mask, status=None if mstat is None else mstat[b0:b0 + B],
                               sigma_exact_sym=prec == "fp64")
            if m_keep is not None:
                sel = [(bi, kpos[int(d)]) for bi, d in enumerate(bt.months) if int(d) in kpos]
                if sel:
                    src = torch.as_tensor([x[0] for x in sel], device=dev)
                    dst = torch.as_tensor([x[1] for x in sel], device=dev)
                    m_keep["mt"][dst] = mt[src]
                    m_keep["a"][dst] = a[src]
                    for bi, k in sel:
                        m_keep["n"][k] = int(bt.ns[bi])
            # (24) Horner chain over [S_theta | I | R], one fused GEMM launch per step:
            #   T_theta = [S_theta | I] + diag(a) m_tilde diag(D_theta / a) T_{theta+1}
            # The lag-1 chain of omega_l1 (PFML_Input_Data.py:425-450: gtm_agg_l1, same m_t) is
            #   U_0 = sum_{j=1..12} (prod_{tau=1..j-1} m D_tau) [S_j | I] = T_1 + Q [S_12 | I],
            #   Q = m D_1 m D_2 ... m D_11,
            # and Q rides along the T steps theta = 10..1 as an N-column block R (R_11 = m D_11,
            # R_theta = m D_theta R_{theta+1}, no addend): 10 steps of width GP + 2N plus two of
            # GP + N instead of 22 of GP + N (29 % fewer Horner flops at N = 490, GP = 1026).
            Dg = plan.gt[bt.idx]                                        # [B, 13, N]
            ainv = 1.0 / a
            # k-scales D_theta / a of every step; step theta's GEMM takes T_{theta+1} with its rows
            # already scaled by ks[theta] (written so by step theta + 1's epilogue, out_row_scale),
            # so the ten width-(GP + 2N) main loops carry no k-scale (T_1 stays unscaled: T_0 and
            # U_0 use it)
            ks = Dg * ainv.unsqueeze(1)                                 # [B, 13, N]
            Wr = Wd + N
            Tb = [torch.empty((B, N, Wr), dtype=torch.float64, device=dev) for _ in range(2)]
            # T_11 = [S_11 | I | R_11], every row pre-scaled by ks_10: the signal block by the
            # standardisation itself (output row scale), the identity block diag(ks_10), and
            # R_11 = diag(a) m_tilde diag(D_11 / a) elementwise, in the rounding order the fused
            # GEMM against the identity produced ((m_tilde * k-scale) * row scale), then ks_10
            idx11 = bt.idx[:, lb:lb + 1].contiguous()
            T11 = Tb[0].unsqueeze(1)
            for g in range(Gc):
                standardize_signals(rffs[g], idx11, bt.mask, vol, P=P,
                                    out=T11[..., g * Pp:(g + 1) * Pp], n_real=bt.n_real,
                                    row_scale=ks[:, lb - 1])
            la.horner_init(Tb[0][:, :, GP:], mt, ks[:, lb - 1], ks[:, lb], a)
            cur = 0
            for th in range(lb - 1, 0, -1):
                gemm_fused(mt, Tb[cur], Tb[cur ^ 1], row_scale=a,
                           addend=Fcat, addend_cols=GP, addend_rows=bt.idx[:, th],
                           addend_col_shift=stats[:, th - 1, 0], addend_col_scale=stats[:, th - 1, 1],
                           addend_row_scale=ivol[:, th - 1], diag_col0=GP, diag_value=1.0,
                           out_row_scale=ks[:, th - 1] if th > 1 else None)
                cur ^= 1
            T1 = Tb[cur]
            # T0 / U0 carry LU_PANEL_COLS scratch columns for the two-level solve below
            Wz = Wd + la.LU_PANEL_COLS
            # (T_0 and U_0 side by side: their two solves below are ONE batched launch sequence)
            TU0 = torch.empty((2, B, N, Wz), dtype=torch.float64, device=dev)
            T0f, U0f = TU0[0], TU0[1]
            T0, U0 = T0f[:, :, :Wd], U0f[:, :, :Wd]
            gemm_fused(mt, T1[:, :, :Wd], T0, row_scale=a, k_scale=ks[:, 0].contiguous(),
                       addend=S0[:, 0], addend_cols=GP, diag_col0=GP, diag_value=1.0)
            # U_0 = T_1 + Q [S_12 | I]: the S_12 block on the GEMM, the identity block as Q + T_1
            gemm_fused(T1[:, :, Wd:], S12[:, 0], U0[:, :, :GP], addend=T1[:, :, :GP],
                       addend_cols=GP)
            la.block_add(U0[:, :, GP:], T1[:, :, Wd:], T1[:, :, GP:Wd])
            del Tb, T1
            sig0 = S0[:, 0]                                             # signal_t blocks
            del S12, stats, ivol
            # omega = const^-1 Omega, solved in place on the augmented [Omega | const] rows (K7)
            om2 = la.solve_augmented(TU0.view(2 * B, N, Wz), N, GP, a0=GP, b0=0,
                                     status=sing[:2 * B], z0=Wd)                  # [2B, N, GP]
            omega, omega_l1 = om2[:B], om2[B:]
            # omega_chg = omega - diag(D_0) omega_l1: one strided pass over the solve buffer
            omega_chg = la.block_add(torch.empty((B, N, GP), dtype=torch.float64, device=dev),
                                     omega, omega_l1, y_row_scale=-Dg[:, 0])
            nsing_t += torch.maximum(sing[:B], sing[B:2 * B]).sum()
            sing.zero_()
            # (25): r_tilde = omega' r, risk = gamma omega' Sigma omega (Sigma in low-rank form:
            # X (F (X' omega)) + ivol o omega), tc = w omega_chg' Lambda omega_chg, denom
            # (omega stays a row-strided view of the solve buffer: every consumer takes the
            # row stride; omega_chg is a fresh tensor)
            # [X | r | 0]' omega: X' omega for the risk term and r_tilde = omega' r (row K) in
            # one GEMM
            XtO = torch.empty((B, Kf + 2, GP), dtype=torch.float64, device=dev)
            gemm_fused(Xr, omega, XtO, trans_a=True, tile_cfg=7)     # (K + 2 rows: 64-row tiles)
            rt_ = XtO[:, Kf]                                                     # [B, GP]
            FXO = gemm(Fb, XtO[:, :Kf], backend="own")
            SO = torch.empty_like(omega)
            gemm_fused(Xl, FXO, SO, addend=omega, addend_row_scale=iv)
            lw = (bt.lam * bt.w.view(B, 1)).contiguous()
            Dt = torch.empty((B, Pp, Pp), dtype=torch.float64, device=dev)
            Dk = torch.empty_like(Dt) if keep_risk_tc else None
            for g in range(G):
                sl = slice(b0, b0 + B)
                if g >= Gc:                                  # shared block (quirk Q1)
                    d_out[g, sl] = d_out[0, sl]
                    r_out[g, sl] = r_out[0, sl]
                    if keep_risk_tc:
                        risk_out[g, sl] = risk_out[0, sl]
                        tc_out[g, sl] = tc_out[0, sl]
                    for bi in range(B):
                        signal_t[g][b0 + bi] = signal_t[0][b0 + bi]
                    continue
                cs = slice(g * Pp, (g + 1) * Pp)
                og, cg, sg = omega[:, :, cs], omega_chg[:, :, cs], SO[:, :, cs]
                # risk = gamma omega' (Sigma omega) and tc = w omega_chg' Lambda omega_chg are
                # symmetric: the GEMM's symmetric mode computes the lower tiles and mirrors them
                if prec == "fp64" and not keep_risk_tc:
                    # computed at the even width Pp, the P x P block stored straight into the
                    # denom stack (store clip; same arithmetic as the padded temporary)
                    dd = d_out[g, sl]
                    gemm_fused(og, sg, dd, trans_a=True, alpha=gamma, sym=True, clip=True)
                    gemm_fused(cg, cg, dd, trans_a=True, k_scale=lw, beta=1.0, sym=True,
                               clip=True)
                    r_out[g, sl] = rt_[:, g * Pp:g * Pp + P]
                    for bi in range(B):
                        signal_t[g][b0 + bi] = sig0[bi, : int(bt.ns[bi]), g * Pp:g * Pp + P]
                    continue
                if prec == "fp64":
                    gemm_fused(og, sg, Dt, trans_a=True, alpha=gamma, sym=True)
                else:
                    gemm_prec(og.contiguous(), sg.contiguous(), prec, trans_a=True, alpha=gamma,
                              out=Dt)
                if keep_risk_tc:
                    risk_out[g, sl] = Dt[:, :P, :P]
                    gemm_fused(cg, cg, Dk, trans_a=True, k_scale=lw, sym=True)
                    tc_out[g, sl] = Dk[:, :P, :P]
                    Dt.add_(Dk)
                else:
                    gemm_fused(cg, cg, Dt, trans_a=True, k_scale=lw, beta=1.0, sym=True)
                d_out[g, sl] = Dt[:, :P, :P]
                r_out[g, sl] = rt_[:, g * Pp:g * Pp + P]
                for bi in range(B):
                    signal_t[g][b0 + bi] = sig0[bi, : int(bt.ns[bi]), g * Pp:g * Pp + P]
            range_pop()
        b0 += B
        log.info(f"PFML inputs: months {b0}/{T}")
    if streams:
        for st_ in streams:
            torch.cuda.current_stream(dev).wait_stream(st_)
    nsing_t = nsing_all.sum()
    reals = PfmlReals(months=plan.months, r_tilde=r_out, denom=d_out, risk=risk_out, tc=tc_out)
    out = PfmlInputs(reals=reals, months=plan.months, signal_rows=plan.sig_rows,
                     signal_t=signal_t, rff_w=plan.W, ids=plan.sig_ids, m_keep=m_keep,
                     pending={"mstat": mstat, "nsing": nsing_t, "keep_risk_tc": keep_risk_tc})
    return out if defer_checks else finish_inputs(plan, cfg, out)


def _sub_plan(plan: S4Plan, pos: np.ndarray) -> S4Plan:
    """The plan restricted to the months at positions ``pos`` (one batch)."""
    import dataclasses
    offs = np.cumsum([0] + [len(b.months) for b in plan.batches])
    parts = []
    for bi, bt in enumerate(plan.batches):
        sel = pos[(pos >= offs[bi]) & (pos < offs[bi + 1])] - offs[bi]
        if len(sel):
            parts.append((bt, sel))

    def cat(f):
        return torch.cat([getattr(bt, f)[torch.as_tensor(sel, device=bt.idx.device)]
                          for bt, sel in parts])

    sub = _Batch(months=np.concatenate([bt.months[sel] for bt, sel in parts]),
                 ns=np.concatenate([bt.ns[sel] for bt, sel in parts]),
                 **{f: cat(f) for f in ("idx", "mask", "n_real", "brow", "fpos", "lam", "r",
                                         "w", "rf")})
    if all(bt.ex_rows is not None for bt, _ in parts):
        # the lag-statistics tiles of the selected months (TH per month), padded to one width
        # (padding slots are never read: ex_n counts the real ones) - the re-run's statistics
        # are then the same sums as the full run's
        th = parts[0][0].ex_rows.shape[0] // len(parts[0][0].months)
        emax = max(bt.ex_rows.shape[1] for bt, _ in parts)
        rows, ns_, dps = [], [], []
        for bt, sel in parts:
            t = (torch.as_tensor(sel, device=bt.idx.device).unsqueeze(1) * th
                 + torch.arange(th, device=bt.idx.device)).reshape(-1)
            rows.append(torch.nn.functional.pad(bt.ex_rows[t], (0, emax - bt.ex_rows.shape[1]),
                                                value=plan.R))
            ns_.append(bt.ex_n[t])
            dps.append(bt.ex_dpos[t])
        sub.ex_rows, sub.ex_n, sub.ex_dpos = torch.cat(rows), torch.cat(ns_), torch.cat(dps)
    return dataclasses.replace(plan, months=plan.months[pos], batches=[sub],
                               sig_rows=[plan.sig_rows[i] for i in pos],
                               sig_ids=[plan.sig_ids[i] for i in pos])


def finish_inputs(plan: S4Plan, cfg: Config, out: PfmlInputs) -> PfmlInputs:
    """The checks of an S4 run, one host sync: months whose m_func met a non-positive pivot
    are recomputed with the reference-form repair (a one-batch re-run of those months, patched
    into the outputs), then the singular-const count is reported."""
    pend = out.pending
    if pend is None:
        return out
    out.pending = None
    if pend["mstat"] is not None:
        bad = torch.nonzero(pend["mstat"]).flatten().cpu().numpy()
        if len(bad):
            COUNTERS.add("pfml_inputs.mfunc_repaired_months", len(bad))
            keep = None
            if out.m_keep is not None:
                keep = np.intersect1d(out.m_keep["months"], plan.months[bad])
            # (the re-run's m_tilde repairs its flagged months and counts them)
            fix = run_plan(_sub_plan(plan, bad), cfg, keep_risk_tc=pend["keep_risk_tc"],
                           keep_m=keep if keep is not None and len(keep) else None,
                           inline_repair=True)
            r, f = out.reals, fix.reals
            bi = torch.as_tensor(bad, device=r.denom.device)
            r.r_tilde[:, bi] = f.r_tilde
            r.denom[:, bi] = f.denom
            if r.risk is not None:
                r.risk[:, bi] = f.risk
                r.tc[:, bi] = f.tc
            for g in range(len(out.signal_t)):
                for k, i in enumerate(bad):
                    out.signal_t[g][i] = fix.signal_t[g][k]
            if fix.m_keep is not None:
                pos = {int(m): i for i, m in enumerate(out.m_keep["months"])}
                for k, m in enumerate(fix.m_keep["months"]):
                    out.m_keep["mt"][pos[int(m)]] = fix.m_keep["mt"][k]
                    out.m_keep["a"][pos[int(m)]] = fix.m_keep["a"][k]
    nsing = int(pend["nsing"].item())
    if nsing:
        COUNTERS.add("pfml_inputs.singular_const", nsing)
        log.warning(f"PFML inputs: {nsing} month(s) with a numerically singular sum of agg")
    return out


def build_inputs(cfg: Config, chars: pd.DataFrame, barra: BarraCov, wealth: pd.DataFrame,
                 risk_free: pd.DataFrame, device, months: np.ndarray | None = None,
                 keep_risk_tc: bool = False, batch: int | None = None,
                 plan: S4Plan | None = None, keep_m: np.ndarray | None = None) -> PfmlInputs:
    """S4 for ``months`` (default dates_m2): ``make_s4_plan`` + ``run_plan``."""
    if plan is None:
        plan = make_s4_plan(cfg, chars, barra, wealth, risk_free, device, months, batch)
    return run_plan(plan, cfg, keep_risk_tc, keep_m=keep_m)


def to_reference_order(x: torch.Tensor, p_max: int, dims: tuple = (-1,)) -> torch.Tensor:
    """Permute internal [const, cos1, sin1, ...] axes to the reference feat_all order."""
    inv = np.argsort(interleaved_order(p_max))
    idx = torch.as_tensor(inv, device=x.device)
    for d in dims:
        x = x.index_select(d, idx)
    return x
