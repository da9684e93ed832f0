"""L5 hyper-parameter search: ridge coefficients (26) and out-of-sample utilities.

Replaces PFML_Search_Coef.py (expanding running sums + 101 ``np.linalg.solve`` per
(g, year, p), :60-143) and PFML_hp_reals.py (one quadratic form per (g, year, p, lambda,
month) from Python, :62-130) with one batched device pipeline:

1. window sums   - one segmented-sum pass over the resident [G, T, P, P] / [G, T, P] stacks
                   (burn-in block + one block per hp year), prefix over blocks (K14);
2. ridge grid    - band reduction (bandwidth 16) per (g, year, p) cell, a banded Cholesky
                   per lambda and a blocked-WY back-transform (K15, csrc/ridge_band.hip);
3. utilities     - fused D_t B GEMM + dot epilogue per (cell, validation month) (K16);
4. scores        - expanding mean by (p, l) and dense rank per month (K17), in torch.

Signals are kept in the interleaved order [constant, cos1, sin1, cos2, sin2, ...]
(config.interleaved_order) so every hyper-parameter p uses the LEADING (p+1) x (p+1) block.

Distributed: the months are cut into 2 C canonical chunks (C = 8 burn-in pieces, C groups of
whole hp-year blocks; ``win_layout``) that ranks own whole, so S4 months balance across ranks
(the burn-in is spread) and every world size adds the same numbers in the same order: chunk
totals are left folds of their segment sums, the prefix over chunks is a left fold in chunk
order, and a window is the left fold of its chunk's year segments from that prefix - N-rank
results are BITWISE the 1-rank results.  The chunk totals cross ranks by ONE all-gather (a
P x P matrix per owned chunk per g) and the per-month utilities are ONE
all-gather at the end (a few MB; every rank's row count follows from the shared plan).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np
import pandas as pd
import torch

from ..config import Config
from ..ops import _native as nat
from ..ops.ridge import _HostClock, ridge_utilities, window_prefix_sym, window_prefix_vec
from ..parallel import collectives as coll
from ..parallel.dist import env as dist_env
from ..utils.dates import mi_from_ym, month_end
from ..utils.log import get_logger
from ..utils.trace import range_push, range_pop

log = get_logger("search")


nat.register_hip("pfml_validation_scores", [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.c_int, C.c_void_p, C.c_void_p, C.c_void_p])
nat.register_hip("pfml_scores_max_per_month", [])
nat.register_hip("pfml_validation_scores_all", [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                                C.c_void_p, C.c_void_p, C.c_void_p])


@dataclass
class PfmlReals:
    """Per-month PFML summands of (25) for every g (internal interleaved feature order).

    ``months`` are the months held here; with ``all_months`` set they are a sorted subset of
    that global list (a rank's chunks plus its validation halo, see ``local_month_rows``) and
    the search plans over the global list."""
    months: np.ndarray                 # [T] month indices, sorted ascending
    r_tilde: torch.Tensor              # [G, T, P]
    denom: torch.Tensor                # [G, T, P, P]
    risk: torch.Tensor | None = None   # [G, T, P, P] (kept for artifact parity)
    tc: torch.Tensor | None = None
    all_months: np.ndarray | None = None

    @property
    def G(self):
        return self.r_tilde.shape[0]

    @property
    def P(self):
        return self.r_tilde.shape[-1]


@dataclass
class SearchPlan:
    years: np.ndarray                  # hp years
    seg_start: np.ndarray              # [nY] first month row of year block
    seg_stop: np.ndarray
    burn_stop: int                     # months[:burn_stop] are the burn-in block
    count: np.ndarray                  # [nY] months in the expanding window of year Y
    val_start: np.ndarray              # [nY] validation month rows [(Y-1)-12, Y-11]
    val_stop: np.ndarray
    n_months: int = 0                  # months in the list the plan was made for


def make_plan(months: np.ndarray, years: np.ndarray) -> SearchPlan:
    months = np.asarray(months, dtype=np.int64)
    y0 = int(years.min())
    # burn-in: eom < (y0-2)-12-31  (PFML_Search_Coef.py:69-72)
    burn_stop = int(np.searchsorted(months, mi_from_ym(y0 - 2, 12), side="left"))
    seg_start = np.searchsorted(months, [mi_from_ym(y - 2, 12) for y in years], side="left")
    seg_stop = np.searchsorted(months, [mi_from_ym(y - 1, 11) for y in years], side="right")
    # contiguous blocks: year Y's block begins where the previous block ended
    seg_start = np.maximum(seg_start, np.r_[burn_stop, seg_stop[:-1]])
    count = seg_stop.astype(np.int64)   # every month up to (Y-1)-11 is in the window
    val_start = np.searchsorted(months, [mi_from_ym(y - 1, 12) for y in years], side="left")
    val_stop = np.searchsorted(months, [mi_from_ym(y, 11) for y in years], side="right")
    return SearchPlan(np.asarray(years), seg_start.astype(np.int64), seg_stop.astype(np.int64),
                      burn_stop, count, val_start.astype(np.int64), val_stop.astype(np.int64),
                      len(months))


NCHUNK = 8            # canonical chunks per kind (covers world 1, 2, 4, 8 bitwise alike)


@dataclass
class WinLayout:
    """World-size independent cut of the month axis for the window sums: C burn-in pieces
    (global month rows [a, b), possibly empty, sized to balance the per-rank S4 months) and C
    groups of consecutive hp years.  Chunk c of either kind belongs to rank c * world // C."""
    C: int
    burn: list
    ychunks: list


def win_layout(plan: "SearchPlan", nY: int, world: int) -> WinLayout:
    """The year chunks are near-equal in years; the burn-in months are cut so that burn piece
    c plus year chunk c (its months, and for the last chunk the months after the last block,
    which its owner also builds) are near-equal in MONTHS - the per-rank S4 load, since rank r
    of a W-rank run owns pieces and chunks c with c * W // C == r.  (Equal burn pieces left a
    W = 8 run 95 / 82 months on its busiest / lightest ranks.)  The cut depends on C only,
    never on the world size, so the window sums stay bitwise the same on every world size."""
    C = max(NCHUNK, int(world))
    nb = int(plan.burn_stop)
    ych = [coll.contiguous_split(nY, C, c) for c in range(C)]
    ym = np.zeros(C, np.int64)
    for c, ys in enumerate(ych):
        if len(ys):
            ym[c] = int(plan.seg_stop[ys[-1]]) - int(plan.seg_start[ys[0]])
    if nY and len(ych[-1]):
        ym[-1] += int(plan.n_months) - int(plan.seg_stop[-1])
    sizes = _water_fill(nb, ym)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    burn = [(int(off[k]), int(off[k + 1])) for k in range(C)]
    return WinLayout(C, burn, ych)


def _water_fill(total: int, base: np.ndarray) -> np.ndarray:
    """Non-negative integers s (sum = total) making base + s as level as possible: s_c =
    max(0, level - base_c) for the level that spends ``total``, the remainder dealt one by one
    to the lowest base + s (ties: the lower index) - deterministic."""
    base = np.asarray(base, np.int64)
    s = np.zeros(len(base), np.int64)
    if total <= 0 or len(base) == 0:
        return s
    lo, hi = int(base.min()), int(base.max()) + total
    while lo < hi:                       # largest level whose fill does not exceed total
        mid = (lo + hi + 1) // 2
        if int(np.maximum(0, mid - base).sum()) <= total:
            lo = mid
        else:
            hi = mid - 1
    s = np.maximum(0, lo - base)
    for _ in range(int(total - s.sum())):
        s[int(np.argmin(base + s))] += 1
    return s


def chunk_owner(c: int, C: int, world: int) -> int:
    return c * world // C


def rank_years(nY: int, world: int, rank: int) -> np.ndarray:
    """hp-year indices owned by ``rank`` (contiguous: its year chunks are consecutive)."""
    C = max(NCHUNK, int(world))
    ys = [y for c in range(C) if chunk_owner(c, C, world) == rank
          for y in coll.contiguous_split(nY, C, c)]
    return np.asarray(ys, dtype=np.int64)


def local_month_rows(all_months: np.ndarray, years: np.ndarray, world: int,
                     rank: int) -> np.ndarray:
    """Global rows of ``all_months`` whose S4 summands ``rank`` computes:
    its burn-in pieces, the blocks of its hp years and the validation months of its last
    year (the next block: a one-block halo).  Sorted; not contiguous in general (the burn-in
    pieces are spread over the ranks so the S4 months balance).  Every rank thus builds the
    summands of its own months only; window prefixes cross ranks as P x P chunk totals."""
    all_months = np.asarray(all_months, np.int64)
    plan = make_plan(all_months, np.asarray(years))
    lay = win_layout(plan, len(years), world)
    rows = []
    for k, (a, b) in enumerate(lay.burn):
        if chunk_owner(k, lay.C, world) == rank:
            rows.append(np.arange(a, b))
    yl = rank_years(len(years), world, rank)
    for y in yl:
        rows.append(np.arange(int(plan.seg_start[y]), int(plan.seg_stop[y])))
    if len(yl):
        rows.append(np.arange(int(plan.val_start[yl[-1]]), int(plan.val_stop[yl[-1]])))
    if not rows:
        return np.zeros(0, np.int64)
    return np.unique(np.concatenate(rows)).astype(np.int64)


def owned_month_rows(all_months: np.ndarray, years: np.ndarray, world: int,
                     rank: int) -> np.ndarray:
    """Global rows OWNED by ``rank``: its burn-in pieces and hp-year blocks, and (owner of the
    last hp year) the months after the last block - every month has exactly one owner, and in
    time order
    the owners never decrease, so a time-sequential chain (the S9 recursion) can run over
    the owned months rank after rank with one hand-off each."""
    all_months = np.asarray(all_months, np.int64)
    plan = make_plan(all_months, np.asarray(years))
    lay = win_layout(plan, len(years), world)
    rows = [np.arange(a, b) for k, (a, b) in enumerate(lay.burn)
            if chunk_owner(k, lay.C, world) == rank]
    for y in rank_years(len(years), world, rank):
        rows.append(np.arange(int(plan.seg_start[y]), int(plan.seg_stop[y])))
    # the months after the last block go to the owner of the last year (its halo holds them)
    if len(years) and len(rank_years(len(years), world, rank)) and \
            rank_years(len(years), world, rank)[-1] == len(years) - 1:
        rows.append(np.arange(int(plan.seg_stop[-1]), len(all_months)))
    return np.unique(np.concatenate(rows)).astype(np.int64) if rows else np.zeros(0, np.int64)


def s4_compute_rows(all_months: np.ndarray, years: np.ndarray, world: int,
                    rank: int) -> np.ndarray:
    """Global rows whose S4 summands ``rank`` computes: its local rows (``local_month_rows``)
    that it also owns.  The rest of its local rows - the validation halo of its last hp year,
    which is the next rank's first block - arrive from their owners (``complete_local_reals``)
    instead of being built twice: every month's S4 runs on exactly one rank."""
    return np.intersect1d(local_month_rows(all_months, years, world, rank),
                          owned_month_rows(all_months, years, world, rank)).astype(np.int64)


def s4_month_counts(all_months: np.ndarray, years: np.ndarray, world: int) -> list:
    """S4 months per rank (load balance report)."""
    return [len(s4_compute_rows(all_months, years, world, r)) for r in range(world)]


_HALO: dict = {}


def _halo_layout(all_months: np.ndarray, years: np.ndarray, world: int, rank: int,
                 dev) -> dict:
    """Index layout of the S4 halo exchange, cached per shape (and device: the index tensors
    are uploaded once, outside any graph capture).  Each rank sends the rows of its computed
    months that another rank holds as halo (``send``, sorted); the sends are concatenated in
    rank order by ONE known-size all-gather, and rank ``rank`` takes its halo rows from it
    (``gidx``)."""
    key = (np.asarray(all_months).tobytes(), np.asarray(years).tobytes(), world, rank, str(dev))
    hit = _HALO.get(key)
    if hit is not None:
        return hit
    loc = [local_month_rows(all_months, years, world, r) for r in range(world)]
    comp = [s4_compute_rows(all_months, years, world, r) for r in range(world)]
    halo = [np.setdiff1d(loc[r], comp[r]) for r in range(world)]
    need = np.unique(np.concatenate(halo)) if world > 1 else np.zeros(0, np.int64)
    send = [np.intersect1d(comp[r], need) for r in range(world)]
    off = np.concatenate([[0], np.cumsum([len(s) for s in send])]).astype(np.int64)
    gidx = []
    for h in halo[rank]:
        src = [s for s in range(world) if s != rank and h in set(send[s].tolist())]
        if len(src) != 1:
            raise ValueError(f"rank {rank}: halo month row {h} has {len(src)} senders")
        s = src[0]
        gidx.append(off[s] + int(np.searchsorted(send[s], h)))
    L = loc[rank]

    def tens(a):
        return torch.as_tensor(np.asarray(a, np.int64), device=dev)

    out = dict(T=len(L), counts=[len(s) for s in send],
               pos_comp=tens(np.searchsorted(L, comp[rank])),
               pos_halo=tens(np.searchsorted(L, halo[rank])),
               send_in_comp=tens(np.searchsorted(comp[rank], send[rank])),
               gidx=tens(gidx), n_halo=len(halo[rank]))
    if len(_HALO) > 16:
        _HALO.clear()
    _HALO[key] = out
    return out


def complete_local_reals(r_c: torch.Tensor, d_c: torch.Tensor, all_months: np.ndarray,
                         years) -> "PfmlReals":
    """This rank's local PFML summands (``local_month_rows``: its chunks plus the validation
    halo) from the ones it computed (``s4_compute_rows``: r_c [G, Tc, P], d_c [G, Tc, P, P]):
    the halo months come from their owners by one known-size all-gather of the rows other
    ranks need (~12 months x G x P x P doubles per rank over xGMI, ~50 MB at P = 513) instead
    of a second S4 of them.  In a one-process rehearsal of a W-rank run (tools/bench_shard.py:
    collectives are no-ops) the halo rows are zeros: the shapes are real, only the timing is
    meaningful."""
    all_months = np.asarray(all_months, np.int64)
    years = np.asarray(years)
    env = dist_env()
    W, r = env.world_size, env.rank
    rows_l = local_month_rows(all_months, years, W, r)
    if W == 1:
        return PfmlReals(months=all_months[rows_l], r_tilde=r_c, denom=d_c,
                         all_months=all_months)
    lay = _halo_layout(all_months, years, W, r, d_c.device)
    G, _, P = r_c.shape
    R = torch.empty((G, lay["T"], P), dtype=r_c.dtype, device=r_c.device)
    D = torch.empty((G, lay["T"], P, P), dtype=d_c.dtype, device=d_c.device)
    R.index_copy_(1, lay["pos_comp"], r_c)
    D.index_copy_(1, lay["pos_comp"], d_c)
    if env.is_dist:
        sD = d_c.index_select(1, lay["send_in_comp"]).transpose(0, 1).contiguous()
        sR = r_c.index_select(1, lay["send_in_comp"]).transpose(0, 1).contiguous()
        gD = coll.all_gather_known(sD, lay["counts"])          # [sum sends, G, P, P]
        gR = coll.all_gather_known(sR, lay["counts"])
        if lay["n_halo"]:
            D.index_copy_(1, lay["pos_halo"], gD.index_select(0, lay["gidx"]).transpose(0, 1))
            R.index_copy_(1, lay["pos_halo"], gR.index_select(0, lay["gidx"]).transpose(0, 1))
    elif lay["n_halo"]:
        D.index_fill_(1, lay["pos_halo"], 0.0)
        R.index_fill_(1, lay["pos_halo"], 0.0)
    return PfmlReals(months=all_months[rows_l], r_tilde=R, denom=D, all_months=all_months)


@dataclass
class GridResult:
    years: np.ndarray
    p_vec: list
    l_vec: np.ndarray
    years_local: np.ndarray            # hp years whose betas live on this rank
    beta: torch.Tensor                 # [G, nY_local, nP, L, P] (zero beyond p+1)
    val_months: np.ndarray             # [nVal] month indices of all validation rows
    val_year: np.ndarray               # [nVal] hp_end of each validation month
    obj: torch.Tensor                  # [nVal, G, nP, L]  (all ranks once gathered)
    timings: dict = field(default_factory=dict)
    # this rank's window sums (SD [G, nYl, P, P], Sr [G, nYl, P]) and the bookkeeping of
    # gather_grid (utilities local until gathered)
    window: tuple | None = None
    gathered: bool = True
    all_months: np.ndarray | None = None


_SETUP: dict = {}


def _search_setup(months: np.ndarray, years: np.ndarray, p_vec, G: int, T: int, world: int,
                  rank: int, dev, l_vec: np.ndarray, rows: np.ndarray) -> dict:
    """Everything of a grid search that depends only on its shape - the window plan and
    canonical chunk layout, this rank's segments, chunk slots, cells and validation jobs, and
    their device copies - built once per shape and reused by every later search (no host
    planning, no host->device copies in the steady state).  ``months`` is the global month
    list; the T months held locally are the global rows ``rows`` (sorted)."""
    key = (months.tobytes(), np.asarray(years).tobytes(), tuple(p_vec), G, T, world, rank,
           str(dev), l_vec.tobytes(), rows.tobytes())
    hit = _SETUP.get(key)
    if hit is not None:
        return hit
    plan = make_plan(months, years)
    lay = win_layout(plan, len(years), world)
    C = lay.C
    yl = rank_years(len(years), world, rank)
    nYl = len(yl)
    nP = len(p_vec)

    def loc(a: int, b: int, what: str) -> tuple[int, int]:
        la, lb = int(np.searchsorted(rows, a)), int(np.searchsorted(rows, b))
        if lb - la != b - a:
            raise ValueError(f"rank {rank}: local months miss the rows [{a}, {b}) of its {what}")
        return la, lb

    # segments in month order: the owned burn-in pieces (prefix only), then the owned years
    own = [c for c in range(C) if chunk_owner(c, C, world) == rank]
    st, sp, chunk_seg = [], [], []                    # chunk_seg: (kind, c, s0, s1)
    for k in own:
        a, b = loc(*lay.burn[k], "burn-in piece")
        chunk_seg.append(("b", k, len(st), len(st) + 1))
        st.append(a)
        sp.append(b)
    skip = len(st)
    yseg = {}
    for c in own:
        s0 = len(st)
        for y in lay.ychunks[c]:
            a, b = loc(int(plan.seg_start[y]), int(plan.seg_stop[y]), "window blocks")
            st.append(a)
            sp.append(b)
        chunk_seg.append(("y", c, s0, len(st)))
        yseg[c] = (s0, len(st))
    nseg = len(st)
    # canonical slots of the gathered chunk totals: rank blocks in rank order, each rank's
    # chunks as listed above (burn pieces, then year chunks, ascending)
    counts, sb, sy, off = [], [0] * C, [0] * C, 0
    for r in range(world):
        ro = [c for c in range(C) if chunk_owner(c, C, world) == r]
        for i, k in enumerate(ro):
            sb[k] = off + i
        for i, c in enumerate(ro):
            sy[c] = off + len(ro) + i
        counts.append(2 * len(ro))
        off += 2 * len(ro)
    clast = max(own) if nYl else -1
    ys = [yseg.get(c, (0, 0))[0] for c in range(C)]
    ye = [yseg.get(c, (0, 0))[1] for c in range(C)]
    cs = np.asarray([x[2] for x in chunk_seg], np.int32)
    ce = np.asarray([x[3] for x in chunk_seg], np.int32)
    slot = np.arange(len(chunk_seg), dtype=np.int32)          # local totals: local order
    tot_slots = (np.asarray(sb, np.int32), np.asarray(sy, np.int32))
    pv = np.asarray(p_vec, dtype=np.int64)
    gg, yy, pp = np.meshgrid(np.arange(G), np.arange(nYl), np.arange(nP), indexing="ij")
    cell_src = (gg * nYl + yy).reshape(-1)                 # cell order [g][year][p]
    cell_n = (pv[pp] + 1).reshape(-1)
    cnt = np.maximum(np.asarray(plan.count, dtype=np.int64)[yl], 1) if nYl else np.zeros(0)
    cell_scale = (1.0 / cnt[yy].astype(np.float64)).reshape(-1)
    # validation jobs: [val month][g][p]  -> obj reshapes to [nValLocal, G, nP, L]
    vrows = ([loc(int(plan.val_start[y]), int(plan.val_stop[y]), "validation halo")
              for y in yl] if nYl else [])
    vs = np.asarray([a for a, _ in vrows], np.int64)
    ve = np.asarray([b for _, b in vrows], np.int64)
    nv = ve - vs
    v_yi = np.repeat(np.arange(nYl), nv)                   # local year index per val row
    v_m = (np.concatenate([np.arange(a, b) for a, b in zip(vs, ve)])
           if nYl else np.zeros(0, np.int64))
    nVr = len(v_m)
    vi, g2, p2 = np.meshgrid(np.arange(nVr), np.arange(G), np.arange(nP), indexing="ij")
    jc = ((g2 * nYl + v_yi[vi]) * nP + p2).reshape(-1)
    jm = (g2 * T + v_m[vi]).reshape(-1)
    jn = (pv[p2] + 1).reshape(-1)
    out = dict(plan=plan, layout=lay, yl=yl, nYl=nYl, st=st, sp=sp, nseg=nseg, skip=skip,
               cs=cs, ce=ce, slot=slot, sb=tot_slots[0], sy=tot_slots[1],
               ys=np.asarray(ys, np.int32), ye=np.asarray(ye, np.int32), clast=clast,
               counts=counts, nlc=len(chunk_seg),
               cell_src=np.asarray(cell_src), cell_n=np.asarray(cell_n),
               cell_scale=np.asarray(cell_scale), v_yi=v_yi, v_m=v_m, nVr=nVr,
               jc=np.asarray(jc), jm=np.asarray(jm), jn=np.asarray(jn), dev_idx=None,
               lvec=torch.as_tensor(l_vec, dtype=torch.float64, device=dev))
    # every index the window-sum kernels turn into an address, checked on the host
    sta, spa = np.asarray(st, np.int64), np.asarray(sp, np.int64)
    if nseg and (sta.min() < 0 or spa.max() > T or (spa < sta).any() or nseg > 128):
        raise ValueError(f"rank {rank}: window segments out of range (T={T}, nseg={nseg})")
    nlc = len(chunk_seg)
    if nlc and (cs.min() < 0 or ce.max() > nseg or (ce < cs).any()):
        raise ValueError(f"rank {rank}: chunk segment ranges out of range")
    nslot = int(sum(counts))
    for arr in (tot_slots[0], tot_slots[1]):
        if len(arr) and (arr.min() < 0 or arr.max() >= nslot):
            raise ValueError(f"rank {rank}: chunk total slots out of range")
    if nseg and dev is not None and dev.type == "cuda":
        from ..ops.ridge import upload
        out["dev_idx"] = upload([np.asarray(st, np.int32), np.asarray(sp, np.int32),
                                 np.concatenate([cs, ce, slot]).astype(np.int32),
                                 np.concatenate([out["sb"], out["sy"], out["ys"],
                                                 out["ye"]]).astype(np.int32)], dev)
    if len(_SETUP) > 32:
        _SETUP.clear()
    _SETUP[key] = out
    return out


def window_sums(reals: "PfmlReals", su: dict) -> tuple[torch.Tensor, torch.Tensor]:
    """Expanding-window sums (SD [G, nYl, P, P], Sr [G, nYl, P]) of this rank's hp years in
    the canonical chunk order (see the module docstring): local chunk totals, ONE all-gather
    of them, then the windows.  Device: csrc/segsum.hip (segment sums + totals, windows);
    CPU: the same folds in torch."""
    from ..ops.ridge import chunk_totals, chunk_windows
    X, R = reals.denom, reals.r_tilde.contiguous()
    totD, totR, scratch = chunk_totals(X, R, su)
    env = dist_env()
    if env.is_dist:
        # chunk-major rows [slot][matrix totals | vector totals]: ONE known-size all-gather of
        # every rank's chunk totals (matrices and vectors together)
        G, P = totD.shape[1], totD.shape[-1]
        tot = coll.all_gather_known(scratch["tot"], [c for c in su["counts"]])
        totD = tot[:, :G * P * P].view(-1, G, P, P)
        totR = tot[:, G * P * P:].view(-1, G, P)
    elif env.world_size > 1:
        # one-process rehearsal of a rank of a W-rank run (tools/bench_shard.py: collectives
        # are no-ops): the gathered layout with this rank's totals in its own slots and zeros
        # for the other ranks' - the kernels see the real shapes; the sums lack the other
        # ranks' chunks, so only the timing is meaningful
        off = int(sum(su["counts"][:env.rank]))
        fullD = torch.zeros((int(sum(su["counts"])),) + tuple(totD.shape[1:]), dtype=totD.dtype,
                            device=totD.device)
        fullR = torch.zeros((int(sum(su["counts"])),) + tuple(totR.shape[1:]), dtype=totR.dtype,
                            device=totR.device)
        fullD[off:off + totD.shape[0]] = totD
        fullR[off:off + totR.shape[0]] = totR
        totD, totR = fullD, fullR
    return chunk_windows(X, R, su, totD, totR, scratch)


def grid_search(reals: PfmlReals, cfg: Config, *, gather: bool = True) -> GridResult:
    th = _HostClock()
    env = dist_env()
    dev = reals.denom.device
    G, T, P = reals.G, reals.denom.shape[1], reals.P
    years = cfg.hp_years
    p_vec = cfg.p_vec
    nP = len(p_vec)
    all_months = np.asarray(reals.months if reals.all_months is None else reals.all_months,
                            dtype=np.int64)
    rows = np.searchsorted(all_months, np.asarray(reals.months, np.int64)).astype(np.int64)
    if len(rows) and (int(rows.max()) >= len(all_months)
                      or not np.array_equal(all_months[rows], np.asarray(reals.months))):
        raise ValueError("grid_search: local months must be a subset of all_months")
    su = _search_setup(all_months, np.asarray(years), p_vec, G, T, env.world_size, env.rank, dev,
                       np.asarray(cfg.l_vec, dtype=np.float64), rows)
    lvec = su["lvec"]
    L = lvec.numel()
    plan, yl, nYl = su["plan"], su["yl"], su["nYl"]

    # ---- 1. window sums over this rank's chunks (canonical order; one all-gather) -----
    range_push("search.window_sums")
    SD, Sr = window_sums(reals, su)
    range_pop()

    # ---- 2. ridge grid + 3. utilities for every (cell, validation month) -------------
    th("grid_search.window_sums")
    range_push("search.ridge_utilities")
    v_yi, v_m = su["v_yi"], su["v_m"]
    th("grid_search.plan")
    # ridge grid + utilities, big-n cells overlapped with the rest on a second stream
    beta, obj = ridge_utilities(SD.reshape(G * nYl, P, P), Sr.reshape(G * nYl, P),
                                su["cell_src"], su["cell_n"], su["cell_scale"], lvec,
                                reals.denom.reshape(G * T, P, P),
                                reals.r_tilde.reshape(G * T, P), su["jc"], su["jm"], su["jn"])
    beta = beta.view(G, nYl, nP, L, P)
    obj = obj.view(su["nVr"], G, nP, L)
    range_pop()

    th("grid_search.ridge_utilities")
    v_y = yl[v_yi] if nYl else np.zeros(0, np.int64)
    v_m = rows[v_m] if len(v_m) else v_m                 # local rows -> global rows
    res = GridResult(years=years, p_vec=p_vec, l_vec=cfg.l_vec, years_local=years[yl],
                     beta=beta, val_months=all_months[v_m],
                     val_year=np.asarray(years, dtype=np.int64)[v_y], obj=obj,
                     window=(SD, Sr), gathered=not env.is_dist, all_months=all_months)
    return gather_grid(res) if gather else res


def gather_grid(grid: GridResult) -> GridResult:
    """ONE all-gather of the per-(month, cell) utilities of every rank (each rank's row count
    follows from the shared plan); validation months and years rebuilt locally.  No-op on one
    rank or when already gathered."""
    env = dist_env()
    if grid.gathered or not env.is_dist:
        grid.gathered = True
        return grid
    range_push("search.gather")
    years = np.asarray(grid.years)
    plan = make_plan(grid.all_months, years)
    nv_all = np.asarray(plan.val_stop, np.int64) - np.asarray(plan.val_start, np.int64)
    counts = [int(nv_all[rank_years(len(years), env.world_size, r)].sum())
              for r in range(env.world_size)]
    grid.obj = coll.all_gather_known(grid.obj, counts)
    v_m = np.concatenate([np.arange(a, b) for a, b in zip(plan.val_start, plan.val_stop)])
    grid.val_months = grid.all_months[v_m]
    grid.val_year = years.astype(np.int64)[np.repeat(np.arange(len(years)), nv_all)]
    grid.gathered = True
    range_pop()
    return grid


def _local_val_rows(grid: GridResult, reals: PfmlReals) -> dict:
    """{hp year: [(row in grid.obj, local month row)]} of this rank's validation months (the
    utilities of a not-yet-gathered grid, or the gathered rows whose months are local)."""
    months = np.asarray(reals.months, dtype=np.int64)
    out = {}
    for i, (vm, vy) in enumerate(zip(grid.val_months, grid.val_year)):
        j = int(np.searchsorted(months, vm))
        if j < len(months) and months[j] == vm:
            out.setdefault(int(vy), []).append((i, j))
    return out


def _oracle_cell(grid: GridResult, reals: PfmlReals, g: int, yi: int, pi: int, SD=None,
                 Sr=None):
    """fp64 CPU oracle of one (g, local year, p) cell: one pivoted-LU solve per lambda
    (np.linalg.solve semantics) on the window sums ``SD``/``Sr`` (default: the grid's own),
    and its validation utilities on this rank's months.  Returns (beta [L, P], [(row,
    utilities [L])])."""
    from ..ops.ridge import quadform_utilities, ridge_grid
    years = np.asarray(grid.years)
    plan = make_plan(grid.all_months if grid.all_months is not None else reals.months, years)
    y = int(np.nonzero(years == grid.years_local[yi])[0][0])
    n = int(grid.p_vec[pi]) + 1
    if SD is None:
        SD, Sr = grid.window[0][g, yi].cpu(), grid.window[1][g, yi].cpu()
    lv = torch.as_tensor(grid.l_vec, dtype=torch.float64)
    b = ridge_grid(SD[None], Sr[None], np.array([0]), np.array([n]),
                   np.array([1.0 / max(int(plan.count[y]), 1)]), lv)[0]
    rows = _local_val_rows(grid, reals).get(int(years[y]), [])
    util = []
    if rows:
        denom, rt = reals.denom.cpu(), reals.r_tilde.cpu()
        T = denom.shape[1]
        jm = np.array([g * T + j for _, j in rows])
        o = quadform_utilities(denom.reshape(-1, *denom.shape[2:]), rt.reshape(-1, rt.shape[-1]),
                               b[None], np.zeros(len(rows), np.int64), jm, np.full(len(rows), n))
        util = [(i, o[k]) for k, (i, _) in enumerate(rows)]
    return b, util


def check_against_oracle(grid: GridResult, reals: PfmlReals, cfg: Config, ncells: int = 3,
                         seed: int = 0) -> dict:
    """``--check``: recompute a few (g, year, p) cells of this rank with the
    fp64 CPU oracle - one ``torch.linalg.solve`` per lambda, quadratic forms one by one - and
    report the max relative error of the device coefficients and utilities (the largest-n cell
    is always among them).  The expanding-window sums are re-added by plain summation when
    this rank holds every month up to the window (one rank); a shard checks the solves and
    utilities on its own window sums and reports the window sums as unchecked."""
    years = np.asarray(grid.years)
    nYl = len(grid.years_local)
    G, nP = reals.G, len(grid.p_vec)
    if nYl == 0:
        return {"cells": 0}
    months = np.asarray(reals.months, dtype=np.int64)
    allm = grid.all_months if grid.all_months is not None else months
    full = len(months) == len(allm)
    plan = make_plan(allm, years)
    rng = np.random.default_rng(seed)
    picks = {(0, nYl - 1, nP - 1)}
    while len(picks) < min(ncells, G * nYl * nP):
        picks.add((int(rng.integers(G)), int(rng.integers(nYl)), int(rng.integers(nP))))
    obj_host = grid.obj.cpu()
    eb = eo = ew = 0.0
    for g, yi, pi in sorted(picks):
        SD = Sr = None
        if full:
            y = int(np.nonzero(years == grid.years_local[yi])[0][0])
            stop = int(plan.seg_stop[y])
            SD = reals.denom[g, :stop].cpu().sum(0)
            Sr = reals.r_tilde[g, :stop].cpu().sum(0)
            wd = grid.window[0][g, yi].cpu()
            ew = max(ew, float((wd - SD).abs().max() / SD.abs().max().clamp_min(1e-300)))
        ref, util = _oracle_cell(grid, reals, g, yi, pi, SD, Sr)
        got = grid.beta[g, yi, pi].cpu()
        eb = max(eb, float(((got - ref).norm(dim=-1) / ref.norm(dim=-1).clamp_min(1e-300)).max()))
        for i, oref in util:
            ogot = obj_host[i, g, pi]
            eo = max(eo, float(((ogot - oref).abs() / oref.abs().clamp_min(1e-12)).max()))
    out = {"cells": len(picks), "beta_max_rel_err": eb, "obj_max_rel_err": eo,
           "window_sums_max_rel_err": ew if full else None}
    log.info(f"check vs CPU oracle on {len(picks)} cells: beta {eb:.2e}, utilities {eo:.2e}")
    return out


def nonfinite_cells(grid: GridResult) -> list:
    """(g, local year, p) cells whose coefficients are not finite for some lambda (after the
    device repair a non-finite cell means a fault, or a system singular even for pivoted LU)."""
    G, nYl, nP = grid.beta.shape[:3]
    out = []
    if nYl == 0:
        return out
    for pi, p in enumerate(grid.p_vec):
        ok = torch.isfinite(grid.beta[:, :, pi, :, : int(p) + 1]).flatten(2).all(-1)   # [G, nYl]
        for g, yi in torch.nonzero(~ok).cpu().numpy():
            out.append((int(g), int(yi), pi))
    return sorted(out)


def recompute_cells(grid: GridResult, reals: PfmlReals, cells) -> dict:
    """Failure recovery: recompute the coefficients of ``cells`` [(g, local
    year, p)] and their validation utilities with the fp64 CPU oracle - one pivoted-LU solve
    per lambda (np.linalg.solve semantics: an exactly singular system stays NaN, where the
    reference raises) on the rank's own window sums (kept by grid_search; the fault being
    repaired is in the solves, the summands were checked finite in S4) - and write them back
    into ``grid``.  Works on every rank: call it before ``gather_grid`` (the utilities are
    still local).  Returns counts."""
    if grid.gathered and dist_env().is_dist:
        raise RuntimeError("recompute_cells: repair the local grid before gather_grid")
    still = 0
    for g, yi, pi in cells:
        n = int(grid.p_vec[pi]) + 1
        b, util = _oracle_cell(grid, reals, g, yi, pi)
        grid.beta[g, yi, pi] = b.to(grid.beta.device)
        still += int(not bool(torch.isfinite(b[:, :n]).all()))
        for i, o in util:
            grid.obj[i, g, pi] = o.to(grid.obj.device)
    return {"recomputed": len(cells), "singular": still}


# ---------------------------------------------------------------------------------------
# Scores (K17): expanding mean by (p, l) over eom_ret, dense rank per eom_ret.
# ---------------------------------------------------------------------------------------
def _cumsum0(x: torch.Tensor) -> torch.Tensor:
    """cumsum along dim 0 as an innermost-dim scan (the outer-dim scan kernel of torch-ROCm
    takes ~0.2-0.4 ms on these [months, cells] shapes; the innermost one ~30 us)."""
    n = x.shape[0]
    y = x.reshape(n, -1).t().contiguous().cumsum(dim=1)
    return y.t().reshape(x.shape)


def validation_scores(obj: torch.Tensor, frame_g: int, compat: bool):
    """cum_obj and dense rank for the validation frame of ``frame_g``.

    obj: [nVal, G, nP, L].  In compat mode (quirk Q2, PFML_hp_reals.py:60) the frame of g
    holds the rows of every g' <= g, interleaved per month in g order (stable sort by
    (p, l, eom_ret)); otherwise only g's own rows.
    Returns (obj_seq, cum, rank) each [nVal, k, nP, L] with k = frame_g+1 (compat) or 1.
    """
    g0, g1 = (0, frame_g + 1) if compat else (frame_g, frame_g + 1)
    seq = obj[:, g0:g1]
    nV, k, nP, L = seq.shape
    if nat.is_device(obj) and k * nP * L <= nat.hip_lib().pfml_scores_max_per_month():
        # csrc/scores.hip: chunked prefix mean + per-month bitonic dense rank, two launches
        o = obj.contiguous()
        cum = torch.empty((nV, k, nP, L), dtype=obj.dtype, device=obj.device)
        rank = torch.empty_like(cum)
        nat.check(nat.hip_lib().pfml_validation_scores(o.data_ptr(), nV, o.shape[1], g0, g1,
                                                       nP * L, cum.data_ptr(), rank.data_ptr(),
                                                       nat.stream_of(o)),
                  "pfml_validation_scores")
        return seq, cum, rank
    flat = seq.reshape(nV * k, nP, L)
    # pandas expanding().mean(): NaN skipped (NaN until the first finite value)
    ok = ~torch.isnan(flat)
    cnt = _cumsum0(ok.to(flat.dtype))
    tot = _cumsum0(torch.where(ok, flat, torch.zeros_like(flat)))
    cum = torch.where(cnt > 0, tot / cnt.clamp_min(1.0),
                      torch.full_like(tot, float("nan"))).view(nV, k, nP, L)
    # dense rank (descending) within each month over k * nP * L rows; NaN unranked
    vals = cum.reshape(nV, -1)
    isn = torch.isnan(vals)
    key = torch.where(isn, torch.full_like(vals, float("-inf")), vals)
    sv, idx = torch.sort(key, dim=1, descending=True, stable=True)
    snan = torch.gather(isn, 1, idx)
    # NaN after every number, a real -inf included (stable: value order kept within groups)
    o2 = torch.sort(snan.to(torch.int8), dim=1, stable=True)[1]
    sv, idx, snan = sv.gather(1, o2), idx.gather(1, o2), snan.gather(1, o2)
    new = torch.ones_like(sv, dtype=torch.int64)
    new[:, 1:] = (sv[:, 1:] != sv[:, :-1]).to(torch.int64)
    new[snan] = 0
    dense = torch.cumsum(new, dim=1).to(vals.dtype)
    dense[snan] = float("nan")
    rank = torch.empty_like(vals)
    rank.scatter_(1, idx, dense)
    return seq, cum, rank.view(nV, k, nP, L)


def validation_scores_all(obj: torch.Tensor, compat: bool) -> list:
    """validation_scores for every frame g = 0 .. G-1; on the device all frames go through
    ONE prefix-mean and ONE dense-rank launch (csrc/scores.hip, blockIdx.y = frame)."""
    nV, G, nP, L = obj.shape
    kmax = G if compat else 1
    if not (nat.is_device(obj) and kmax * nP * L <= nat.hip_lib().pfml_scores_max_per_month()):
        return [validation_scores(obj, g, compat) for g in range(G)]
    o = obj.contiguous()
    ks = [(g + 1) if compat else 1 for g in range(G)]
    tot = nV * sum(ks) * nP * L
    cum_all = torch.empty(tot, dtype=obj.dtype, device=obj.device)
    rank_all = torch.empty_like(cum_all)
    nat.check(nat.hip_lib().pfml_validation_scores_all(o.data_ptr(), nV, G, nP * L, int(compat),
                                                       cum_all.data_ptr(), rank_all.data_ptr(),
                                                       nat.stream_of(o)),
              "pfml_validation_scores_all")
    out, off = [], 0
    for g, k in enumerate(ks):
        n = nV * k * nP * L
        g0 = 0 if compat else g
        out.append((obj[:, g0:g0 + k], cum_all[off:off + n].view(nV, k, nP, L),
                    rank_all[off:off + n].view(nV, k, nP, L)))
        off += n
    return out


def validation_frame(grid: GridResult, cfg: Config) -> pd.DataFrame:
    """validation.csv (columns eom, eom_ret, obj, l, p, hp_end, cum_obj, rank, g)."""
    compat = cfg.run.compat_mode
    G = grid.obj.shape[1]
    frames = []
    order = np.argsort(grid.val_months, kind="stable")
    obj = grid.obj[torch.as_tensor(order, device=grid.obj.device)]
    vm, vy = grid.val_months[order], grid.val_year[order]
    eom = month_end(vm)
    eom_ret = month_end(vm + 1)
    nP, L = len(grid.p_vec), len(grid.l_vec)
    for g, (seq, cum, rank) in enumerate(validation_scores_all(obj, compat)):
        nV, k = seq.shape[:2]
        # rows sorted by (p, l, eom_ret, g') as the reference's stable sort leaves them
        o = seq.permute(2, 3, 0, 1).reshape(-1).cpu().numpy()
        c = cum.permute(2, 3, 0, 1).reshape(-1).cpu().numpy()
        r = rank.permute(2, 3, 0, 1).reshape(-1).cpu().numpy()
        pp = np.repeat(np.asarray(grid.p_vec), L * nV * k)
        ll = np.tile(np.repeat(np.arange(L), nV * k), nP)
        mm = np.tile(np.repeat(np.arange(nV), k), nP * L)
        frames.append(pd.DataFrame({
            "eom": eom[mm], "eom_ret": eom_ret[mm], "obj": o, "l": ll, "p": pp,
            "hp_end": vy[mm], "cum_obj": c, "rank": r, "g": g}))
    return pd.concat(frames, ignore_index=True)


def gather_beta(grid: GridResult) -> tuple[np.ndarray, torch.Tensor]:
    """All hp years' coefficients on every rank: (years, beta [G, nY, nP, L, P])."""
    env = dist_env()
    b = grid.beta.permute(1, 0, 2, 3, 4).contiguous()       # [nYl, G, nP, L, P]
    if not env.is_dist:
        return np.asarray(grid.years_local), b.permute(1, 0, 2, 3, 4).contiguous()
    nY = len(grid.years)
    counts = [len(rank_years(nY, env.world_size, r)) for r in range(env.world_size)]
    b = coll.all_gather_known(b, counts)                    # years split contiguously
    return np.asarray(grid.years), b.permute(1, 0, 2, 3, 4).contiguous()
