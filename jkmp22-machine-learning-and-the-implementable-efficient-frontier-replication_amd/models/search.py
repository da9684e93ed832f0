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

Distributed: hp years are split contiguously over ranks.  Each rank sums only its own
window blocks; the cross-rank exclusive prefix of the block totals is ONE all-gather of a
P x P matrix per g per rank and the per-month utilities are ONE all-gather at
the end (a few MB; every rank's row count follows from the shared plan).
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

    ``months`` are the months held here; with ``all_months`` set they are a contiguous window
    of that global list (a rank's hp-year shard plus its validation halo, see
    ``local_month_range``) and the search plans over the global list."""
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
                      burn_stop, count, val_start.astype(np.int64), val_stop.astype(np.int64))


def local_month_range(all_months: np.ndarray, years: np.ndarray, world: int,
                      rank: int) -> tuple[int, int]:
    """[lo, hi) rows of ``all_months`` that the rank owning a contiguous share of the hp years
    needs: its own expanding-window blocks (rank 0 also the burn-in), and the
    validation months of its last year - the next year's block - as a halo.  Every rank thus
    computes the S4 summands of its own months only; the window prefixes cross ranks as one
    P x P all-gather of block totals, no per-month matrix is ever exchanged."""
    plan = make_plan(np.asarray(all_months, np.int64), np.asarray(years))
    yl = list(coll.contiguous_split(len(years), world, rank))
    if not yl:
        return 0, 0
    lo = 0 if yl[0] == 0 else int(plan.seg_start[yl[0]])
    hi = max(int(plan.seg_stop[yl[-1]]), int(plan.val_stop[yl[-1]]))
    return lo, hi


@dataclass
class GridResult:
    years: np.ndarray
    p_vec: list
    l_vec: np.ndarray
    years_local: np.ndarray            # hp years whose betas live on this rank
    beta: torch.Tensor                 # [G, nY_local, nP, L, P] (zero beyond p+1)
    val_months: np.ndarray             # [nVal] month indices of all validation rows
    val_year: np.ndarray               # [nVal] hp_end of each validation month
    obj: torch.Tensor                  # [nVal, G, nP, L]  (all ranks, gathered)
    timings: dict = field(default_factory=dict)


_SETUP: dict = {}


def _search_setup(months: np.ndarray, years: np.ndarray, p_vec, G: int, T: int, world: int,
                  rank: int, dev, l_vec: np.ndarray, off: int = 0) -> dict:
    """Everything of a grid search that depends only on its shape - the window plan, this
    rank's segments, cells and validation jobs, and the device copies of the segment bounds -
    built once per shape and reused by every later search (no host planning, no host->device
    copies in the steady state).  ``months`` is the global month list; the T months held
    locally start at global row ``off`` (all local row indices below are relative to it)."""
    key = (months.tobytes(), np.asarray(years).tobytes(), tuple(p_vec), G, T, world, rank,
           str(dev), l_vec.tobytes(), off)
    hit = _SETUP.get(key)
    if hit is not None:
        return hit
    plan = make_plan(months, years)
    yl = np.asarray(list(coll.contiguous_split(len(years), world, rank)), dtype=np.int64)
    nYl = len(yl)
    nP = len(p_vec)
    st = [int(plan.seg_start[i]) - off for i in yl]
    sp = [int(plan.seg_stop[i]) - off for i in yl]
    if nYl and yl[0] == 0:
        st = [0 - off] + st
        sp = [plan.burn_stop - off] + sp
    if any(a < 0 or b > T for a, b in zip(st, sp)):
        raise ValueError(f"rank {rank}: local months [{off}, {off + T}) miss its window blocks")
    nseg = len(st)
    starts = np.concatenate([np.asarray(st, np.int64) + g * T for g in range(G)]).astype(np.int32)
    stops = np.concatenate([np.asarray(sp, np.int64) + g * T for g in range(G)]).astype(np.int32)
    pv = np.asarray(p_vec, dtype=np.int64)
    gg, yy, pp = np.meshgrid(np.arange(G), np.arange(nYl), np.arange(nP), indexing="ij")
    cell_src = (gg * nYl + yy).reshape(-1)                 # cell order [g][year][p]
    cell_n = (pv[pp] + 1).reshape(-1)
    cnt = np.maximum(np.asarray(plan.count, dtype=np.int64)[yl], 1) if nYl else np.zeros(0)
    cell_scale = (1.0 / cnt[yy].astype(np.float64)).reshape(-1)
    # job order: [val month][g][p]  -> obj reshapes to [nValLocal, G, nP, L]
    vs = np.asarray(plan.val_start, dtype=np.int64)[yl] - off if nYl else np.zeros(0, np.int64)
    ve = np.asarray(plan.val_stop, dtype=np.int64)[yl] - off if nYl else np.zeros(0, np.int64)
    if nYl and (vs.min() < 0 or ve.max() > T):
        raise ValueError(f"rank {rank}: local months [{off}, {off + T}) miss its validation halo")
    nv = ve - vs
    v_yi = np.repeat(np.arange(nYl), nv)                   # local year index per val row
    v_m = (np.concatenate([np.arange(a, b) for a, b in zip(vs, ve)])
           if nYl else np.zeros(0, np.int64))
    nVr = len(v_m)
    vi, g2, p2 = np.meshgrid(np.arange(nVr), np.arange(G), np.arange(nP), indexing="ij")
    jc = ((g2 * nYl + v_yi[vi]) * nP + p2).reshape(-1)
    jm = (g2 * T + v_m[vi]).reshape(-1)
    jn = (pv[p2] + 1).reshape(-1)
    out = dict(plan=plan, yl=yl, nYl=nYl, st=st, sp=sp, nseg=nseg, starts=starts, stops=stops,
               cell_src=np.asarray(cell_src), cell_n=np.asarray(cell_n),
               cell_scale=np.asarray(cell_scale), v_yi=v_yi, v_m=v_m, nVr=nVr,
               jc=np.asarray(jc), jm=np.asarray(jm), jn=np.asarray(jn), dev_bounds=None,
               lvec=torch.as_tensor(l_vec, dtype=torch.float64, device=dev))
    if nseg and dev is not None and dev.type == "cuda":
        from ..ops.ridge import upload
        out["dev_bounds"] = upload([np.asarray(st, np.int32), np.asarray(sp, np.int32),
                                    starts, stops], dev)
    if len(_SETUP) > 32:
        _SETUP.clear()
    _SETUP[key] = out
    return out


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
    row_off = int(np.searchsorted(all_months, int(reals.months[0]))) if len(reals.months) else 0
    if len(reals.months) and not np.array_equal(all_months[row_off:row_off + T],
                                                np.asarray(reals.months, np.int64)):
        raise ValueError("grid_search: local months must be a contiguous window of all_months")
    su = _search_setup(all_months, np.asarray(years), p_vec, G, T, env.world_size, env.rank, dev,
                       np.asarray(cfg.l_vec, dtype=np.float64), row_off)
    lvec = su["lvec"]
    L = lvec.numel()
    plan, yl, nYl, nseg = su["plan"], su["yl"], su["nYl"], su["nseg"]

    # ---- 1. window sums over this rank's blocks ------------------------------------
    range_push("search.window_sums")
    ready = None
    if nseg and _pipelined_sums(dev, env, G, su["cell_n"]):
        # one g at a time: g's big cells start their band reductions while the next g's sums
        # stream (ridge_utilities waits per group on these events, not on the whole pass)
        SD, Sr, ready = _window_sums_pipelined(reals, su, G, P, nseg, nYl)
        totD = totr = None
    elif nseg:
        # running sums at every block end in one pass over the symmetric upper triangles
        # (the burn-in block, rank 0 only, is a prefix segment and not an output row)
        db = su["dev_bounds"]
        skip = nseg - nYl
        SD = window_prefix_sym(reals.denom, su["st"], su["sp"],
                               dev_bounds=None if db is None else db[:2], skip=skip)
        Sr = window_prefix_vec(reals.r_tilde.contiguous(), su["st"], su["sp"],
                               dev_bounds=None if db is None else db[:2], skip=skip)
        totD, totr = SD[:, -1], Sr[:, -1]
    else:
        SD = torch.zeros((G, 0, P, P), dtype=torch.float64, device=dev)
        Sr = torch.zeros((G, 0, P), dtype=torch.float64, device=dev)
        totD = torch.zeros((G, P, P), dtype=torch.float64, device=dev)
        totr = torch.zeros((G, P), dtype=torch.float64, device=dev)
    if env.is_dist:
        flat = torch.cat([totD.reshape(G, -1), totr], dim=1)
        off = coll.exclusive_prefix_sum(flat)
        SD = SD + off[:, : P * P].view(G, 1, P, P)
        Sr = Sr + off[:, P * P:].view(G, 1, P)
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
                                reals.r_tilde.reshape(G * T, P), su["jc"], su["jm"], su["jn"],
                                ready=ready)
    beta = beta.view(G, nYl, nP, L, P)
    obj = obj.view(su["nVr"], G, nP, L)
    range_pop()

    th("grid_search.ridge_utilities")
    v_y = yl[v_yi] if nYl else np.zeros(0, np.int64)
    if gather and env.is_dist:
        # every rank's share of the validation rows follows from the global plan: ONE
        # all-gather of the utilities; months and years are rebuilt locally
        range_push("search.gather")
        nv_all = np.asarray(plan.val_stop, np.int64) - np.asarray(plan.val_start, np.int64)
        counts = [int(nv_all[list(coll.contiguous_split(len(years), env.world_size, r))].sum())
                  for r in range(env.world_size)]
        obj = coll.all_gather_known(obj, counts)
        v_m = np.concatenate([np.arange(a, b) for a, b in zip(plan.val_start, plan.val_stop)])
        v_y = np.repeat(np.arange(len(years)), nv_all)
        range_pop()
    else:
        v_m = v_m + row_off                               # local rows -> global rows
    vm = all_months[v_m]
    vy = np.asarray(years, dtype=np.int64)[v_y]
    return GridResult(years=years, p_vec=p_vec, l_vec=cfg.l_vec, years_local=years[yl],
                      beta=beta, val_months=vm, val_year=vy, obj=obj)


def check_against_oracle(grid: GridResult, reals: PfmlReals, cfg: Config, ncells: int = 3,
                         seed: int = 0) -> dict:
    """``--check``: recompute a few (g, year, p) cells of this rank from scratch
    with the fp64 CPU oracle - expanding-window sums by plain summation, one
    ``torch.linalg.solve`` per lambda, quadratic forms one by one - and report the max
    relative error of the device coefficients and utilities (the largest-n cell is always
    among them)."""
    from ..ops.ridge import quadform_utilities, ridge_grid
    months = np.asarray(reals.months, dtype=np.int64)
    plan = make_plan(months, np.asarray(grid.years))
    yl = np.nonzero(np.isin(np.asarray(grid.years), np.asarray(grid.years_local)))[0]
    G, nP = reals.G, len(grid.p_vec)
    if len(yl) == 0:
        return {"cells": 0}
    rng = np.random.default_rng(seed)
    picks = {(0, len(yl) - 1, nP - 1)}
    while len(picks) < min(ncells, G * len(yl) * nP):
        picks.add((int(rng.integers(G)), int(rng.integers(len(yl))), int(rng.integers(nP))))
    lv = torch.as_tensor(grid.l_vec, dtype=torch.float64)
    denom, rt = reals.denom.cpu(), reals.r_tilde.cpu()
    obj_host = grid.obj.cpu()
    v_rows = {}
    if obj_host.shape[0] == len(grid.val_months):       # gathered or single-rank utilities
        for i, (vm, vy) in enumerate(zip(grid.val_months, grid.val_year)):
            v_rows.setdefault(int(vy), []).append((i, int(vm)))
    eb = eo = 0.0
    for g, yi, pi in sorted(picks):
        y = int(yl[yi])
        n = int(grid.p_vec[pi]) + 1
        stop = int(plan.seg_stop[y])
        SD = denom[g, :stop].sum(0)[None]
        Sr = rt[g, :stop].sum(0)[None]
        ref = ridge_grid(SD, Sr, np.array([0]), np.array([n]),
                         np.array([1.0 / max(int(plan.count[y]), 1)]), lv)[0]
        got = grid.beta[g, yi, pi].cpu()
        eb = max(eb, float(((got - ref).norm(dim=-1) / ref.norm(dim=-1).clamp_min(1e-300)).max()))
        rows = v_rows.get(int(grid.years[y]), [])
        if rows:
            jm = np.array([g * len(months) + int(np.searchsorted(months, vm)) for _, vm in rows])
            oref = quadform_utilities(denom.reshape(-1, *denom.shape[2:]),
                                      rt.reshape(-1, rt.shape[-1]), ref[None],
                                      np.zeros(len(rows), np.int64), jm, np.full(len(rows), n))
            ogot = obj_host[[i for i, _ in rows], g, pi]
            eo = max(eo, float(((ogot - oref).abs() / oref.abs().clamp_min(1e-12)).max()))
    out = {"cells": len(picks), "beta_max_rel_err": eb, "obj_max_rel_err": eo}
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
    year, p)] and their validation utilities from scratch with the fp64 CPU oracle - window
    sums by plain summation, one pivoted-LU solve per lambda (np.linalg.solve semantics: an
    exactly singular system stays NaN, where the reference raises) - and write them back into
    ``grid``.  Needs every month from the first one on this rank (world 1, or the rank that
    holds the burn-in); returns counts."""
    from ..ops.ridge import quadform_utilities, ridge_grid
    months = np.asarray(reals.months, dtype=np.int64)
    allm = np.asarray(reals.months if reals.all_months is None else reals.all_months, np.int64)
    if len(cells) and (len(months) == 0 or months[0] != allm[0]):
        raise RuntimeError("recompute_cells: this rank lacks the months before its windows")
    plan = make_plan(months, np.asarray(grid.years))
    yl = np.nonzero(np.isin(np.asarray(grid.years), np.asarray(grid.years_local)))[0]
    lv = torch.as_tensor(grid.l_vec, dtype=torch.float64)
    denom, rt = reals.denom.cpu(), reals.r_tilde.cpu()
    rows_of = {}
    if grid.obj.shape[0] == len(grid.val_months):
        for i, (vm, vy) in enumerate(zip(grid.val_months, grid.val_year)):
            rows_of.setdefault(int(vy), []).append((i, int(vm)))
    still = 0
    for g, yi, pi in cells:
        y = int(yl[yi])
        n = int(grid.p_vec[pi]) + 1
        stop = int(plan.seg_stop[y])
        SD = denom[g, :stop].sum(0)[None]
        Sr = rt[g, :stop].sum(0)[None]
        b = ridge_grid(SD, Sr, np.array([0]), np.array([n]),
                       np.array([1.0 / max(int(plan.count[y]), 1)]), lv)[0]
        grid.beta[g, yi, pi] = b.to(grid.beta.device)
        still += int(not bool(torch.isfinite(b[:, :n]).all()))
        rows = rows_of.get(int(grid.years[y]), [])
        if rows:
            jm = np.array([g * len(months) + int(np.searchsorted(months, vm)) for _, vm in rows])
            o = quadform_utilities(denom.reshape(-1, *denom.shape[2:]),
                                   rt.reshape(-1, rt.shape[-1]), b[None],
                                   np.zeros(len(rows), np.int64), jm, np.full(len(rows), n))
            grid.obj[[i for i, _ in rows], g, pi] = o.to(grid.obj.device)
    return {"recomputed": len(cells), "singular": still}


# ---------------------------------------------------------------------------------------
# Scores (K17): expanding mean by (p, l) over eom_ret, dense rank per eom_ret.
# ---------------------------------------------------------------------------------------
def _pipelined_sums(dev, env, G: int, cell_n) -> bool:
    """Per-g pipelined window sums (opt-in, PFML_PIPE_SUMS=1): one device holding the whole
    grid (not a multi-rank shard), 2 g (three streams in all) and the two-stream band policy
    (many big cells).  Measured on MI355X (profiles/r02_pipe_sums_ab.json): eager launches
    6.06-6.11 vs 6.48-6.54 ms per step, but under HIP-graph replay (the default) 6.00 vs
    6.02-6.10 ms - the graph executor regroups the three branches onto its own queues and the
    g = 1 big cells then wait ~0.3 ms for CUs behind the small cells - so it stays off."""
    import os
    from ..ops.ridge import band_policy
    if (dev.type != "cuda" or env.is_dist or G != 2
            or os.environ.get("PFML_PIPE_SUMS", "0") != "1"):
        return False
    return band_policy(np.asarray(cell_n))[1]


def _window_sums_pipelined(reals: PfmlReals, su: dict, G: int, P: int, nseg: int, nYl: int):
    """Window sums of every g into one [G, nYl, P, P] stack, g after g: g = 0 on the current
    stream, g > 0 on a side stream chained after g - 1 (the passes are HBM-bound, so running
    them concurrently would only delay g = 0); the r̄ sums (tiny) lead that side stream.
    Returns (SD, Sr, ready) with ready as ridge_utilities takes it.  Three streams in all:
    current, this side stream, and the small cells' stream in ridge_utilities."""
    from ..ops.ridge import _side_stream
    dev = reals.denom.device
    T = reals.denom.shape[1]
    db = su["dev_bounds"]
    skip = nseg - nYl
    cur = torch.cuda.current_stream(dev)
    side = _side_stream(dev, 16)
    side.wait_stream(cur)
    SD = torch.empty((G, nYl, P, P), dtype=torch.float64, device=dev)
    with torch.cuda.stream(side):
        Sr = window_prefix_vec(reals.r_tilde.contiguous(), su["st"], su["sp"],
                               dev_bounds=None if db is None else db[:2], skip=skip)
        ev_r = torch.cuda.Event()
        ev_r.record(side)
    events = []
    for g in range(G):
        st = cur if g == 0 else side
        if g > 0:
            st.wait_event(events[-1])
        with torch.cuda.stream(st):
            window_prefix_sym(reals.denom[g:g + 1], su["st"], su["sp"],
                              dev_bounds=None if db is None else db[:2], skip=skip,
                              out=SD[g:g + 1])
            ev = torch.cuda.Event()
            ev.record(st)
        events.append(ev)
    # big cells of g run on the stream that summed g (g = 0: after its sums on cur; g > 0:
    # after its sums on the side stream); only the r̄ sums need an event wait
    ready = {"key": su["cell_src"] // max(nYl, 1), "streams": [cur] + [side] * (G - 1),
             "events": [[ev_r]] + [[]] * (G - 1), "all": [events[-1], ev_r]}
    return SD, Sr, ready


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
    counts = [len(coll.contiguous_split(nY, env.world_size, r)) for r in range(env.world_size)]
    b = coll.all_gather_known(b, counts)                    # years split contiguously
    return np.asarray(grid.years), b.permute(1, 0, 2, 3, 4).contiguous()
