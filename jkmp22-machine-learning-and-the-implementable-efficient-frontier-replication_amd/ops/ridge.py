"""Hyper-parameter grid kernels: window sums (K14), ridge solves (K15), utilities (K16).

Device paths run csrc/segsum.hip, csrc/ridge.hip and csrc/quadform.hip; CPU paths are the
fp64 oracle in the reference's own formulation (np.linalg.solve per lambda,
PFML_Search_Coef.py:131-133; r'b - 1/2 b'Db per month, PFML_hp_reals.py:94).
"""
from __future__ import annotations

import ctypes as C

import os

import numpy as np
import torch

from . import _native as nat

CELL_DTYPE = np.dtype([("src", "<i8"), ("rsrc", "<i8"), ("work", "<i8"), ("out", "<i8"),
                       ("n", "<i4"), ("_pad", "<i4"), ("scale", "<f8")])
JOB_DTYPE = np.dtype([("d_off", "<i8"), ("r_off", "<i8"), ("b_off", "<i8"), ("o_off", "<i8"),
                      ("n", "<i4"), ("ptile0", "<i4")])


def segment_sums(X: torch.Tensor, starts, stops, dev_bounds=None) -> torch.Tensor:
    """out[s] = X[starts[s]:stops[s]].sum(0) for X of shape [T, ...].  ``dev_bounds``:
    device int32 copies of (starts, stops), e.g. from a cached plan (no host->device copy)."""
    T = X.shape[0]
    tail = X.shape[1:]
    starts = np.asarray(starts, dtype=np.int32)
    stops = np.asarray(stops, dtype=np.int32)
    S = len(starts)
    out = torch.empty((S, *tail), dtype=X.dtype, device=X.device)
    if nat.is_device(X):
        if X.dtype != torch.float64 or not X.is_contiguous():
            raise ValueError("segment_sums: contiguous fp64 required")
        E = X[0].numel() if T > 0 else int(np.prod(tail))
        st, sp = dev_bounds if dev_bounds is not None else upload([starts, stops], X.device)
        nat.check(nat.hip_lib().pfml_segsum(X.data_ptr(), E, st.data_ptr(), sp.data_ptr(), S,
                                            out.data_ptr(), nat.stream_of(X)), "pfml_segsum")
    else:
        for s in range(S):
            out[s] = X[starts[s]:stops[s]].sum(0)
    return out


nat.register_hip("pfml_window_prefix_vec", [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p])
nat.register_hip("pfml_window_prefix_vec_max_segments", [], C.c_int)


def window_prefix_vec(X: torch.Tensor, starts, stops, dev_bounds=None,
                      skip: int = 0) -> torch.Tensor:
    """out[g, s - skip] = sum of X[g, t] over the months of segments 0..s, for s >= skip (X:
    [G, T, E], e.g. the r_tilde vectors).  Device: one launch (csrc/segsum.hip); contiguous
    [G, S - skip, E] output."""
    G, T, E = X.shape
    starts = np.asarray(starts, dtype=np.int32)
    stops = np.asarray(stops, dtype=np.int32)
    S = len(starts)
    out = torch.empty((G, max(S - skip, 0), E), dtype=X.dtype, device=X.device)
    if S - skip <= 0:
        return out
    if nat.is_device(X) and S <= nat.hip_lib().pfml_window_prefix_vec_max_segments():
        if X.dtype != torch.float64 or not X.is_contiguous():
            raise ValueError("window_prefix_vec: contiguous fp64 required")
        st, sp = dev_bounds if dev_bounds is not None else upload([starts, stops], X.device)
        nat.check(nat.hip_lib().pfml_window_prefix_vec(
            X.data_ptr(), E, T, G, st.data_ptr(), sp.data_ptr(), S, int(skip), out.data_ptr(),
            nat.stream_of(X)), "pfml_window_prefix_vec")
        return out
    acc = torch.zeros((G, E), dtype=X.dtype, device=X.device)
    for s in range(S):
        acc = acc + X[:, starts[s]:stops[s]].sum(1)
        if s >= skip:
            out[:, s - skip] = acc
    return out


nat.register_hip("pfml_window_prefix_sym", [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                            C.c_void_p])


def window_prefix_sym(X: torch.Tensor, starts, stops, dev_bounds=None,
                      skip: int = 0, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[g, s - skip] = sum of X[g, t] over the months of segments 0..s, for s >= skip (X:
    [G, T, P, P], every X[g, t] symmetric; the first ``skip`` segments only feed the prefix).
    Device: one pass over the upper triangles (csrc/segsum.hip), contiguous output (``out``:
    a preallocated contiguous [G, S - skip, P, P] destination, e.g. one g's slice)."""
    G, T, P, _ = X.shape
    starts = np.asarray(starts, dtype=np.int32)
    stops = np.asarray(stops, dtype=np.int32)
    S = len(starts)
    if out is None:
        out = torch.empty((G, max(S - skip, 0), P, P), dtype=X.dtype, device=X.device)
    elif out.shape != (G, max(S - skip, 0), P, P) or not out.is_contiguous():
        raise ValueError("window_prefix_sym: out must be a contiguous [G, S - skip, P, P] tensor")
    if S == 0:
        return out
    if nat.is_device(X):
        if X.dtype != torch.float64 or not X.is_contiguous():
            raise ValueError("window_prefix_sym: contiguous fp64 required")
        st, sp = dev_bounds if dev_bounds is not None else upload([starts, stops], X.device)
        scratch = (torch.empty((G, skip, P, P), dtype=X.dtype, device=X.device) if skip
                   else None)
        nat.check(nat.hip_lib().pfml_window_prefix_sym(
            X.data_ptr(), P, T, G, st.data_ptr(), sp.data_ptr(), S, int(skip), out.data_ptr(),
            scratch.data_ptr() if scratch is not None else None, nat.stream_of(X)),
            "pfml_window_prefix_sym")
        return out
    acc = torch.zeros((G, P, P), dtype=X.dtype)
    for s in range(S):
        acc = acc + X[:, starts[s]:stops[s]].sum(1)
        if s >= skip:
            out[:, s - skip] = acc
    return out


nat.register_hip("pfml_wsum_chunk_totals", [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                            C.c_int, C.c_void_p, C.c_void_p, C.c_int64,
                                            C.c_void_p])
nat.register_hip("pfml_wsum_chunk_prefix", [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                            C.c_int64, C.c_int, C.c_void_p])
nat.register_hip("pfml_wvec_chunk", [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_void_p,
                                     C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int64,
                                     C.c_void_p, C.c_void_p])


def _fold_months(X: torch.Tensor, a: int, b: int) -> torch.Tensor:
    """CPU segment sum: left fold over months a .. b-1 of X [G, T, ...] (a fixed order, the
    same on every rank that holds these months)."""
    acc = torch.zeros_like(X[:, 0])
    for t in range(a, b):
        acc = acc + X[:, t]
    return acc


def chunk_totals(X: torch.Tensor, R: torch.Tensor, su: dict):
    """Kernel A of the canonical chunked window sums (models/search.py): segment sums of this
    rank's segments and the totals of its chunks, chunk-major [nlc, G, P, P] / [nlc, G, P].
    Returns (totD, totR, bufs); ``bufs`` carries the segment sums to ``chunk_windows``."""
    G, T, P, _ = X.shape
    nlc, nseg, skip, nYl = su["nlc"], su["nseg"], su["skip"], su["nYl"]
    # matrix and vector totals of a chunk side by side in ONE row of one buffer (``bufs["tot"]``,
    # [nlc, G P P + G P]): the multi-rank path all-gathers them as one collective; totD / totR
    # are row-strided views and the kernels take that row stride
    GPP = G * P * P
    tot = torch.empty((nlc, GPP + G * P), dtype=X.dtype, device=X.device)
    totD = tot[:, :GPP].view(nlc, G, P, P)
    totR = tot[:, GPP:].view(nlc, G, P)
    out = torch.empty((G, nYl, P, P), dtype=X.dtype, device=X.device)
    if nat.is_device(X):
        if X.dtype != torch.float64 or not X.is_contiguous():
            raise ValueError("chunk_totals: contiguous fp64 required")
        scratch = (torch.empty((G, skip, P, P), dtype=X.dtype, device=X.device) if skip
                   else None)
        st, sp, idx, cidx = su["dev_idx"]
        lib = nat.hip_lib()
        s = nat.stream_of(X)
        nat.check(lib.pfml_wsum_chunk_totals(
            X.data_ptr(), P, T, G, st.data_ptr(), sp.data_ptr(), nseg, skip, out.data_ptr(),
            scratch.data_ptr() if scratch is not None else None, nlc, idx.data_ptr(),
            totD.data_ptr(), totD.stride(0), s), "pfml_wsum_chunk_totals")
        nat.check(lib.pfml_wvec_chunk(
            R.data_ptr(), P, T, G, st.data_ptr(), sp.data_ptr(), nseg, skip, 0, nlc,
            idx.data_ptr(), su["layout"].C, cidx.data_ptr(), su["clast"], totR.data_ptr(),
            totR.stride(0), None, s), "pfml_wvec_chunk")
        return totD, totR, {"out": out, "scratch": scratch, "tot": tot}
    segD = [_fold_months(X, a, b) for a, b in zip(su["st"], su["sp"])]
    segR = [_fold_months(R, a, b) for a, b in zip(su["st"], su["sp"])]
    for lc in range(nlc):
        accD, accR = torch.zeros_like(X[:, 0]), torch.zeros_like(R[:, 0])
        for s in range(int(su["cs"][lc]), int(su["ce"][lc])):
            accD = accD + segD[s]
            accR = accR + segR[s]
        totD[lc], totR[lc] = accD, accR
    return totD, totR, {"out": out, "segD": segD, "segR": segR, "tot": tot}


def chunk_windows(X: torch.Tensor, R: torch.Tensor, su: dict, totD: torch.Tensor,
                  totR: torch.Tensor, bufs: dict) -> tuple[torch.Tensor, torch.Tensor]:
    """Kernel B of the canonical chunked window sums: E = fold of the burn-in totals, then per
    year chunk the fold of its segments from the prefix P_c (``totD``/``totR``: every chunk's
    total, gathered, in the canonical slot order of ``su``).  Returns (SD, Sr)."""
    G, T, P, _ = X.shape
    nseg, skip, nYl, clast = su["nseg"], su["skip"], su["nYl"], su["clast"]
    C = su["layout"].C
    out = bufs["out"]
    nslot = int(sum(su["counts"]))
    if totD.shape[0] != nslot or totR.shape[0] != nslot:
        # the slot map addresses the GATHERED totals of every rank (a local-only buffer here
        # would be read out of bounds by the device kernels)
        raise ValueError(f"chunk_windows: {totD.shape[0]} chunk totals, the canonical layout "
                         f"has {nslot} slots (all-gather missing?)")
    Sr = torch.empty((G, nYl, P), dtype=X.dtype, device=X.device)
    if nat.is_device(X):
        st, sp, idx, cidx = su["dev_idx"]
        lib = nat.hip_lib()
        s = nat.stream_of(X)
        scratch = bufs["scratch"]
        # (row-strided totals: each slot's G blocks contiguous, the slots totD.stride(0) apart)
        if totD.stride()[1:] != (P * P, P, 1) or totR.stride()[1:] != (P, 1):
            raise ValueError("chunk_windows: chunk totals must be row-strided [slot][g] blocks")
        nat.check(lib.pfml_wsum_chunk_prefix(
            P, G, nseg, skip, out.data_ptr(), scratch.data_ptr() if scratch is not None else None,
            C, cidx.data_ptr(), totD.data_ptr(), totD.stride(0), clast, s),
            "pfml_wsum_chunk_prefix")
        nat.check(lib.pfml_wvec_chunk(
            R.data_ptr(), P, T, G, st.data_ptr(), sp.data_ptr(), nseg, skip, 1, 0,
            idx.data_ptr(), C, cidx.data_ptr(), clast, totR.data_ptr(), totR.stride(0),
            Sr.data_ptr(), s), "pfml_wvec_chunk")
        return out, Sr
    segD, segR = bufs["segD"], bufs["segR"]
    pD, pR = torch.zeros_like(X[:, 0]), torch.zeros_like(R[:, 0])
    for k in range(C):
        pD = pD + totD[int(su["sb"][k])]
        pR = pR + totR[int(su["sb"][k])]
    for c in range(clast + 1):
        aD, aR = pD, pR
        for s in range(int(su["ys"][c]), int(su["ye"][c])):
            aD = aD + segD[s]
            aR = aR + segR[s]
            if s >= skip:
                out[:, s - skip] = aD
                Sr[:, s - skip] = aR
        if c < clast:
            pD = pD + totD[int(su["sy"][c])]
            pR = pR + totR[int(su["sy"][c])]
    return out, Sr


class _HostClock:
    """PFML_HOST_TIMING=1: print host-side section times (microseconds) to stderr;
    PFML_HOST_TIMING=sync: synchronise the device at every mark (section = wall time of the
    queued work)."""

    def __init__(self):
        import os
        import time
        v = os.environ.get("PFML_HOST_TIMING", "")
        self.on = bool(v)
        self.sync = v == "sync" and torch.cuda.is_available()
        self.time = time.perf_counter
        if self.sync:
            torch.cuda.synchronize()
        self.t = self.time()

    def __call__(self, what: str) -> None:
        if self.on:
            import sys
            if self.sync:
                torch.cuda.synchronize()
            now = self.time()
            print(f"[host] {what}: {1e6 * (now - self.t):.0f} us", file=sys.stderr)
            self.t = now


def upload(arrays, device) -> list[torch.Tensor]:
    """Copy several small host arrays to the device with ONE pinned, non-blocking H2D copy
    (the host never waits for queued kernels).  Returns uint8 device views, one per array."""
    offs, nbytes = [], 0
    for a in arrays:
        offs.append(nbytes)
        nbytes += (a.nbytes + 255) // 256 * 256
    host = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    for a, o in zip(arrays, offs):
        hv[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    dev = host.to(device, non_blocking=True)
    return [dev[o:o + a.nbytes] for a, o in zip(arrays, offs)]


_WORK_CACHE: dict = {}


def _work_doubles(n_arr: np.ndarray, L: int) -> np.ndarray:
    lib = nat.hip_lib()
    out = np.empty(len(n_arr), dtype=np.int64)
    for n in np.unique(n_arr):
        key = (int(n), L)
        if key not in _WORK_CACHE:
            _WORK_CACHE[key] = int(lib.pfml_ridge_work_doubles(int(n), L))
        out[n_arr == n] = _WORK_CACHE[key]
    return out


COOP_KMAX = 16          # workgroups per cell of the cooperative band reduction (wgmap: 4 bits)
COOP_SYNC_WORDS = 32    # csrc/ridge_band.hip COOP_SYNC: int32 sync words per cell


COOP_BIG_SHARE = 0.42   # share of the CUs the largest cells' cooperative launch gets (coop_k)


def coop_k(cell_n: np.ndarray, ncu: int) -> np.ndarray:
    """Workgroups per cell of the cooperative band reduction.

    The largest-n cells of a launch are the p = 512 cells (n > 256: 32 panels, the grid step's
    critical chain); they share about COOP_BIG_SHARE of the chip's CUs, round(0.42 ncu / n_big)
    workgroups each (at least 1, at most COOP_KMAX), and every other cell gets one workgroup:
    the smaller cells' whole chain (reduction, solves, back-transform, utilities) runs on the
    rest from a second stream and must keep pace.  Measured on the one-GPU rank rehearsal
    (tools/gpu_run.sh shardk, profiles/r04_coop_k_sweep.json): the best K is 1 / 2 / 4 / 6-8 at
    W = 1 / 2 / 4 / 8 ranks (106 / 53 / 27 / 13 big cells per rank), i.e. ~106 of 256 CUs for the
    big cells whatever W - giving them all the CUs the small cells leave (K = 16 at W = 8) was
    27 % slower per rank.  The betas do not depend on K (bitwise: see band_coop_kernel), only
    the time does.  PFML_COOP_K=k forces k for the largest cells."""
    n = np.asarray(cell_n)
    k = np.ones(len(n), dtype=np.int64)
    if not len(n):
        return k
    big = n == n.max()
    v = os.environ.get("PFML_COOP_K")
    if v:
        kb = int(v)
    elif int(n.max()) > 256:
        kb = int(round(COOP_BIG_SHARE * ncu / int(big.sum())))
    else:
        kb = 1
    k[big] = min(max(kb, 1), COOP_KMAX)
    return k


def coop_wgmap(k: np.ndarray) -> np.ndarray:
    """Block -> (cell, rank, K) codes ``cell << 8 | w << 4 | K - 1`` for cells in plan order.
    Runs of up to 8 cells with the same K are interleaved (block b and b + 8 hold ranks w and
    w + 1 of one cell: the same XCD under the observed round-robin placement - speed only)."""
    codes = []
    c = 0
    nc = len(k)
    while c < nc:
        g = 1
        while c + g < nc and g < 8 and k[c + g] == k[c]:
            g += 1
        for w in range(int(k[c])):
            for j in range(g):
                codes.append(((c + j) << 8) | (w << 4) | (int(k[c]) - 1))
        c += g
    return np.asarray(codes, dtype=np.int32)


_NCU: dict = {}


def ranks_per_device() -> int:
    """Processes of this node sharing one device (torchrun's LOCAL_WORLD_SIZE over the visible
    devices, ranks placed LOCAL_RANK mod device_count): 1 on an N-GPU node with one rank per
    GPU, W in the one-GPU multi-process rehearsal."""
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    nd = max(1, torch.cuda.device_count())
    return max(1, -(-lw // nd))


def num_cus(dev) -> int:
    """CUs this process may count on for the cooperative reduction: the device's, split among
    the processes that share it.  A cooperative cell's K workgroups wait for each other, so
    they must be co-resident; several processes each filling the whole chip with spinning
    workgroups would starve each other (their cells time out)."""
    key = str(dev)
    if key not in _NCU:
        _NCU[key] = int(torch.cuda.get_device_properties(dev).multi_processor_count)
    return max(1, _NCU[key] // ranks_per_device())


def ridge_plan(P: int, L: int, cell_src, cell_n, cell_scale, ncu: int = 256) -> dict:
    """Host-side descriptors of one ridge-grid launch (CELL_DTYPE, big cells first) and the
    workgroup map of the cooperative reduction (``ncu``: the device's CUs)."""
    lib = nat.hip_lib()
    if lib.pfml_ridge_cell_desc_size() != CELL_DTYPE.itemsize:
        raise RuntimeError("CellDesc layout mismatch between python and libpfml_hip")
    nc = len(cell_src)
    cell_n = np.asarray(cell_n)
    wsz = _work_doubles(cell_n, L)
    desc = np.zeros(nc, dtype=CELL_DTYPE)
    desc["src"] = np.asarray(cell_src, np.int64) * P * P
    desc["rsrc"] = np.asarray(cell_src, np.int64) * P
    desc["out"] = np.arange(nc, dtype=np.int64) * L * P
    desc["n"] = cell_n.astype(np.int32)
    desc["scale"] = np.asarray(cell_scale, np.float64)
    # big cells first: they bound the kernel's makespan
    order = np.argsort(-desc["n"], kind="stable")
    desc = desc[order]
    wsz = wsz[order]
    desc["work"] = np.concatenate([[0], np.cumsum(wsz)[:-1]])
    wgmap = coop_wgmap(coop_k(desc["n"], ncu))
    # host copy of n in plan order: the back-transform's instance per size class
    n_host = np.ascontiguousarray(desc["n"], dtype=np.int32)
    return {"desc": desc, "work": int(wsz.sum()), "nmax": int(cell_n.max()), "nc": nc,
            "wgmap": wgmap, "n_host": n_host}


nat.register_hip("pfml_ridge_repair", [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int,
                                       C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int64,
                                       C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p])
nat.register_hip("pfml_ridge_repair_work_doubles", [C.c_int], C.c_int64)
nat.register_hip("pfml_ridge_repair_work_doubles_cap", [C.c_int, C.c_int], C.c_int64)
_REPAIR_WORK: dict = {}

# device repair counts of the most recent ridge launches (int32 device scalars; read them
# only when reporting - reading forces a sync)
LAST_REPAIRS: list = []


def repair_launch(plan: dict, d_desc: torch.Tensor, SD: torch.Tensor, Sr: torch.Tensor,
                  lv: torch.Tensor, beta: torch.Tensor) -> torch.Tensor:
    """Queue the device repair of the NaN-marked (non-SPD) systems of one ridge launch
    (csrc/ridge_repair.hip: pivoted-LU re-solve, np.linalg.solve semantics) on the current
    stream; returns the device count of repaired systems (no host sync)."""
    P = SD.shape[-1]
    L = int(lv.numel())
    lib = nat.hip_lib()
    count = torch.zeros(1, dtype=torch.int32, device=SD.device)
    cap = plan["nc"] * L
    lst = torch.empty(cap, dtype=torch.int32, device=SD.device)
    # scratch sized by the launch's own capacity and kept per (device, size): allocated once,
    # not per launch (540 MB per tridiagonal-path launch at n = 1025)
    nwd = int(lib.pfml_ridge_repair_work_doubles_cap(plan["nmax"], cap))
    wkey = (str(SD.device), nat.stream_of(SD), nwd)     # (per stream: no sharing across streams)
    # never evicted: a HIP graph that captured a launch keeps this buffer's raw pointer (it is
    # not in the graph's private pool), so freeing it would hand the graph's scratch to other
    # tensors; one buffer per (device, stream, size) key stays bounded
    work = _REPAIR_WORK.get(wkey)
    if work is None:
        work = _REPAIR_WORK[wkey] = torch.empty(nwd, dtype=torch.float64, device=SD.device)
    nat.check(lib.pfml_ridge_repair(SD.data_ptr(), P, Sr.data_ptr(), d_desc.data_ptr(),
                                    plan["nc"], plan["nmax"], lv.data_ptr(), L, beta.data_ptr(),
                                    beta.shape[-1], lst.data_ptr(), count.data_ptr(), cap,
                                    work.data_ptr(), nat.stream_of(SD)), "pfml_ridge_repair")
    return count


def repairs_done() -> int:
    """Host read of the repair counts of the last grid launches (one sync)."""
    return int(sum(int(c.item()) for c in LAST_REPAIRS))


def _n_host_ptr(plan: dict):
    """Host pointer to the plan's per-cell n (read during the launch call only);
    PFML_BT_CLASSES=0: None, every cell on the 8-wave back-transform."""
    if os.environ.get("PFML_BT_CLASSES", "1") == "0" or "n_host" not in plan:
        return None
    return plan["n_host"].ctypes.data


def band_path(plan: dict) -> bool:
    """True when the launch takes the band path (ridge_band.hip, n <= 528), whose non-SPD
    lambdas are repaired in the band domain inside the launch; the tridiagonal path
    (ridge.hip, 528 < n <= 1024) leaves NaN markers for ``repair_launch``."""
    return plan["nmax"] <= nat.hip_lib().pfml_ridge_band_nmax()


def ridge_launch(plan: dict, d_desc: torch.Tensor, SD: torch.Tensor, Sr: torch.Tensor,
                 lv: torch.Tensor, beta: torch.Tensor, repair: bool = True,
                 d_wgmap: torch.Tensor | None = None) -> torch.Tensor | None:
    """Queue one ridge-grid launch; returns the device count of non-SPD systems re-solved by
    the band path's pivoted banded LU (kernel 2b of ridge_band.hip), None when the launch has
    no in-band repair (``repair=False`` or the tridiagonal path).  ``d_wgmap``: the device
    copy of plan["wgmap"] (the cooperative band reduction's workgroup map)."""
    P = SD.shape[-1]
    L = int(lv.numel())
    work = torch.empty(plan["work"], dtype=torch.float64, device=SD.device)
    count = lst = None
    band = band_path(plan)
    if repair and band:
        count = torch.empty(1, dtype=torch.int32, device=SD.device)   # zeroed by the solve
        lst = torch.empty(plan["nc"] * L, dtype=torch.int32, device=SD.device)
    if band and d_wgmap is None:
        raise ValueError("ridge_launch: the cooperative reduction needs the device wgmap")
    sync = (torch.empty(plan["nc"] * COOP_SYNC_WORDS, dtype=torch.int32, device=SD.device)
            if band else None)
    if band:
        _spin_from_env()
        # every launch's sync words are kept until the next grid search starts (the big and the
        # small cells' launches run on two streams: neither may hide the other's timeouts)
        LAST_COOP_SYNC.append(sync)
    nat.check(nat.hip_lib().pfml_ridge_grid(SD.data_ptr(), P, Sr.data_ptr(), d_desc.data_ptr(),
                                            plan["nc"], plan["nmax"], lv.data_ptr(), L,
                                            work.data_ptr(), beta.data_ptr(), beta.shape[-1],
                                            lst.data_ptr() if lst is not None else None,
                                            count.data_ptr() if count is not None else None,
                                            plan["nc"] * L,
                                            d_wgmap.data_ptr() if band else None,
                                            len(plan["wgmap"]) if band else 0,
                                            sync.data_ptr() if band else None,
                                            _n_host_ptr(plan), nat.stream_of(SD)),
              "pfml_ridge_grid")
    return count


# sync words of the cooperative launches since the last ``reset_coop_sync`` (one per launch;
# the error word is index 1 of every cell's COOP_SYNC_WORDS): a timed-out cell's betas are NaN
# (the back-transform poisons them) and the grid search's non-finite recovery recomputes them
LAST_COOP_SYNC: list = []
nat.register_hip("pfml_coop_set_spin_max", [C.c_uint], None)


def reset_coop_sync() -> None:
    LAST_COOP_SYNC.clear()


def coop_errors() -> int:
    """Number of cells whose cooperative hand-off wait timed out, over every launch since the
    last ``reset_coop_sync`` (one host sync)."""
    if not LAST_COOP_SYNC:
        return 0
    return int(sum(int((s.view(-1, COOP_SYNC_WORDS)[:, 1] != 0).sum().item())
                   for s in LAST_COOP_SYNC))


_SPIN_ENV: list = []


def set_coop_spin_max(n: int) -> None:
    """Poll bound of the cooperative reduction's waits for later launches (0: the default,
    ~1 s).  Tests lower it to force timeouts; ``PFML_COOP_SPIN_MAX`` sets it before the first
    launch."""
    _SPIN_ENV[:] = [True]
    nat.hip_lib().pfml_coop_set_spin_max(int(n))


def _spin_from_env() -> None:
    if not _SPIN_ENV:
        set_coop_spin_max(int(os.environ.get("PFML_COOP_SPIN_MAX", "0") or 0))


def ridge_grid(SD: torch.Tensor, Sr: torch.Tensor, cell_src: np.ndarray, cell_n: np.ndarray,
               cell_scale: np.ndarray, lvec: torch.Tensor, repair: bool = True) -> torch.Tensor:
    """beta[c, l, :n_c] = solve(SD[src_c][:n,:n]*scale_c + l I, Sr[src_c][:n]*scale_c).

    SD: [S, P, P] running sums, Sr: [S, P]; returns [ncells, L, P] (zero beyond n_c).
    Non-SPD systems (NaN-marked by the banded Cholesky) are re-solved on the device by a
    pivoted banded LU before the back-transform (band path) or a dense pivoted LU after it
    (tridiagonal path, ``repair_launch``), no host sync; ``repair=False`` leaves the NaNs.
    """
    S, P, _ = SD.shape
    L = int(lvec.numel())
    nc = len(cell_src)
    beta = torch.zeros((nc, L, P), dtype=SD.dtype, device=SD.device)
    if nc == 0:
        return beta
    if nat.is_device(SD):
        reset_coop_sync()
        plan = ridge_plan(P, L, cell_src, cell_n, cell_scale, ncu=num_cus(SD.device))
        d_desc, d_wg = upload([plan["desc"], plan["wgmap"]], SD.device)
        lv = lvec.to(device=SD.device, dtype=torch.float64).contiguous()
        SDc, Src = SD.contiguous(), Sr.contiguous()
        count = ridge_launch(plan, d_desc, SDc, Src, lv, beta, repair=repair, d_wgmap=d_wg)
        if repair:
            LAST_REPAIRS[:] = [count if count is not None
                               else repair_launch(plan, d_desc, SDc, Src, lv, beta)]
        return beta
    eye_cache = {}
    lv = lvec.to(dtype=SD.dtype)
    for c in range(nc):
        n, s = int(cell_n[c]), int(cell_src[c])
        A = SD[s, :n, :n] * float(cell_scale[c])
        r = Sr[s, :n] * float(cell_scale[c])
        if n not in eye_cache:
            eye_cache[n] = torch.eye(n, dtype=SD.dtype)
        sys_ = A.unsqueeze(0) + lv.view(-1, 1, 1) * eye_cache[n]
        sol, info = torch.linalg.solve_ex(sys_, r.unsqueeze(0).expand(L, n).unsqueeze(-1))
        sol = sol.squeeze(-1)
        sol[info != 0] = float("nan")          # singular system (reference: LinAlgError)
        beta[c, :, :n] = sol
    return beta


def repair_nonspd(beta, SD, Sr, cell_src, cell_n, cell_scale, lv) -> np.ndarray:
    """Host-side reference of the repair: re-solve the NaN-marked (cell, lambda) systems with
    torch's pivoted LU (np.linalg.solve semantics, PFML_Search_Coef.py:131-133).  The engine
    uses the device form (``repair_launch``); this one is the test oracle."""
    bad = torch.isnan(beta).any(dim=-1)
    if not bool(bad.any()):
        return np.zeros(0, dtype=np.int64)
    cells = torch.nonzero(bad.any(dim=1)).flatten().tolist()
    for c in cells:
        ls = torch.nonzero(bad[c]).flatten()
        n, s = int(cell_n[c]), int(cell_src[c])
        A = SD[s, :n, :n] * float(cell_scale[c])
        r = Sr[s, :n] * float(cell_scale[c])
        eye = torch.eye(n, dtype=A.dtype, device=A.device)
        sys_ = A.unsqueeze(0) + lv[ls].view(-1, 1, 1) * eye
        sol, info = torch.linalg.solve_ex(sys_, r.expand(len(ls), n).unsqueeze(-1))
        sol = sol.squeeze(-1)
        sol[info != 0] = float("nan")
        beta[c, ls, :n] = sol
    return np.asarray(cells, dtype=np.int64)


_SIDE: dict = {}


def _side_stream(dev: torch.device, k: int = 0) -> torch.cuda.Stream:
    """Cached secondary HIP streams per device (stream creation is not free)."""
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), k)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


def two_streams() -> bool:
    """The largest cells' ridge group and the rest on two streams (default; the small cells'
    chain fills the CUs the big cells leave idle).  PFML_RIDGE_STREAMS=1 puts them on one."""
    import os
    v = os.environ.get("PFML_RIDGE_STREAMS")
    return (v.strip() == "2") if v else True


_UTIL_PLANS: dict = {}


def _utilities_plan(P: int, L: int, dev, cell_src, cell_n, cell_scale, job_cell, job_month,
                    job_n, split: bool = True) -> dict:
    """Launch plan of ridge_utilities on a device, cached: the descriptors depend only on the
    grid's shape (cells, jobs, P, L), so repeated grid searches (every step of a run, every
    benchmark step) reuse the uploaded device copies and skip all host planning.  Each group's
    cells / jobs write straight into the full beta / obj arrays (global out offsets)."""
    key = (P, L, str(dev), split, os.environ.get("PFML_QUAD_MM", "1"),
           os.environ.get("PFML_COOP_K", ""),
           cell_src.tobytes(), cell_n.tobytes(), cell_scale.tobytes(),
           job_cell.tobytes(), job_month.tobytes(), job_n.tobytes())
    hit = _UTIL_PLANS.get(key)
    if hit is not None:
        return hit
    big = cell_n == cell_n.max()
    if split:
        # the largest cells (their own cooperative launch: the chip's CUs shared among them)
        # and the rest (one workgroup each), each group on a stream of its own
        parts = (big, ~big)
    else:
        parts = (np.ones(len(cell_n), dtype=bool),)
    groups, arrays = [], []
    for grp in parts:
        cells = np.nonzero(grp)[0]
        jobs = np.nonzero(grp[job_cell])[0]
        rp = ridge_plan(P, L, cell_src[cells], cell_n[cells], cell_scale[cells], ncu=num_cus(dev))
        # ridge_plan orders cells big-first and numbers outputs 0..: map to global rows
        rp["desc"]["out"] = cells[rp["desc"]["out"] // (L * P)].astype(np.int64) * L * P
        qp = quad_plan(P, L, P, job_cell[jobs], job_month[jobs], job_n[jobs], job_out=jobs)
        groups.append((cells, jobs, rp, qp))
        arrays += [rp["desc"], qp["desc"], qp["tile_job"], rp["wgmap"]]
    dv = upload(arrays, dev)                     # all descriptors, one async copy
    plan = {"groups": groups, "dv": dv}
    if len(_UTIL_PLANS) > 64:
        _UTIL_PLANS.clear()
    _UTIL_PLANS[key] = plan
    return plan


def check_launch_bounds(S: int, P: int, T: int, cell_src, cell_n, job_cell, job_month,
                        job_n) -> None:
    """Host-side guard before any ridge / utilities kernel sees the plan: every index the
    descriptors turn into a device address must be in range (a bad plan would otherwise be a
    GPU memory fault, not an exception)."""
    nc = len(cell_src)
    bad = []
    if nc and (int(np.min(cell_src)) < 0 or int(np.max(cell_src)) >= S):
        bad.append(f"cell_src outside [0, {S})")
    if nc and (int(np.min(cell_n)) < 1 or int(np.max(cell_n)) > P):
        bad.append(f"cell_n outside [1, {P}]")
    if len(job_cell):
        if int(np.min(job_cell)) < 0 or int(np.max(job_cell)) >= nc:
            bad.append(f"job_cell outside [0, {nc})")
        if int(np.min(job_month)) < 0 or int(np.max(job_month)) >= T:
            bad.append(f"job_month outside [0, {T})")
        if int(np.min(job_n)) < 1 or int(np.max(job_n)) > P:
            bad.append(f"job_n outside [1, {P}]")
    if bad:
        raise ValueError("ridge_utilities: invalid launch plan: " + "; ".join(bad))


def ridge_utilities(SD: torch.Tensor, Sr: torch.Tensor, cell_src, cell_n, cell_scale,
                    lvec: torch.Tensor, D: torch.Tensor, R: torch.Tensor, job_cell, job_month,
                    job_n) -> tuple[torch.Tensor, torch.Tensor]:
    """(beta, obj) = (ridge_grid(...), quadform_utilities(D, R, beta, jobs)).

    On a device the cells split into the largest-n group and the rest; each group's ridge ->
    utilities chain is issued on its own HIP stream, the big group first, so the small cells'
    chain runs on the CUs the big cells' reduction leaves idle.  (Holding the small cells'
    utilities back until the big cells' solves are done measured slower: 5.43 vs 5.12 ms, the
    big back-transform then shares the chip with them, profiles/r04_quad_after_solve_ab.json.)  beta / obj rows are written in
    place from cached launch plans, and the non-SPD systems are re-solved on the device inside
    each group's ridge launch (pivoted banded LU; no host sync, counts in ``LAST_REPAIRS``).
    """
    cell_src, cell_n = np.asarray(cell_src), np.asarray(cell_n)
    cell_scale = np.asarray(cell_scale, dtype=np.float64)
    job_cell, job_month, job_n = (np.asarray(job_cell), np.asarray(job_month),
                                  np.asarray(job_n))
    if not nat.is_device(SD):
        beta = ridge_grid(SD, Sr, cell_src, cell_n, cell_scale, lvec)
        return beta, quadform_utilities(D, R, beta, job_cell, job_month, job_n)
    split = two_streams() and len(np.unique(cell_n)) >= 2
    reset_coop_sync()
    th = _HostClock()
    S, P, _ = SD.shape
    check_launch_bounds(S, P, D.shape[0], cell_src, cell_n, job_cell, job_month, job_n)
    L = int(lvec.numel())
    nc = len(cell_src)
    dev = SD.device
    plan = _utilities_plan(P, L, dev, cell_src, cell_n, cell_scale, job_cell, job_month, job_n,
                           split=split)
    th("plans")
    # every [L, P] block is written whole by the ridge grid (zero padding past n included), so
    # no fill on the stream the big cells' chain forks from
    beta = torch.empty((nc, L, P), dtype=SD.dtype, device=dev)
    obj = torch.empty((len(job_cell), L), dtype=SD.dtype, device=dev)
    SD, Sr, D, R = SD.contiguous(), Sr.contiguous(), D.contiguous(), R.contiguous()
    lv = lvec.to(device=dev, dtype=torch.float64).contiguous()
    cur = torch.cuda.current_stream(dev)
    dv = plan["dv"]
    ng = len(plan["groups"])
    # big cells' factorisations issued first, on side streams; the small cells on `cur`
    streams = [_side_stream(dev, k) for k in range(ng - 1)] + [cur]
    for st in streams[:-1]:
        st.wait_stream(cur)
    counts = []
    for gi in range(ng):
        stream = streams[gi]
        _, _, rp, qp = plan["groups"][gi]
        with torch.cuda.stream(stream):
            cnt = ridge_launch(rp, dv[4 * gi], SD, Sr, lv, beta, d_wgmap=dv[4 * gi + 3])
            counts.append(cnt if cnt is not None else repair_launch(rp, dv[4 * gi], SD, Sr, lv, beta))
            quad_launch(qp, dv[4 * gi + 1], dv[4 * gi + 2], D, R, beta, obj)
    th("launch")
    for st in streams:
        if st == cur:
            continue
        cur.wait_stream(st)
        for t in (SD, Sr, D, R, lv, beta, obj, *counts):
            t.record_stream(st)
    LAST_REPAIRS[:] = counts
    return beta, obj


def quad_plan(P: int, L: int, Pb: int, job_cell, job_month, job_n, job_out=None) -> dict:
    """Host-side descriptors of one utilities launch (JOB_DTYPE + row-tile -> job map).
    ``job_out``: row of each job in the obj array the launch writes (default: 0..nj-1)."""
    lib = nat.hip_lib()
    if lib.pfml_quadform_job_desc_size() != JOB_DTYPE.itemsize:
        raise RuntimeError("JobDesc layout mismatch between python and libpfml_hip")
    job_n = np.asarray(job_n)
    nj = len(job_n)
    # row tiles per job as the kernel counts them (the tail index n - 1 split off when n - 1
    # is a multiple of the K step: csrc/quadform.hip quad_main)
    tiles_of = {int(v): int(lib.pfml_quadform_row_tiles(int(v))) for v in np.unique(job_n)}
    ntile = np.array([tiles_of[int(v)] for v in job_n], dtype=np.int64)
    pt0 = np.concatenate([[0], np.cumsum(ntile)[:-1]]).astype(np.int32)
    desc = np.zeros(nj, dtype=JOB_DTYPE)
    desc["d_off"] = np.asarray(job_month, np.int64) * P * P
    desc["r_off"] = np.asarray(job_month, np.int64) * P
    desc["b_off"] = np.asarray(job_cell, np.int64) * L * Pb
    desc["o_off"] = (np.arange(nj, dtype=np.int64) if job_out is None
                     else np.asarray(job_out, np.int64)) * L
    desc["n"] = job_n.astype(np.int32)
    desc["ptile0"] = pt0
    if nj and int(ntile.max()) > 32:
        raise ValueError("quad_plan: more than 32 row tiles per job (n > 32 * 64)")
    # a tile covers `mm` jobs of ONE cell (same beta, same n: its validation months), so the
    # staged beta K-tiles feed mm D tiles; an odd job out gets -1 in the spare entries
    # (2 months per tile: measured 5.90 vs 5.78 ms per grid step on MI355X - fewer resident
    # workgroups cost more than the halved beta traffic saves - so 1 is the default)
    mm = 2 if os.environ.get("PFML_QUAD_MM", "1") == "2" else 1
    jc = np.asarray(job_cell, np.int64)
    # jobs grouped by (cell, n), stable: a tile's jobs share beta AND the row / K extent
    by_cell = np.lexsort((np.arange(nj), job_n, jc))
    key = jc * 65536 + job_n.astype(np.int64)
    groups = []
    i = 0
    while i < nj:
        c = key[by_cell[i]]
        k = i
        while k < nj and key[by_cell[k]] == c and k - i < mm:
            k += 1
        groups.append(by_cell[i:k])
        i = k
    ng = len(groups)
    gj = np.full((ng, mm), -1, dtype=np.int64)
    for gi, grp in enumerate(groups):
        gj[gi, :len(grp)] = grp
    gnt = ntile[gj[:, 0]] if ng else np.zeros(0, np.int64)
    # tiles longest-first (row tile 0 of every group, then row tile 1, ...): the triangular K
    # loop of row tile rt is ~(n - 64 rt) long, so the launch ends on the short tiles;
    # entry = job << 5 | rt (the kernel writes partial slot ptile0 + rt of each live job)
    gg = np.repeat(np.arange(ng, dtype=np.int64), gnt)
    g0 = np.concatenate([[0], np.cumsum(gnt)[:-1]]).astype(np.int64) if ng else np.zeros(0, np.int64)
    rt = np.arange(len(gg), dtype=np.int64) - np.repeat(g0, gnt)
    order = np.lexsort((gg, rt))
    gg, rt = gg[order], rt[order]
    jobs_t = gj[gg]                                      # [ntiles, mm]
    if len(jobs_t) and os.environ.get("PFML_QUAD_XCD", "1") != "0":
        jobs_t, rt = _xcd_affine(jobs_t, rt, jc[jobs_t[:, 0]])
    tile_job = np.where(jobs_t >= 0, (jobs_t << 5) | rt[:, None], -1).astype(np.int32).reshape(-1)
    return {"desc": desc, "tile_job": tile_job, "nj": nj, "ntiles": len(gg),
            "nslots": int(ntile.sum()), "mm": mm}


NXCD = 8   # MI355X: workgroup b of a launch is dispatched to XCD b mod 8


def _xcd_affine(jobs_t: np.ndarray, rt: np.ndarray, cell: np.ndarray):
    """Reorder a utilities launch's tiles (kept in their longest-first order per XCD) so that
    every tile of one cell runs on XCD ``cell mod 8``: slot s of the launch goes to XCD s mod 8
    and takes the next tile of that XCD's queue (cells numbered densely within the launch).  A cell's beta block (L x n, ~0.4 MB at
    n = 513) is then read by its 12 months x row tiles through ONE L2 instead of all eight -
    in launch order every XCD saw every cell, and the L2s kept re-fetching beta from HBM.
    Queues that run dry hand their slots to the longest remaining one (the tail loses the
    affinity, not the order)."""
    _, x = np.unique(np.asarray(cell, np.int64), return_inverse=True)   # dense cell ranks
    x = x.reshape(-1) % NXCD
    queues = [list(np.nonzero(x == k)[0]) for k in range(NXCD)]
    heads = [0] * NXCD
    order = np.empty(len(x), dtype=np.int64)
    for s in range(len(x)):
        k = s % NXCD
        if heads[k] >= len(queues[k]):
            k = int(np.argmax([len(q) - h for q, h in zip(queues, heads)]))
        order[s] = queues[k][heads[k]]
        heads[k] += 1
    return jobs_t[order], rt[order]


def quad_launch(plan: dict, d_desc: torch.Tensor, d_tj: torch.Tensor, D: torch.Tensor,
                R: torch.Tensor, beta: torch.Tensor, obj: torch.Tensor) -> None:
    if plan["nj"] == 0:
        return
    P = D.shape[-1]
    L, Pb = beta.shape[1], beta.shape[2]
    nt = plan["ntiles"]
    partial = torch.empty((plan["nslots"], L), dtype=torch.float64, device=D.device)
    # one-month tiles take the direct-A form (csrc/quadform.hip quadform_direct_kernel: D
    # fragments straight to registers two steps ahead, only beta through LDS) unless
    # PFML_QUAD_DIRECT=0
    mm = plan["mm"]
    if mm == 1 and os.environ.get("PFML_QUAD_DIRECT", "1") != "0":
        mm = 3
    nat.check(nat.hip_lib().pfml_quadform(D.data_ptr(), P, R.data_ptr(), beta.data_ptr(), Pb,
                                          d_desc.data_ptr(), plan["nj"], d_tj.data_ptr(), nt,
                                          mm, L,
                                          partial.data_ptr(), obj.data_ptr(),
                                          nat.stream_of(D)), "pfml_quadform")


def quadform_utilities(D: torch.Tensor, R: torch.Tensor, beta: torch.Tensor,
                       job_cell: np.ndarray, job_month: np.ndarray, job_n: np.ndarray
                       ) -> torch.Tensor:
    """obj[j, l] = R[m_j,:n]·beta[c_j,l,:n] - 1/2 beta[c_j,l,:n]' D[m_j,:n,:n] beta[c_j,l,:n]."""
    T, P, _ = D.shape
    nc, L, Pb = beta.shape
    nj = len(job_cell)
    obj = torch.empty((nj, L), dtype=D.dtype, device=D.device)
    if nj == 0:
        return obj
    if nat.is_device(D):
        plan = quad_plan(P, L, Pb, job_cell, job_month, job_n)
        d_desc, d_tj = upload([plan["desc"], plan["tile_job"]], D.device)
        quad_launch(plan, d_desc, d_tj, D.contiguous(), R.contiguous(), beta.contiguous(), obj)
        return obj
    for j in range(nj):
        n, m, c = int(job_n[j]), int(job_month[j]), int(job_cell[j])
        Bm = beta[c, :, :n]                       # [L, n]
        quad = ((Bm @ D[m, :n, :n]) * Bm).sum(1)
        obj[j] = Bm @ R[m, :n] - 0.5 * quad
    return obj
