"""Hyper-parameter grid kernels: window sums (K14), ridge solves (K15), utilities (K16).

Device paths run csrc/segsum.hip, csrc/ridge.hip and csrc/quadform.hip; CPU paths are the
fp64 oracle in the reference's own formulation (np.linalg.solve per lambda,
PFML_Search_Coef.py:131-133; r'b - 1/2 b'Db per month, PFML_hp_reals.py:94).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native as nat

CELL_DTYPE = np.dtype([("src", "<i8"), ("rsrc", "<i8"), ("work", "<i8"), ("out", "<i8"),
                       ("n", "<i4"), ("_pad", "<i4"), ("scale", "<f8")])
JOB_DTYPE = np.dtype([("d_off", "<i8"), ("r_off", "<i8"), ("b_off", "<i8"), ("n", "<i4"),
                      ("ptile0", "<i4")])


def segment_sums(X: torch.Tensor, starts, stops) -> torch.Tensor:
    """out[s] = X[starts[s]:stops[s]].sum(0) for X of shape [T, ...]."""
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
        st = torch.as_tensor(starts, device=X.device)
        sp = torch.as_tensor(stops, device=X.device)
        nat.check(nat.hip_lib().pfml_segsum(X.data_ptr(), E, st.data_ptr(), sp.data_ptr(), S,
                                            out.data_ptr(), nat.stream_of(X)), "pfml_segsum")
    else:
        for s in range(S):
            out[s] = X[starts[s]:stops[s]].sum(0)
    return out


def ridge_grid(SD: torch.Tensor, Sr: torch.Tensor, cell_src: np.ndarray, cell_n: np.ndarray,
               cell_scale: np.ndarray, lvec: torch.Tensor, repair: bool = True) -> torch.Tensor:
    """beta[c, l, :n_c] = solve(SD[src_c][:n,:n]*scale_c + l I, Sr[src_c][:n]*scale_c).

    SD: [S, P, P] running sums, Sr: [S, P]; returns [ncells, L, P] (zero beyond n_c).
    ``repair=False`` leaves the band path's non-SPD markers (NaN rows) for the caller to
    repair (``repair_nonspd``), so no device->host sync happens here.
    """
    S, P, _ = SD.shape
    L = int(lvec.numel())
    nc = len(cell_src)
    beta = torch.zeros((nc, L, P), dtype=SD.dtype, device=SD.device)
    if nc == 0:
        return beta
    if nat.is_device(SD):
        lib = nat.hip_lib()
        if lib.pfml_ridge_cell_desc_size() != CELL_DTYPE.itemsize:
            raise RuntimeError("CellDesc layout mismatch between python and libpfml_hip")
        desc = np.zeros(nc, dtype=CELL_DTYPE)
        wsz = np.array([lib.pfml_ridge_work_doubles(int(n), L) for n in cell_n], dtype=np.int64)
        woff = np.concatenate([[0], np.cumsum(wsz)[:-1]])
        desc["src"] = np.asarray(cell_src, np.int64) * P * P
        desc["rsrc"] = np.asarray(cell_src, np.int64) * P
        desc["work"] = woff
        desc["out"] = np.arange(nc, dtype=np.int64) * L * P
        desc["n"] = np.asarray(cell_n, np.int32)
        desc["scale"] = np.asarray(cell_scale, np.float64)
        # big cells first: they bound the kernel's makespan
        order = np.argsort(-desc["n"], kind="stable")
        desc = desc[order]
        d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(SD.device)
        work = torch.empty(int(wsz.sum()), dtype=torch.float64, device=SD.device)
        lv = lvec.to(device=SD.device, dtype=torch.float64).contiguous()
        SDc, Src = SD.contiguous(), Sr.contiguous()
        nat.check(lib.pfml_ridge_grid(SDc.data_ptr(), P, Src.data_ptr(), d_desc.data_ptr(), nc,
                                      int(np.max(cell_n)),
                                      lv.data_ptr(), L, work.data_ptr(), beta.data_ptr(), P,
                                      nat.stream_of(SD)), "pfml_ridge_grid")
        if repair:
            repair_nonspd(beta, SDc, Src, cell_src, cell_n, cell_scale, lv)
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
    """The band path marks a (cell, lambda) whose banded Cholesky met a non-positive pivot
    (Dbar + l I not numerically SPD) with NaN; re-solve exactly those systems with pivoted LU
    (np.linalg.solve semantics, PFML_Search_Coef.py:131-133).  One device->host flag read."""
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


def ridge_utilities(SD: torch.Tensor, Sr: torch.Tensor, cell_src, cell_n, cell_scale,
                    lvec: torch.Tensor, D: torch.Tensor, R: torch.Tensor, job_cell, job_month,
                    job_n) -> tuple[torch.Tensor, torch.Tensor]:
    """(beta, obj) = (ridge_grid(...), quadform_utilities(D, R, beta, jobs)).

    On a device the cells split into the largest-n group and the rest; each group's
    ridge -> utilities chain is issued on its own HIP stream, the big group first, so the
    small cells' whole chain runs on the CUs the big cells' one-workgroup-per-cell band
    reductions leave idle.  Non-SPD repairs (rare) are applied once at the end, and the
    utilities of repaired cells recomputed.
    """
    cell_src, cell_n = np.asarray(cell_src), np.asarray(cell_n)
    cell_scale = np.asarray(cell_scale)
    job_cell, job_month, job_n = (np.asarray(job_cell), np.asarray(job_month),
                                  np.asarray(job_n))
    if not nat.is_device(SD) or len(np.unique(cell_n)) < 2:
        beta = ridge_grid(SD, Sr, cell_src, cell_n, cell_scale, lvec)
        return beta, quadform_utilities(D, R, beta, job_cell, job_month, job_n)
    S, P, _ = SD.shape
    L = int(lvec.numel())
    nc = len(cell_src)
    beta = torch.zeros((nc, L, P), dtype=SD.dtype, device=SD.device)
    obj = torch.empty((len(job_cell), L), dtype=SD.dtype, device=SD.device)
    big = cell_n == cell_n.max()
    cur = torch.cuda.current_stream(SD.device)
    side = torch.cuda.Stream(device=SD.device)
    side.wait_stream(cur)
    parts = []
    for grp, stream in ((big, side), (~big, cur)):
        cells = np.nonzero(grp)[0]
        remap = np.full(nc, -1, dtype=np.int64)
        remap[cells] = np.arange(len(cells))
        jobs = np.nonzero(grp[job_cell])[0]
        with torch.cuda.stream(stream):
            b = ridge_grid(SD, Sr, cell_src[cells], cell_n[cells], cell_scale[cells], lvec,
                           repair=False)
            o = quadform_utilities(D, R, b, remap[job_cell[jobs]], job_month[jobs],
                                   job_n[jobs])
        parts.append((cells, jobs, b, o))
    cur.wait_stream(side)
    for t in (SD, Sr, D, R, lvec):
        t.record_stream(side)
    for cells, jobs, b, o in parts:
        ci = torch.as_tensor(cells, device=SD.device)
        beta.index_copy_(0, ci, b)
        obj.index_copy_(0, torch.as_tensor(jobs, device=SD.device), o)
    fixed = repair_nonspd(beta, SD, Sr, cell_src, cell_n, cell_scale,
                          lvec.to(device=SD.device, dtype=torch.float64))
    if len(fixed):
        jobs = np.nonzero(np.isin(job_cell, fixed))[0]
        obj[torch.as_tensor(jobs, device=SD.device)] = quadform_utilities(
            D, R, beta, job_cell[jobs], job_month[jobs], job_n[jobs])
    return beta, obj


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
        lib = nat.hip_lib()
        if lib.pfml_quadform_job_desc_size() != JOB_DTYPE.itemsize:
            raise RuntimeError("JobDesc layout mismatch between python and libpfml_hip")
        rows = lib.pfml_quadform_rows_per_tile()
        ntile = (np.asarray(job_n) + rows - 1) // rows
        pt0 = np.concatenate([[0], np.cumsum(ntile)[:-1]]).astype(np.int32)
        desc = np.zeros(nj, dtype=JOB_DTYPE)
        desc["d_off"] = np.asarray(job_month, np.int64) * P * P
        desc["r_off"] = np.asarray(job_month, np.int64) * P
        desc["b_off"] = np.asarray(job_cell, np.int64) * L * Pb
        desc["n"] = np.asarray(job_n, np.int32)
        desc["ptile0"] = pt0
        tile_job = np.repeat(np.arange(nj, dtype=np.int32), ntile)
        dev = D.device
        d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
        d_tj = torch.from_numpy(tile_job).to(dev)
        partial = torch.empty((len(tile_job), L), dtype=torch.float64, device=dev)
        Dc, Rc, Bc = D.contiguous(), R.contiguous(), beta.contiguous()
        nat.check(lib.pfml_quadform(Dc.data_ptr(), P, Rc.data_ptr(), Bc.data_ptr(), Pb,
                                    d_desc.data_ptr(), nj, d_tj.data_ptr(), len(tile_job), L,
                                    partial.data_ptr(), obj.data_ptr(), nat.stream_of(D)),
                  "pfml_quadform")
        return obj
    for j in range(nj):
        n, m, c = int(job_n[j]), int(job_month[j]), int(job_cell[j])
        Bm = beta[c, :, :n]                       # [L, n]
        quad = ((Bm @ D[m, :n, :n]) * Bm).sum(1)
        obj[j] = Bm @ R[m, :n] - 0.5 * quad
    return obj
