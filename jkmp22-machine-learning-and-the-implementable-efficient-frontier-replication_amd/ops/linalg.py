"""Batched dense linear algebra for the per-month PFML step.

* ``spd_inverse``  - SPD inverse (csrc/spd_inverse.hip): recursive Schur-complement form over
                     64 x 64 register Gauss-Jordan leaves for n >= 160, blocked Gauss-Jordan
                     below; matrices whose pivots are not positive fall back to a pivoted LU
                     inverse (counted).
* ``sqrtm_spd``    - principal square root by the scaled product-form Denman-Beavers
                     iteration (inverses + GEMMs only).  Replaces scipy.linalg.sqrtm (Schur,
                     General_functions.py:956): the argument sigma_hat^2 - 4I is symmetric PSD.
* ``solve``        - general (non-symmetric) batched solve with partial pivoting, K7.
* ``m_func``       - trading-speed matrix m of Lemma 1 (General_functions.py:919-963), batched
                     over months with block-diagonal padding for ragged universes.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _native as nat
from .gemm import gemm, gemm_fused
from ..utils import work as _work
from ..utils.log import COUNTERS


def _eye_like(A: torch.Tensor) -> torch.Tensor:
    return torch.eye(A.shape[-1], dtype=A.dtype, device=A.device).expand_as(A)


def spd_inverse_into(A: torch.Tensor, out: torch.Tensor, status: torch.Tensor) -> torch.Tensor:
    """out = A^-1 for a device batch [B, n, n] of SPD matrices without modifying or copying A
    (the recursive form reads A and writes only ``out``); other forms copy A into out first.
    Non-positive pivots are flagged in ``status`` (no host sync)."""
    B, n, _ = A.shape
    if nat.is_device(A) and n >= _BLOCKED_MIN_N and A.is_contiguous() and out.is_contiguous():
        _spd_inverse_recursive(out, status, src=A)
        return out
    out.copy_(A)
    return spd_inverse(out, inplace=True, status=status)


def spd_inverse(A: torch.Tensor, inplace: bool = False,
                status: torch.Tensor | None = None) -> torch.Tensor:
    """Inverse of a batch [B, n, n] of SPD matrices.

    Device: the recursive Schur-complement form for n >= 160 (GEMMs over register-resident
    64 x 64 Gauss-Jordan leaves), blocked Gauss-Jordan below (csrc/spd_inverse.hip).  With
    ``status`` (a [B] int32 device
    tensor) non-positive pivots are only flagged there - no host sync - and the caller repairs
    the flagged matrices once, after a whole chain of inverses (m_func); without it a flagged
    matrix is re-inverted by a pivoted LU here (one sync)."""
    squeeze = A.dim() == 2
    X = A if inplace else A.clone()
    if squeeze:
        X = X.unsqueeze(0)
    if nat.is_device(X):
        X = X.contiguous() if not X.is_contiguous() else X
        B, n, _ = X.shape
        lib = nat.hip_lib()
        st = status if status is not None else torch.zeros(B, dtype=torch.int32, device=X.device)
        if n >= _BLOCKED_MIN_N:
            _spd_inverse_recursive(X, st)
        else:
            work = torch.empty(lib.pfml_spd_inverse_work_doubles(n, B), dtype=torch.float64,
                               device=X.device)
            nat.check(lib.pfml_spd_inverse(X.data_ptr(), n, n, n * n, B, work.data_ptr(),
                                           st.data_ptr(), nat.stream_of(X)),
                      "pfml_spd_inverse")
        if status is None:
            bad = torch.nonzero(st).flatten()
            if bad.numel():
                COUNTERS.add("linalg.spd_inverse_lu_fallback", int(bad.numel()))
                src = A.unsqueeze(0) if squeeze else A
                X[bad] = torch.linalg.inv(src[bad])
    else:
        X.copy_(torch.linalg.inv(X))
    return X.squeeze(0) if squeeze else X


_BLOCKED_MIN_N = 160


nat.register_hip("pfml_spd_leafinv_to", [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64,
                                         C.c_int64, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                         C.c_int, C.c_void_p])

nat.register_hip("pfml_spd_node_sym", [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int,
                                       C.c_int, C.c_int, C.c_void_p, C.c_void_p])

_REC_LEAF = 64
_REC_BUFS: dict = {}
# streams that run recursive inverses concurrently with others (the multi-stream S4 batches,
# models/pfml_inputs.py): their scratch buffers are their own; every other stream shares one
# set (so a graph capture reuses the eager run's buffers)
CONCURRENT_STREAMS: set = set()


def _buf_tag(X: torch.Tensor) -> int:
    h = nat.stream_of(X)
    return h if h in CONCURRENT_STREAMS else 0


def _rec_split(n: int) -> int:
    """Leading block of a recursive split: a multiple of the leaf size, about n / 2."""
    return _REC_LEAF * ((n + 2 * _REC_LEAF - 1) // (2 * _REC_LEAF))


def _spd_inverse_recursive(X: torch.Tensor, status: torch.Tensor,
                           src: torch.Tensor | None = None) -> None:
    """SPD inverse by recursive 2 x 2 Schur-complement blocks, into X (from ``src`` when given:
    the source is only read, so no copy of it is made; else in place):

        X11 = A11^-1 (recursive),  W = X11 A12,  S = A22 - A21 W,  X22 = S^-1 (recursive),
        X12 = -W X22,  X21 = -X22 W',  X11 -= X12 W'

    Every product is one fused-GEMM launch whose inner dimension is the block size
    (256 / 128 / 64 on the m_func shape) instead of the rank-64 updates of the Gauss-Jordan
    form, so the pass is MFMA-bound rather than a bandwidth-bound sweep over the whole matrix
    per 64 columns; the 64 x 64 leaves are the register-resident leaf kernel
    (csrc/spd_inverse.hip).  Schur complements of an SPD matrix are SPD, so no pivoting; a
    non-positive leaf pivot flags ``status`` like the other forms.  One W buffer per depth
    (the parent's W lives across the child's recursion)."""
    lib = nat.hip_lib()
    B, n, _ = X.shape
    st = nat.stream_of(X)
    ld, sX = X.stride(1), X.stride(0)

    def buf(depth, h, m):
        key = (X.device, B, depth, _buf_tag(X))
        w = _REC_BUFS.get(key)
        if w is None or w.numel() < B * h * m:
            w = torch.empty(B * h * m, dtype=torch.float64, device=X.device)
            _REC_BUFS[key] = w
        return w[:B * h * m].view(B, h, m)

    def rec(r0, nn, depth, A):
        if nn <= _REC_LEAF:
            _work.add("spd_leafinv_kernel", 2.0 * B * nn ** 3, 16.0 * B * nn * nn)
            nat.check(lib.pfml_spd_leafinv_to(A.data_ptr(), A.stride(1), A.stride(0),
                                              X.data_ptr(), ld, sX, B, r0, nn,
                                              status.data_ptr(), 0, st), "pfml_spd_leafinv_to")
            return
        h = _rec_split(nn)
        m = nn - h
        a, c, e = r0, r0 + h, r0 + nn
        rec(a, h, depth + 1, A)
        W = buf(depth, h, m)
        gemm_fused(X[:, a:c, a:c], A[:, a:c, c:e], W)                        # W = X11 A12
        if A is X:
            gemm_fused(X[:, c:e, a:c], W, X[:, c:e, c:e], alpha=-1.0, beta=1.0)  # S
        else:
            gemm_fused(A[:, c:e, a:c], W, X[:, c:e, c:e], alpha=-1.0,
                       addend=A[:, c:e, c:e], addend_cols=m)                  # S = A22 - A21 W
        rec(c, m, depth + 1, X)
        gemm_fused(W, X[:, c:e, c:e], X[:, a:c, c:e], alpha=-1.0)            # X12
        # X21 = -X22 W' as its own product, not X12^T: the two carry independent rounding,
        # and the Denman-Beavers iterate Y M^-1 (which sees both triangles) measured 20x
        # closer to eigh with the product (2e-10 -> < 1e-11 on tests/test_gpu_pipeline.py)
        gemm_fused(X[:, c:e, c:e], W, X[:, c:e, a:c], trans_b=True, alpha=-1.0)
        gemm_fused(X[:, a:c, c:e], W, X[:, a:c, a:c], trans_b=True, alpha=-1.0,
                   beta=1.0)                                                  # X11 -= X12 W'

    rec(0, n, 0, X if src is None else src)


# GEMM tile config of the symmetric form's products (csrc/gemm_f64.hip tile_cfg; 0: auto);
# PFML_SPD_SYM=0 takes the two-sided form for every m_func inverse, PFML_DB_SYM=0 /
# PFML_DB_SYMPROD=0 the two-sided inverse / product inside Denman-Beavers (A/B switches)
SYM_GEMM_CFG = int(os.environ.get("PFML_SYM_GEMM_CFG", "0"))
SYM_INVERSE = os.environ.get("PFML_SPD_SYM", "1") != "0"
DB_SYM = os.environ.get("PFML_DB_SYM", "1") != "0"
DB_SYMPROD = os.environ.get("PFML_DB_SYMPROD", "1") != "0"
# nodes of 65..128 rows in one launch (csrc/spd_inverse.hip spd_node_sym_kernel: both leaves and
# the four products in LDS, bitwise the GEMM + leaf launches it replaces); 0: those launches
SYM_NODE = os.environ.get("PFML_SPD_NODE", "1") != "0"


def spd_inverse_sym(X: torch.Tensor, status: torch.Tensor,
                    src: torch.Tensor | None = None) -> torch.Tensor:
    """In-place inverse of a device batch [B, n, n] of EXACTLY symmetric SPD matrices whose
    result is used as a symmetric matrix (m_tilde_0 and the fixed-point steps of m_func,
    General_functions.py:957-960): the recursive Schur form with every symmetric product
    computed on its lower block triangle only and mirrored -

        X11 = A11^-1,  W = X11 A12,  S = A22 - A21 W  (lower tiles),  X22 = S^-1,
        X12 = -W X22  (X21 = X12' written by the same launch),  X11 -= X12 W'  (lower tiles)

    about n^3 flops instead of the two-sided form's ~1.67 n^3, with exactly symmetric leaves
    and products, so the result is exactly symmetric.  Non-positive pivots flag ``status``.
    ``src`` (same shape, contiguous): the input, only read - the inverse goes to X without a
    copy of the input first (the input blocks along the recursion's left spine and the A12 /
    A21 / A22 blocks of its nodes are read from src; A22 enters the Schur GEMM as its addend,
    the same arithmetic as the in-place beta)."""
    B, n, _ = X.shape
    if src is not None and (src.shape != X.shape or not src.is_contiguous()):
        raise ValueError("spd_inverse_sym: src must be contiguous and shaped like X")
    if not nat.is_device(X) or n < _BLOCKED_MIN_N or not X.is_contiguous() or not SYM_INVERSE:
        if src is not None:
            X.copy_(src)
        return spd_inverse(X, inplace=True, status=status)
    lib = nat.hip_lib()
    st = nat.stream_of(X)
    ld, sX = X.stride(1), X.stride(0)
    cfg = SYM_GEMM_CFG

    def buf(depth, h, m):
        key = (X.device, B, depth, "sym", _buf_tag(X))
        w = _REC_BUFS.get(key)
        if w is None or w.numel() < B * h * m:
            w = torch.empty(B * h * m, dtype=torch.float64, device=X.device)
            _REC_BUFS[key] = w
        return w[:B * h * m].view(B, h, m)

    def rec(r0, nn, depth, A):
        # A: where this block's input lives (src along the left spine, else X itself)
        if nn <= _REC_LEAF:
            _work.add("spd_leafinv_kernel", 2.0 * B * nn ** 3, 16.0 * B * nn * nn)
            nat.check(lib.pfml_spd_leafinv_to(A.data_ptr(), ld, sX, X.data_ptr(), ld, sX, B, r0,
                                              nn, status.data_ptr(), 1, st),
                      "pfml_spd_leafinv_to")
            return
        if SYM_NODE and nn <= 2 * _REC_LEAF:
            m = nn - _REC_LEAF
            _work.add("spd_node_sym_kernel", B * (2.0 * _REC_LEAF ** 3 + 2.0 * m ** 3
                                                  + 3.0 * _REC_LEAF ** 2 * m
                                                  + 3.0 * _REC_LEAF * m * m),
                      8.0 * B * 2 * nn * nn)
            nat.check(lib.pfml_spd_node_sym(A.data_ptr(), X.data_ptr(), ld, sX, B, r0, nn,
                                            status.data_ptr(), st), "pfml_spd_node_sym")
            return
        h = _rec_split(nn)
        m = nn - h
        a, c, e = r0, r0 + h, r0 + nn
        rec(a, h, depth + 1, A)
        W = buf(depth, h, m)
        gemm_fused(X[:, a:c, a:c], A[:, a:c, c:e], W, tile_cfg=cfg)              # W = X11 A12
        if A is X:
            gemm_fused(X[:, c:e, a:c], W, X[:, c:e, c:e], alpha=-1.0, beta=1.0, sym=True,
                       tile_cfg=cfg)                                              # S
        else:
            gemm_fused(A[:, c:e, a:c], W, X[:, c:e, c:e], alpha=-1.0, addend=A[:, c:e, c:e],
                       sym=True, tile_cfg=cfg)                                    # S
        rec(c, m, depth + 1, X)
        gemm_fused(W, X[:, c:e, c:e], X[:, a:c, c:e], alpha=-1.0, mirror_out=X[:, c:e, a:c],
                   tile_cfg=cfg)                                                  # X12, X21
        gemm_fused(X[:, a:c, c:e], W, X[:, a:c, a:c], trans_b=True, alpha=-1.0, beta=1.0,
                   sym=True, tile_cfg=cfg)                                        # X11 -= X12 W'

    rec(0, n, 0, X if src is None else src)
    return X


def _lu_max_n() -> int:
    return int(nat.hip_lib().pfml_lu_solve_max_n())


LU_PANEL_COLS = 128            # scratch columns of the two-level solve (pfml_lu_panel_cols)
nat.register_hip("pfml_lu_solve2", [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int,
                                    C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                    C.c_void_p])


def _lu_ledger(M, n, m, ldm, sM, a0, b0, z0, batch) -> None:
    """Work-ledger entries of one pfml_lu_solve / pfml_lu_solve2 call (csrc/lu_solve.hip loop
    structure): the rank-nb Gauss-Jordan updates, the panel pivoting and, in the two-level
    form, the K = 128 panel-transform GEMMs under the dgemm kernel name they launch."""
    nb = 32 if n <= 512 else 16
    upd, piv = f"lu_update_kernel<{nb}>", f"lu_pivot_kernel<{nb}, {512 if n <= 512 else 1024}>"
    if z0 is None:
        for k0 in range(0, n, nb):
            b = min(nb, n - k0)
            nlive = n - (k0 + b) + m
            _work.add(upd, 2.0 * batch * n * nlive * b, 8.0 * batch * 2 * n * nlive)
            _work.add(piv, 2.0 * batch * (n - k0) * b * b, 8.0 * batch * (n - k0) * b)
        return
    kbw = LU_PANEL_COLS
    for K0 in range(0, n, kbw):
        kb = min(kbw, n - K0)
        aend = K0 + kb
        for k0 in range(K0, aend, nb):
            b = min(nb, aend - k0)
            nlive = aend - (k0 + b) + (k0 - K0) + b      # (only Z's populated columns)
            _work.add(upd, 2.0 * batch * n * nlive * b, 8.0 * batch * 2 * n * nlive)
            _work.add(piv, 2.0 * batch * (n - k0) * b * b, 8.0 * batch * (n - k0) * b)
        nAr = n - aend
        nrest = nAr + m
        if nrest <= 0:
            continue
        for off, wdt in ((0, nAr), (nAr, m)):
            if wdt <= 0:
                continue
            # pfml_dgemm(0, 0, rows, wdt, kb): A = Z rows (ld ldm), B = RK + off (ld nrest)
            vec = (kb % 2 == 0 and wdt % 2 == 0 and ldm % 2 == 0 and nrest % 2 == 0
                   and sM % 2 == 0 and (kb * nrest) % 2 == 0 and z0 % 2 == 0 and off % 2 == 0
                   and M.data_ptr() % 16 == 0)
            for rows in (K0, kb, n - aend):
                if rows <= 0:
                    continue
                big = rows >= 1024 and wdt >= 1024
                t = "128, 128" if big else "64, 64"
                _work.add(f"dgemm_kernel<false, false, {t}, {2 if vec else 1}, false, 16, 2>",
                         2.0 * batch * rows * wdt * kb, 8.0 * batch * (rows * kb + 2 * rows * wdt))


def solve_augmented(M: torch.Tensor, n: int, m: int, a0: int, b0: int,
                    status: torch.Tensor | None = None, z0: int | None = None) -> torch.Tensor:
    """In-place solve of augmented systems: rows of M [B, n, W] hold A at columns a0..a0+n and
    B at b0..b0+m; on return the B columns hold X = A^-1 B (returned as a view).

    Device: csrc/lu_solve.hip (blocked Gauss-Jordan with partial pivoting; 32-wide blocks up to
    n = 512, 16-wide up to 3072 - the pivot panel in LDS up to 1024 rows, in the registers of a
    1024-thread workgroup beyond, which covers the 3000-stock stress); larger systems take the
    library (rocSOLVER) LU through torch.  ``z0``: M holds LU_PANEL_COLS free scratch columns
    there, and the two-level form runs (128-wide panels whose transform reaches the other
    columns through K = 128 GEMMs).  With ``status`` (a [B] int32
    device tensor) singular systems are only flagged there (no host sync; the caller checks
    once), otherwise they are counted here."""
    if nat.is_device(M) and n <= _lu_max_n():
        if not M.is_contiguous():
            raise ValueError("solve_augmented: contiguous storage required")
        Bt, nn, W = M.shape
        lib = nat.hip_lib()
        work = torch.empty(lib.pfml_lu_solve_work_doubles(n, m, Bt), dtype=torch.float64,
                           device=M.device)
        st = status if status is not None else torch.zeros(Bt, dtype=torch.int32,
                                                           device=M.device)
        if _work.on():
            _lu_ledger(M, n, m, W, nn * W, a0, b0, z0, Bt)
        if z0 is not None:
            if z0 + LU_PANEL_COLS > W:
                raise ValueError("solve_augmented: z0 needs LU_PANEL_COLS scratch columns")
            nat.check(lib.pfml_lu_solve2(M.data_ptr(), n, m, W, nn * W, a0, b0, z0, Bt,
                                         work.data_ptr(), st.data_ptr(), nat.stream_of(M)),
                      "pfml_lu_solve2")
        else:
            nat.check(lib.pfml_lu_solve(M.data_ptr(), n, m, W, nn * W, a0, b0, Bt,
                                        work.data_ptr(), st.data_ptr(), nat.stream_of(M)),
                      "pfml_lu_solve")
        if status is None:
            nbad = int(st.sum().item())
            if nbad:
                COUNTERS.add("linalg.singular_solve", nbad)
    else:
        X, info = torch.linalg.solve_ex(M[:, :, a0:a0 + n], M[:, :, b0:b0 + m])
        bad = info != 0
        if status is not None:
            status |= bad.to(status.dtype)
        elif bool(bad.any()):
            COUNTERS.add("linalg.singular_solve", int(bad.sum()))
        M[:, :, b0:b0 + m] = X
    return M[:, :, b0:b0 + m]


def solve(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """Batched general solve A X = B with partial pivoting (np.linalg.solve semantics)."""
    squeeze = A.dim() == 2
    A3 = A.unsqueeze(0) if squeeze else A
    B3 = B.unsqueeze(0) if squeeze else B
    vec = B3.dim() == 2
    if vec:
        B3 = B3.unsqueeze(-1)
    n, m = A3.shape[-1], B3.shape[-1]
    M = torch.cat([B3, A3], dim=-1).contiguous()
    X = solve_augmented(M, n, m, a0=m, b0=0).clone()
    if vec:
        X = X.squeeze(-1)
    return X.squeeze(0) if squeeze else X


def sqrtm_spd(S: torch.Tensor, max_iter: int = 40, tol: float = 1e-13) -> torch.Tensor:
    """Principal square root of a batch of symmetric PSD matrices (reference/oracle form).

    Scaled product-form Denman-Beavers (Higham, Functions of Matrices, (6.29)):
        M_{k+1} = (I + (mu^2 M_k + mu^-2 M_k^-1)/2)/2,  Y_{k+1} = mu Y_k (I + mu^-2 M_k^-1)/2
    with M_0 = Y_0 = S and norm scaling mu^4 = ||M^-1||_F / ||M||_F; stops when every
    ||M_k - I||_F < tol * sqrt(n).  The production path is ``_db_sqrt`` (fixed iteration count,
    no host synchronisation).
    """
    M = S.clone()
    Y = S.clone()
    n = S.shape[-1]
    I = _eye_like(S)
    for it in range(max_iter):
        Mi = spd_inverse(M)
        nm = torch.linalg.matrix_norm(M).clamp_min(1e-300)
        ni = torch.linalg.matrix_norm(Mi).clamp_min(1e-300)
        mu = (ni / nm) ** 0.25
        mu2 = (mu * mu).view(-1, 1, 1)
        if it > 6:
            mu2 = torch.ones_like(mu2)        # near convergence: unscaled (quadratic) steps
            mu = torch.ones_like(mu)
        Mi_s = Mi / mu2
        Y = gemm(Y, I + Mi_s, alpha=0.5) * mu.view(-1, 1, 1)
        M = 0.5 * (I + 0.5 * (mu2 * M + Mi_s))
        M = 0.5 * (M + M.transpose(-1, -2))   # keep exact symmetry for the SPD inverse
        err = torch.linalg.matrix_norm(M - I).max().item()
        if err < tol * n ** 0.5:
            break
    else:
        COUNTERS.add("linalg.sqrtm_not_converged")
    return 0.5 * (Y + Y.transpose(-1, -2))


# ---------------------------------------------------------------------------------------
# Fused symmetric passes (csrc/s4.hip) and the device m_func
# ---------------------------------------------------------------------------------------
MF_X, MF_FIX, MF_DB, MF_SHAT, MF_M0 = 0, 1, 2, 3, 4


class _MfArgs(C.Structure):
    _fields_ = [("mode", C.c_int), ("B", C.c_int), ("N", C.c_int), ("ld", C.c_int64),
                ("sX", C.c_int64), ("X", C.c_void_p), ("Y", C.c_void_p), ("out", C.c_void_p),
                ("svec", C.c_void_p), ("cvec", C.c_void_p), ("a", C.c_void_p),
                ("mask", C.c_void_p), ("sv", C.c_int64), ("d", C.c_double), ("flat", C.c_int)]


nat.register_hip("pfml_mfunc_sym", [C.POINTER(_MfArgs), C.c_void_p])
nat.register_hip("pfml_mf_args_size", [])
nat.register_hip("pfml_db_mu_rows", [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int64,
                                     C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p])
nat.register_hip("pfml_db_mu", [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_int64,
                                C.c_int, C.c_void_p, C.c_void_p, C.c_void_p])
nat.register_hip("pfml_db_mu_work_doubles2", [C.c_int, C.c_int], C.c_int64)


def _sym(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * (x + x.transpose(-1, -2))


def mf_sym(mode: int, X: torch.Tensor, Y: torch.Tensor | None, out: torch.Tensor, *,
           svec: torch.Tensor | None = None, cvec: torch.Tensor | None = None,
           a: torch.Tensor | None = None, mask: torch.Tensor | None = None,
           d: float = 0.0, flat: bool = False) -> torch.Tensor:
    """One fused symmetric pass over a [B, N, N] batch (csrc/s4.hip, header for the modes);
    the CPU branch is the torch oracle of the same formulas.  ``flat``: X and Y are known to
    be exactly symmetric (sym() is then the identity, bit for bit): the mirror reads are
    skipped."""
    B, N, _ = X.shape
    if nat.is_device(X):
        for t in (X, Y, out):
            if t is not None and (not t.is_contiguous() or t.shape != X.shape):
                raise ValueError("mf_sym: contiguous [B, N, N] operands required")
        sv = 0 if a is None else a.stride(0)
        if mask is not None and a is not None and mask.stride(0) != sv:
            raise ValueError("mf_sym: a and mask need the same batch stride")
        if mask is not None and a is None:
            sv = mask.stride(0)
        # (the flat form streams each operand once; the tiled form reads the mirror tile too,
        # mostly from L2: the same minimum bytes)
        _work.add("mfunc_flat_kernel" if flat else "mfunc_sym_kernel", 6.0 * B * N * N,
                  8.0 * B * N * N * (2 + (Y is not None)))
        args = _MfArgs(mode, B, N, N, N * N, X.data_ptr(), nat.ptr(Y), out.data_ptr(),
                       nat.ptr(svec), nat.ptr(cvec), nat.ptr(a), nat.ptr(mask), sv, float(d),
                       int(flat))
        nat.check(nat.hip_lib().pfml_mfunc_sym(C.byref(args), nat.stream_of(X)), "pfml_mfunc_sym")
        return out
    xs = _sym(X)
    ys = _sym(Y) if Y is not None else None
    eye = torch.eye(N, dtype=X.dtype, device=X.device)
    if mode == MF_X:
        r = svec.view(B, 1, 1) * a.unsqueeze(-1) * a.unsqueeze(-2) * xs
    elif mode == MF_FIX:
        ic2 = (1.0 / (cvec * cvec)).view(B, 1, 1)
        mm = mask.unsqueeze(-1) * mask.unsqueeze(-2)
        r = xs * (svec.view(B, 1, 1) * a.unsqueeze(-1) * a.unsqueeze(-2) - ys * ic2) - ys * mm
        r = r + torch.diag_embed(1.0 + torch.diagonal(mm, dim1=-2, dim2=-1)
                                 + torch.diagonal(xs, dim1=-2, dim2=-1) * ic2.view(B, 1))
    elif mode == MF_DB:
        mu2 = (svec * svec).view(B, 1, 1)
        r = 0.25 * (mu2 * xs + ys / mu2) + 0.5 * eye
    elif mode == MF_M0:
        r = 0.5 * ((xs + d * eye) - ys)
    else:
        r = xs + (ys if ys is not None else 0.0) + d * eye
    out.copy_(r)
    return out


nat.register_hip("pfml_horner_init", [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64,
                                      C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                                      C.c_int64, C.c_int, C.c_int, C.c_void_p])
nat.register_hip("pfml_block_add", [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64,
                                    C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p,
                                    C.c_int64, C.c_int, C.c_int, C.c_int, C.c_void_p])


def horner_init(T: torch.Tensor, mt: torch.Tensor, k10: torch.Tensor, ks12: torch.Tensor,
                a: torch.Tensor) -> torch.Tensor:
    """T_11's identity and Q blocks of the (24) Horner chain (models/pfml_inputs.py) in one pass
    (csrc/s4.hip horner_init): T [B, N, 2N] (a column block of the Horner buffer) gets
    [diag(k10) | ((mt * ks12_j) * a_i) * k10_i].  k10 / ks12 [B, N] share a batch stride."""
    B, N, _ = mt.shape
    if nat.is_device(T):
        if (T.stride(-1) != 1 or mt.stride(-1) != 1 or k10.stride(-1) != 1 or
                ks12.stride(-1) != 1 or a.stride(-1) != 1 or k10.stride(0) != ks12.stride(0) or
                T.shape[-1] < 2 * N):
            raise ValueError("horner_init: unsupported layout")
        _work.add("horner_init_kernel", 3.0 * B * N * N, 24.0 * B * N * N)
        nat.check(nat.hip_lib().pfml_horner_init(
            T.data_ptr(), T.stride(1), T.stride(0), mt.data_ptr(), mt.stride(1), mt.stride(0),
            k10.data_ptr(), ks12.data_ptr(), k10.stride(0), a.data_ptr(), a.stride(0), N, B,
            nat.stream_of(T)), "pfml_horner_init")
        return T
    T[:, :, :N] = torch.diag_embed(k10)
    torch.mul(mt * ks12.unsqueeze(-2), a.unsqueeze(-1), out=T[:, :, N:2 * N])
    T[:, :, N:2 * N].mul_(k10.unsqueeze(-1))
    return T


def block_add(out: torch.Tensor, X: torch.Tensor, Y: torch.Tensor,
              y_row_scale: torch.Tensor | None = None) -> torch.Tensor:
    """out = X + Y on [B, M, N] blocks of strided rows (unit inner stride), one pass;
    ``y_row_scale`` [B, M] (unit inner stride): out = X + diag(s) Y, one fma per element."""
    B, M, N = out.shape
    if nat.is_device(out):
        for t in (out, X, Y):
            if t.stride(-1) != 1 or tuple(t.shape) != (B, M, N):
                raise ValueError("block_add: unsupported layout")
        if y_row_scale is not None and (y_row_scale.stride(-1) != 1 or
                                        tuple(y_row_scale.shape) != (B, M)):
            raise ValueError("block_add: y_row_scale must be [B, M] with unit inner stride")
        nat.check(nat.hip_lib().pfml_block_add(
            out.data_ptr(), out.stride(1), out.stride(0), X.data_ptr(), X.stride(1), X.stride(0),
            Y.data_ptr(), Y.stride(1), Y.stride(0), nat.ptr(y_row_scale),
            0 if y_row_scale is None else y_row_scale.stride(0), M, N, B, nat.stream_of(out)),
            "pfml_block_add")
        return out
    if y_row_scale is not None:
        return torch.addcmul(X, y_row_scale.unsqueeze(-1), Y, out=out)
    return torch.add(X, Y, out=out)


def _db_mu_rows(M: torch.Tensor, Minv: torch.Tensor, unscaled: bool, mu: torch.Tensor,
                rs: torch.Tensor, es: torch.Tensor) -> None:
    """``_db_mu`` plus the Y update's row scales rs = 0.5 / mu, es = 0.5 mu as [B, N] rows (one
    device kernel with the mu reduction: csrc/s4.hip db_mu_rows_kernel)."""
    B, N, _ = M.shape
    if nat.is_device(M):
        lib = nat.hip_lib()
        if not unscaled:
            _work.add("db_norm_partial_kernel", 4.0 * B * N * N, 16.0 * B * N * N)
        wbuf = torch.empty(lib.pfml_db_mu_work_doubles2(B, N), dtype=torch.float64,
                           device=M.device)
        nat.check(lib.pfml_db_mu_rows(M.data_ptr(), Minv.data_ptr(), B, N, N, N * N,
                                      int(unscaled), mu.data_ptr(), wbuf.data_ptr(),
                                      rs.data_ptr(), es.data_ptr(), nat.stream_of(M)),
                  "pfml_db_mu_rows")
        return
    _db_mu(M, Minv, unscaled, mu)
    rs.copy_((0.5 / mu).view(B, 1).expand(B, N))
    es.copy_((0.5 * mu).view(B, 1).expand(B, N))


def _db_mu(M: torch.Tensor, Minv: torch.Tensor, unscaled: bool, out: torch.Tensor) -> None:
    B, N, _ = M.shape
    if nat.is_device(M):
        lib = nat.hip_lib()
        if not unscaled:                         # (unscaled steps launch no norm pass)
            _work.add("db_norm_partial_kernel", 4.0 * B * N * N, 16.0 * B * N * N)
        wbuf = torch.empty(lib.pfml_db_mu_work_doubles2(B, N), dtype=torch.float64,
                           device=M.device)
        nat.check(lib.pfml_db_mu(M.data_ptr(), Minv.data_ptr(), B, N, N, N * N, int(unscaled),
                                 out.data_ptr(), wbuf.data_ptr(), nat.stream_of(M)), "pfml_db_mu")
        return
    if unscaled:
        out.fill_(1.0)
    else:
        # (ratio)^(1/4) as two IEEE square roots: torch's CPU pow is vectorised over the batch
        # and not correctly rounded, so x ** 0.25 differed in the last bit between a month in
        # a vector lane and one in the scalar tail - a month's m_tilde then depended on the
        # months batched with it (the S4 summands must be bitwise the same however the months
        # are sharded)
        nm = torch.linalg.matrix_norm(M).clamp_min(1e-300)
        out.copy_((torch.linalg.matrix_norm(Minv) / nm).sqrt().sqrt())


def _db_sqrt(S: torch.Tensor, iters: int, scaled_iters: int, status: torch.Tensor | None,
             ws: list, exact_sym: bool = False, ns_tail: bool | None = None) -> torch.Tensor:
    """sqrtm(S) by ``iters`` scaled product-form Denman-Beavers steps with NO host sync:
    norm scaling mu (computed on the device) for the first ``scaled_iters`` steps, then
    quadratically convergent unscaled steps.  ws: 4 [B, N, N] work buffers; ``exact_sym``: S is
    exactly symmetric (bit for bit).

    ``ns_tail`` (default ``DB_NS_TAIL``): the last (unscaled) step takes M^-1 as its
    first-order Neumann form 2I - M - a Newton-Schulz step Y <- (3Y - Y M) / 2, one product
    and NO inverse, whose error against the exact step is O(|M - I|^2).  By then M is the
    identity to 1e-16 .. 1e-10 on production spectra (cond(x^2 + 4x) up to 7e14,
    profiles/r06_db_tail.json: the exact step changed nothing but the cost of an inverse); a
    matrix with any |M_ij - delta_ij| > DB_TAIL_TOL (1e-7: tail error < 1e-14) sets ``status``
    and is recomputed by the convergence-checked reference form, like a failed pivot."""
    B, N, _ = S.shape
    M, Y, Mi, Yn = ws
    mu = torch.empty(B, dtype=S.dtype, device=S.device)
    rs = torch.empty((B, N), dtype=S.dtype, device=S.device)     # Y update row scales
    es = torch.empty((B, N), dtype=S.dtype, device=S.device)
    if ns_tail is None:
        ns_tail = DB_NS_TAIL
    ns_tail = ns_tail and iters > scaled_iters
    # the first (exact) step reads S itself as both M and Y - no copies; its M update goes to
    # the unused buffer ``spare`` (S is only read)
    spare = None
    if iters >= 2:
        spare, M, Y = M, S, S
    else:
        M.copy_(S)
        Y.copy_(S)
    # S, M, M^-1 and Y are symmetric (M, Y are polynomials in S; in exact arithmetic Y and M^-1
    # commute, so Y M^-1 is symmetric too).  sym_inv: M^-1 by the one-triangle inverse;
    # sym_prod: Y M^-1 on its lower tiles, mirrored.  With both (and S exactly symmetric, as
    # m_tilde builds it; after the first M update otherwise) every iterate is EXACTLY symmetric
    # and the M update skips its mirror reads (flat).  profiles/r05_mfunc_db_accuracy.json: m
    # vs the reference form 4e-14 (two-sided products: 3e-14); S4 -12 ms.
    dev_sym = nat.is_device(M) and N >= _BLOCKED_MIN_N
    sym_inv, sym_prod = DB_SYM and dev_sym, DB_SYMPROD and dev_sym
    for it in range(iters):
        if ns_tail and it == iters - 1:
            # Newton-Schulz tail: Y' = 1.5 Y - 0.5 Y M (Y M symmetric, as Y M^-1 is)
            _db_check(M, DB_TAIL_TOL, status)
            rs.fill_(-0.5)
            es.fill_(1.5)
            gemm_fused(Y, M, Yn, row_scale=rs, addend=Y, addend_row_scale=es, sym=sym_prod)
            Y, Yn = Yn, Y
            break
        if sym_inv:
            spd_inverse_sym(Mi, status, src=M)
        else:
            spd_inverse_into(M, Mi, status)
        # Y' = (mu/2) Y + (1/(2 mu)) Y M^-1 ;  M' = I/2 + (mu^2 M + mu^-2 M^-1)/4
        _db_mu_rows(M, Mi, it >= scaled_iters, mu, rs, es)
        gemm_fused(Y, Mi, Yn, row_scale=rs, addend=Y, addend_row_scale=es, sym=sym_prod)
        Y, Yn = Yn, Y
        if it == 0 and spare is not None:
            # (Yn is S now: the new M goes to the spare buffer; S retires, ws[1] is free)
            mf_sym(MF_DB, M, Mi, spare, svec=mu, flat=sym_inv and exact_sym)
            M, Yn = spare, ws[1]
            continue
        mf_sym(MF_DB, M, Mi, Yn, svec=mu, flat=sym_inv and (exact_sym or it > 0))
        # (Yn was free: the new M went into it)
        M, Yn = Yn, M
    ws[0], ws[1], ws[2], ws[3] = M, Y, Mi, Yn
    return Y


# Denman-Beavers steps: 7 exact steps leave M within 1e-10 of I on production spectra
# (cond(x^2 + 4x) ~ 1e5 - 7e14, TC on and off; profiles/r06_db_tail.json), the 8th is the
# Newton-Schulz tail (above; PFML_DB_NS_TAIL=0: an exact 8th step).  The former 9th exact step
# moved nothing (|M - I| ~ 1e-20 .. 1e-32 at its start).  Norm scaling in the first 6.
DB_ITERS = 8
DB_SCALED_ITERS = 6
DB_NS_TAIL = os.environ.get("PFML_DB_NS_TAIL", "1") != "0"
DB_TAIL_TOL = 1e-7
# m_tilde_0 by the reference's (sigma_hat - root) / 2 (one pass) instead of the inverse form
M0_CANCEL = os.environ.get("PFML_M0_CANCEL", "1") != "0"
nat.register_hip("pfml_db_check", [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_int64,
                                   C.c_double, C.c_void_p, C.c_void_p])


def _db_check(M: torch.Tensor, tol: float, status: torch.Tensor | None) -> None:
    """Flag (status = 1) the matrices of M [B, N, N] with any |M_ij - delta_ij| > tol or a
    non-finite entry (csrc/s4.hip db_check_kernel); the CPU path has no status to set."""
    if status is None or not nat.is_device(M):
        return
    B, N, _ = M.shape
    nat.check(nat.hip_lib().pfml_db_check(M.data_ptr(), B, N, M.stride(1), M.stride(0), tol,
                                          status.data_ptr(), nat.stream_of(M)), "pfml_db_check")


def m_tilde(sigma: torch.Tensor, lam: torch.Tensor, w: torch.Tensor, rf: torch.Tensor,
            mu: float, gamma: float, iterations: int = 10, mask: torch.Tensor | None = None,
            db_iters: int = DB_ITERS, status: torch.Tensor | None = None,
            sigma_exact_sym: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """m_tilde of Lemma 1 and a = lambda^-1/2, so that m = diag(a) m_tilde diag(1/a)
    (General_functions.py:941-963).  All on the device with no host synchronisation except one
    status check at the end (matrices whose SPD inverse met a non-positive pivot anywhere in
    the chain are recomputed by the reference-form ``m_func_reference``).  ``status`` (a
    zeroed [B] int32 device tensor): the flags are left there and NOT checked - no host sync
    at all (graph capture); the caller repairs the flagged months itself."""
    B, N, _ = sigma.shape
    dt, dev = sigma.dtype, sigma.device
    if mask is None:
        mask = torch.ones((B, N), dtype=dt, device=dev)
    mask = mask.contiguous()
    a = lam.rsqrt().contiguous()
    s = (gamma / w).to(dt).contiguous()
    c = (1.0 + rf + mu).to(dt).contiguous()
    sigma = sigma.contiguous()
    deferred = status is not None
    if not deferred:
        status = torch.zeros(B, dtype=torch.int32, device=dev) if nat.is_device(sigma) else None
    x = torch.empty_like(sigma)
    # sigma_exact_sym: the caller built Sigma exactly symmetric (S4's X F X' in the GEMM's
    # symmetric mode), and the one-triangle inverses keep mt exactly symmetric: the x and
    # fixed-point passes then skip their mirror reads (same bits)
    flat = sigma_exact_sym and nat.is_device(sigma) and SYM_INVERSE and N >= _BLOCKED_MIN_N
    mf_sym(MF_X, sigma, None, x, svec=s, a=a, flat=flat)        # x = s L^-1/2 S L^-1/2
    S = torch.empty_like(sigma)
    four = torch.full((B, N), 4.0, dtype=dt, device=dev)
    # sigma_hat^2 - 4I = x^2 + 4x (x exactly symmetric: the GEMM's symmetric mode, half the
    # tiles, an exactly symmetric S - and Denman-Beavers' M stays so)
    gemm_fused(x, x, S, addend=x, addend_row_scale=four, sym=True)
    ws = [torch.empty_like(sigma) for _ in range(4)]
    root = _db_sqrt(S, db_iters, DB_SCALED_ITERS, status, ws, exact_sym=True)
    # m_tilde_0 = (sigma_hat - root) / 2, the reference's form (General_functions.py:955), in
    # one pass.  Its cancellation costs accuracy only along the large eigenvalues l of x (error
    # ~ eps l there), and the first fixed-point step maps an error along such a direction to
    # ~eps / l (the step's derivative there is ~(x + 2I)^-2): m after the ten steps equals the
    # cancellation-free 2 (sigma_hat + root)^-1 start's to rounding, also with eig(x) up to 6e7
    # (TC off) and down to 3e-7 (profiles/r06_m0_form.json) - one SPD inverse per month fewer.
    mt = ws[2]
    # (x is exactly symmetric - MF_X symmetrises - and so is root when its last product was
    # the one-triangle one)
    flat_root = DB_SYMPROD and db_iters > 0 and nat.is_device(x) and N >= _BLOCKED_MIN_N
    if M0_CANCEL:
        mf_sym(MF_M0, x, root, mt, d=2.0, flat=flat_root)
    else:                      # 2 (sigma_hat + root)^-1 (PFML_M0_CANCEL=0: the former form)
        mf_sym(MF_SHAT, x, root, mt, d=2.0, flat=flat_root)
        # (an exactly symmetric argument, used symmetrically: the one-triangle form)
        spd_inverse_sym(mt, status)
        mt.mul_(2.0)
    # (the 10 inverses below are of exactly symmetric arguments and only used symmetrically:
    # the one-triangle form)
    Aq = ws[3]
    for _ in range(iterations):
        mf_sym(MF_FIX, sigma, mt, Aq, svec=s, cvec=c, a=a, mask=mask, flat=flat)
        spd_inverse_sym(Aq, status)
        mt, Aq = Aq, mt
    if status is not None and not deferred:
        bad = torch.nonzero(status).flatten()
        if bad.numel():
            COUNTERS.add("linalg.m_func_repaired", int(bad.numel()))
            ref = m_func_reference(sigma[bad], lam[bad], w[bad], rf[bad], mu, gamma, iterations,
                                   mask=mask[bad])
            mt[bad] = ref * a[bad].unsqueeze(-2) / a[bad].unsqueeze(-1)
    return mt, a


def m_func(sigma: torch.Tensor, lam: torch.Tensor, w: torch.Tensor, rf: torch.Tensor,
           mu: float, gamma: float, iterations: int = 10,
           mask: torch.Tensor | None = None) -> torch.Tensor:
    """Trading-speed matrix m (Lemma 1; General_functions.py:919-963), batched.

    sigma: [B, N, N] Barra covariance (padded entries: identity block), lam: [B, N] Kyle's
    lambda, w: [B] wealth, rf: [B]; mask: [B, N] 1 for real stocks (0 = padding: the rank-one
    mu_bar mu_bar' term of sigma_gr is restricted to real stocks so the pad block decouples).
    """
    mt, a = m_tilde(sigma, lam, w, rf, mu, gamma, iterations, mask)
    return mt * a.unsqueeze(-1) / a.unsqueeze(-2)


def m_func_reference(sigma: torch.Tensor, lam: torch.Tensor, w: torch.Tensor, rf: torch.Tensor,
                     mu: float, gamma: float, iterations: int = 10,
                     mask: torch.Tensor | None = None) -> torch.Tensor:
    """Reference-form m_func in plain torch ops (LU inverses, convergence-checked square root):
    the repair path of ``m_tilde`` and the CPU oracle.

    m_tilde_0 = 1/2 (sigma_hat - sqrtm(sigma_hat^2 - 4I)) is evaluated in the algebraically
    identical, cancellation-free form 2 (sigma_hat + sqrtm(sigma_hat^2 - 4I))^-1.
    """
    B, N, _ = sigma.shape
    dt = sigma.dtype
    if mask is None:
        mask = torch.ones((B, N), dtype=dt, device=sigma.device)
    c = (1.0 + rf + mu).view(B, 1, 1)
    I = _eye_like(sigma)
    sig = _sym(sigma)
    sig_gr = mask.unsqueeze(-1) * mask.unsqueeze(-2) + sig / (c * c)
    a = lam.rsqrt()                                              # Lambda^-1/2 diagonal
    x = (gamma / w).view(B, 1, 1) * sig * a.unsqueeze(-1) * a.unsqueeze(-2)
    ydiag = 1.0 + torch.diagonal(sig_gr, dim1=-2, dim2=-1)
    sig_hat = x + 2.0 * I
    S = _sym(x @ x + 4.0 * x)
    root = sqrtm_spd(S.cpu()).to(sigma.device) if nat.is_device(S) else sqrtm_spd(S)
    mt = 2.0 * torch.linalg.inv(_sym(sig_hat + root))
    base = x + torch.diag_embed(ydiag)
    for _ in range(iterations):
        mt = torch.linalg.inv(_sym(base - _sym(mt) * sig_gr))
    return mt * a.unsqueeze(-1) / a.unsqueeze(-2)
