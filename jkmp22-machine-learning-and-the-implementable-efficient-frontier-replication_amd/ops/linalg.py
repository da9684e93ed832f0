"""Batched dense linear algebra for the per-month PFML step.

* ``spd_inverse``  - blocked Gauss-Jordan SPD inverse (csrc/spd_inverse.hip); matrices whose
                     pivots are not positive fall back to a pivoted LU inverse (counted).
* ``sqrtm_spd``    - principal square root by the scaled product-form Denman-Beavers
                     iteration (inverses + GEMMs only).  Replaces scipy.linalg.sqrtm (Schur,
                     General_functions.py:956): the argument sigma_hat^2 - 4I is symmetric PSD.
* ``solve``        - general (non-symmetric) batched solve with partial pivoting, K7.
* ``m_func``       - trading-speed matrix m of Lemma 1 (General_functions.py:919-963), batched
                     over months with block-diagonal padding for ragged universes.
"""
from __future__ import annotations

import torch

from . import _native as nat
from .gemm import gemm
from ..utils.log import COUNTERS


def _eye_like(A: torch.Tensor) -> torch.Tensor:
    return torch.eye(A.shape[-1], dtype=A.dtype, device=A.device).expand_as(A)


def spd_inverse(A: torch.Tensor, inplace: bool = False) -> torch.Tensor:
    """Inverse of a batch [B, n, n] of SPD matrices."""
    squeeze = A.dim() == 2
    X = A if inplace else A.clone()
    if squeeze:
        X = X.unsqueeze(0)
    if nat.is_device(X):
        X = X.contiguous() if not X.is_contiguous() else X
        B, n, _ = X.shape
        lib = nat.hip_lib()
        status = torch.zeros(B, dtype=torch.int32, device=X.device)
        if n >= _BLOCKED_MIN_N:
            _spd_inverse_blocked(X, status)
        else:
            work = torch.empty(lib.pfml_spd_inverse_work_doubles(n, B), dtype=torch.float64,
                               device=X.device)
            nat.check(lib.pfml_spd_inverse(X.data_ptr(), n, n, n * n, B, work.data_ptr(),
                                           status.data_ptr(), nat.stream_of(X)),
                      "pfml_spd_inverse")
        bad = torch.nonzero(status).flatten()
        if bad.numel():
            COUNTERS.add("linalg.spd_inverse_lu_fallback", int(bad.numel()))
            src = A.unsqueeze(0) if squeeze else A
            import os
            if os.environ.get("PFML_DEBUG_INV"):
                for b in bad.tolist()[:4]:
                    M = src[b]
                    print(f"[spd_inverse] bad b={b} n={M.shape[-1]} nan={int(torch.isnan(M).sum())} "
                          f"absmax={float(M.abs().max()):.3e} "
                          f"diagmin={float(torch.diagonal(M).min()):.3e} "
                          f"asym={float((M - M.T).abs().max()):.3e}", flush=True)
            X[bad] = torch.linalg.inv(src[bad])
    else:
        X.copy_(torch.linalg.inv(X))
    return X.squeeze(0) if squeeze else X


_BLOCKED_MIN_N = 160


def _spd_inverse_blocked(X: torch.Tensor, status: torch.Tensor) -> None:
    """In-place SPD inverse with 128-wide Gauss-Jordan blocks: pivot block inverted in LDS
    (csrc/spd_inverse.hip: pfml_spd_blockinv); row panel, rank-128 trailing update and column
    panel as batched fp64 MFMA GEMMs."""
    lib = nat.hip_lib()
    B, n, _ = X.shape
    NB = lib.pfml_spd_block_size()
    dev = X.device
    P = torch.empty((B, NB, NB), dtype=torch.float64, device=dev)
    Cbuf = torch.empty((B, n, NB), dtype=torch.float64, device=dev)
    Rbuf = torch.empty((B, NB, n), dtype=torch.float64, device=dev)
    st = nat.stream_of(X)
    for k0 in range(0, n, NB):
        nb = min(NB, n - k0)
        nat.check(lib.pfml_spd_blockinv(X.data_ptr(), n, n * n, B, k0, nb, P.data_ptr(),
                                        status.data_ptr(), st), "pfml_spd_blockinv")
        Pk = P[:, :nb, :nb]
        R = Rbuf[:, :nb, :]
        gemm(Pk, X[:, k0:k0 + nb, :], out=R)                     # R = P A_k.
        C = Cbuf[:, :, :nb]
        C.copy_(X[:, :, k0:k0 + nb])                             # old column panel
        gemm(C, R, alpha=-1.0, beta=1.0, out=X)                  # A -= C R   (rank nb)
        X[:, k0:k0 + nb, :] = R                                  # block rows
        gemm(C, Pk, alpha=-1.0, out=X[:, :, k0:k0 + nb])         # block columns: -C P
        X[:, k0:k0 + nb, k0:k0 + nb] = Pk


def _lu_max_n() -> int:
    return int(nat.hip_lib().pfml_lu_solve_max_n())


def solve_augmented(M: torch.Tensor, n: int, m: int, a0: int, b0: int) -> torch.Tensor:
    """In-place solve of augmented systems: rows of M [B, n, W] hold A at columns a0..a0+n and
    B at b0..b0+m; on return the B columns hold X = A^-1 B (returned as a view).

    Device: csrc/lu_solve.hip (blocked LU with partial pivoting, the pivot panel in LDS) up to
    n = pfml_lu_solve_max_n() (1024); larger systems (the 3000-stock stress) take the library
    (rocSOLVER) LU through torch."""
    if nat.is_device(M) and n <= _lu_max_n():
        if not M.is_contiguous():
            raise ValueError("solve_augmented: contiguous storage required")
        Bt, nn, W = M.shape
        lib = nat.hip_lib()
        work = torch.empty(lib.pfml_lu_solve_work_doubles(n, m, Bt), dtype=torch.float64,
                           device=M.device)
        status = torch.zeros(Bt, dtype=torch.int32, device=M.device)
        nat.check(lib.pfml_lu_solve(M.data_ptr(), n, m, W, nn * W, a0, b0, Bt, work.data_ptr(),
                                    status.data_ptr(), nat.stream_of(M)), "pfml_lu_solve")
        nbad = int(status.sum().item())
        if nbad:
            COUNTERS.add("linalg.singular_solve", nbad)
    else:
        X, info = torch.linalg.solve_ex(M[:, :, a0:a0 + n], M[:, :, b0:b0 + m])
        if bool((info != 0).any()):
            COUNTERS.add("linalg.singular_solve", int((info != 0).sum()))
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
    """Principal square root of a batch of symmetric PSD matrices.

    Scaled product-form Denman-Beavers (Higham, Functions of Matrices, (6.29)):
        M_{k+1} = (I + (mu^2 M_k + mu^-2 M_k^-1)/2)/2,  Y_{k+1} = mu Y_k (I + mu^-2 M_k^-1)/2
    with M_0 = Y_0 = S and norm scaling mu^4 = ||M^-1||_F / ||M||_F; stops when every
    ||M_k - I||_F < tol * sqrt(n).
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


def m_func(sigma: torch.Tensor, lam: torch.Tensor, w: torch.Tensor, rf: torch.Tensor,
           mu: float, gamma: float, iterations: int = 10,
           mask: torch.Tensor | None = None) -> torch.Tensor:
    """Trading-speed matrix m (Lemma 1; General_functions.py:919-963), batched.

    sigma: [B, N, N] Barra covariance (padded entries: identity block), lam: [B, N] Kyle's
    lambda, w: [B] wealth, rf: [B]; mask: [B, N] 1 for real stocks (0 = padding: the rank-one
    mu_bar mu_bar' term of sigma_gr is restricted to real stocks so the pad block decouples).

    m_tilde_0 = 1/2 (sigma_hat - sqrtm(sigma_hat^2 - 4I)) is evaluated in the algebraically
    identical, cancellation-free form 2 (sigma_hat + sqrtm(sigma_hat^2 - 4I))^-1.
    """
    B, N, _ = sigma.shape
    dt = sigma.dtype
    if mask is None:
        mask = torch.ones((B, N), dtype=dt, device=sigma.device)
    c = (1.0 + rf + mu).view(B, 1, 1)
    I = _eye_like(sigma)
    sig_gr = mask.unsqueeze(-1) * mask.unsqueeze(-2) + sigma / (c * c)
    a = lam.rsqrt()                                              # Lambda^-1/2 diagonal
    x = (gamma / w).view(B, 1, 1) * sigma * a.unsqueeze(-1) * a.unsqueeze(-2)
    x = 0.5 * (x + x.transpose(-1, -2))
    ydiag = 1.0 + torch.diagonal(sig_gr, dim1=-2, dim2=-1)
    sig_hat = x + 2.0 * I
    S = gemm(sig_hat, sig_hat) - 4.0 * I
    S = 0.5 * (S + S.transpose(-1, -2))
    root = sqrtm_spd(S)
    mt = 2.0 * spd_inverse(sig_hat + root)
    base = x + torch.diag_embed(ydiag)
    for _ in range(iterations):
        Aq = base - mt * sig_gr
        Aq = 0.5 * (Aq + Aq.transpose(-1, -2))
        mt = spd_inverse(Aq)
    return mt * a.unsqueeze(-1) / a.unsqueeze(-2)
