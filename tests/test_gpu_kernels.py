"""Numerics of the hand-written gfx950 kernels vs the fp64 torch CPU oracle of the same op."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rand(*shape, seed=0, dev="cpu"):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g, dtype=torch.float64).to(dev)


def test_native_library_loaded(gpu):
    from pfml.ops import _native as nat
    lib = nat.hip_lib()
    assert lib is not None
    assert any(p.endswith("libpfml_hip.so") for p in nat.loaded_libraries())


def test_mfma_f64_layout(gpu):
    """A = I, asymmetric B: catches a swapped C/D row map (cdna_hip_programming.md §3)."""
    from pfml.ops.gemm import gemm
    A = torch.eye(16, dtype=torch.float64)
    B = torch.arange(16 * 16, dtype=torch.float64).view(16, 16)
    out = gemm(A.to(gpu), B.to(gpu), backend="own").cpu()
    assert torch.equal(out, B)
    out2 = gemm(B.to(gpu), A.to(gpu), backend="own").cpu()
    assert torch.equal(out2, B)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("shape", [(1, 37, 53, 29), (3, 64, 64, 64), (2, 130, 257, 100),
                                   (1, 513, 513, 513)])
def test_dgemm_matches_torch(gpu, ta, tb, shape):
    from pfml.ops.gemm import gemm
    b, M, N, K = shape
    A = _rand(b, K, M, seed=1) if ta else _rand(b, M, K, seed=1)
    B = _rand(b, N, K, seed=2) if tb else _rand(b, K, N, seed=2)
    rs, cs = _rand(b, M, seed=3), _rand(b, N, seed=4)
    C0 = _rand(b, M, N, seed=5)
    ref = gemm(A, B, trans_a=ta, trans_b=tb, alpha=0.7, beta=0.3, out=C0.clone(),
               row_scale=rs, col_scale=cs)
    Cd = C0.to(gpu)
    out = gemm(A.to(gpu), B.to(gpu), trans_a=ta, trans_b=tb, alpha=0.7, beta=0.3, out=Cd,
               row_scale=rs.to(gpu), col_scale=cs.to(gpu)).cpu()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-13, err
    # plain products: hand-written kernel and the rocBLAS route agree with the oracle
    ref2 = gemm(A, B, trans_a=ta, trans_b=tb, alpha=0.7, beta=0.3, out=C0.clone())
    for be in ("own", "blas"):
        out2 = gemm(A.to(gpu), B.to(gpu), trans_a=ta, trans_b=tb, alpha=0.7, beta=0.3,
                    out=C0.to(gpu), backend=be).cpu()
        err2 = (out2 - ref2).abs().max().item() / ref2.abs().max().item()
        assert err2 < 1e-13, (be, err2)


def test_gemm_epi_struct_matches():
    import ctypes
    from pfml.ops import _native as nat
    from pfml.ops.gemm import _Epi
    assert nat.hip_lib().pfml_gemm_epi_size() == ctypes.sizeof(_Epi)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
@pytest.mark.parametrize("shape", [(2, 37, 53, 29), (3, 130, 258, 100), (2, 96, 224, 96),
                                   (3, 130, 258, 99)])
def test_gemm_fused_matches_torch(gpu, ta, tb, cfg, shape):
    """Every fusion of csrc/gemm_f64.hip (k-scale prologue, row/col scale, beta, addend block,
    diagonal vector) vs the fp64 torch oracle, for odd (scalar staging) and even (16-byte
    staging) dimensions and every tile config."""
    from pfml.ops.gemm import gemm_fused
    b, M, N, K = shape
    A = _rand(b, K, M, seed=1) if ta else _rand(b, M, K, seed=1)
    B = _rand(b, N, K, seed=2) if tb else _rand(b, K, N, seed=2)
    kw = dict(trans_a=ta, trans_b=tb, alpha=0.7, beta=0.3, row_scale=_rand(b, M, seed=3),
              col_scale=_rand(N, seed=4), k_scale=_rand(b, K, seed=6),
              addend=_rand(b, M, N // 2, seed=8), addend_cols=N // 2, diag_col0=N // 3,
              diag_vec=_rand(b, M, seed=9), addend_row_scale=_rand(b, M, seed=11))
    C0 = _rand(b, M, N, seed=5)
    ref = gemm_fused(A, B, C0.clone(), **kw)
    kd = {k: (v.to(gpu) if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    out = gemm_fused(A.to(gpu), B.to(gpu), C0.to(gpu), tile_cfg=cfg, **kd).cpu()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-13, err
    # Horner form: identity block via a constant diagonal, broadcast A (batch stride 0)
    E = _rand(b, M, 8, seed=10)
    ref = gemm_fused(A[:1], B, C0.clone(), trans_a=ta, trans_b=tb, addend=E, addend_cols=8,
                     diag_col0=8, diag_value=1.0)
    out = gemm_fused(A[:1].to(gpu), B.to(gpu), C0.to(gpu), trans_a=ta, trans_b=tb,
                     addend=E.to(gpu), addend_cols=8, diag_col0=8, diag_value=1.0,
                     tile_cfg=cfg).cpu()
    assert (out - ref).abs().max().item() / ref.abs().max().item() < 1e-13


def test_gemm_tile_forms_bitwise(gpu):
    """The 64 x 64 and 128 x 64 LDS-DMA tiles (tile_cfg 7 / 8) give BITWISE the same result
    for the S4 GEMM forms - the Horner step (row scale, gathered standardised addend, identity
    diagonal, output row scale), the k-scaled T_0 step, X' omega (trans_a) and a plain product:
    every element sees the same k steps in the same order.  The auto choice may therefore take
    the 64 x 64 form for launches too small to fill the chip (batch-dependent) without the bits
    depending on the batch size or the rank count."""
    from pfml.ops.gemm import gemm_fused
    b, M, K, GP, R = 3, 250, 250, 130, 400
    mt = _rand(b, M, K, seed=1).to(gpu)
    T = _rand(b, K, GP + M, seed=2).to(gpu)
    a = _rand(b, M, seed=3).to(gpu)
    feats = _rand(R, GP, seed=4).to(gpu)
    rows = torch.randint(0, R, (b, M), generator=torch.Generator().manual_seed(5)).to(gpu)
    shift, scale = _rand(b, GP, seed=6).to(gpu), _rand(b, GP, seed=7).to(gpu)
    ivol, ks = _rand(b, M, seed=8).to(gpu), _rand(b, K, seed=9).to(gpu)
    outs = {}
    for cfg in (7, 8):
        o1 = torch.empty(b, M, GP + M, dtype=torch.float64, device=gpu)
        gemm_fused(mt, T, o1, row_scale=a, addend=feats, addend_cols=GP, addend_rows=rows,
                   addend_col_shift=shift, addend_col_scale=scale, addend_row_scale=ivol,
                   diag_col0=GP, diag_value=1.0, out_row_scale=ks, tile_cfg=cfg)
        o2 = torch.empty_like(o1)
        gemm_fused(mt, T, o2, row_scale=a, k_scale=ks, addend=o1[:, :, :GP], addend_cols=GP,
                   diag_col0=GP, diag_value=1.0, tile_cfg=cfg)
        o3 = torch.empty(b, K, GP, dtype=torch.float64, device=gpu)
        gemm_fused(mt, T[:, :M, :GP].contiguous(), o3, trans_a=True, tile_cfg=cfg)
        o4 = torch.empty(b, M, GP + M, dtype=torch.float64, device=gpu)
        gemm_fused(mt, T, o4, tile_cfg=cfg)
        outs[cfg] = (o1, o2, o3, o4)
    for x, y in zip(outs[7], outs[8]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("sym", [False, True])
def test_gemm_store_clip(gpu, sym):
    """Store clip (S4's denom written in place): the product of the even-padded operands, only
    the leading Ms x Ns block read for beta and stored into a [B, Ms, Ns] buffer - equal to the
    padded product's block (bitwise: same kernel, same arithmetic) and to the fp64 oracle."""
    from pfml.ops.gemm import gemm_fused
    b, K, P = 3, 130, 513
    Pp = P + 1
    A, B = _rand(b, K, Pp, seed=1).to(gpu), _rand(b, K, Pp, seed=2).to(gpu)
    if sym:
        B = A
    ks = _rand(b, K, seed=3).to(gpu)
    C0 = _rand(b, Pp, Pp, seed=4).to(gpu)
    C0 = 0.5 * (C0 + C0.transpose(1, 2))
    full = C0.clone()
    gemm_fused(A, B, full, trans_a=True, k_scale=ks, beta=1.0, alpha=0.7, sym=sym)
    dd = C0[:, :P, :P].contiguous()
    gemm_fused(A, B, dd, trans_a=True, k_scale=ks, beta=1.0, alpha=0.7, sym=sym, clip=True)
    assert torch.equal(dd, full[:, :P, :P])
    ref = gemm_fused(A.cpu(), B.cpu(), C0.cpu()[:, :P, :P].contiguous(), trans_a=True,
                     k_scale=ks.cpu(), beta=1.0, alpha=0.7, sym=sym, clip=True)
    assert ((dd.cpu() - ref).abs().max() / ref.abs().max()).item() < 1e-13


def test_gemm_output_above_2gb_row_split(gpu):
    """A C batch entry of 2 GB or more (the epilogue's buffer stores use 32-bit offsets) is
    split into row chunks on the host: row scale, diagonal vector, addend and the
    transposed second output are offset per chunk; vs the torch product on the device."""
    from pfml.ops.gemm import gemm_fused
    M, N, K = 16640, 16400, 8          # C: 2.18 GB
    g = torch.Generator(device=gpu).manual_seed(3)
    A = torch.randn(1, M, K, generator=g, dtype=torch.float64, device=gpu)
    B = torch.randn(1, K, N, generator=g, dtype=torch.float64, device=gpu)
    rs = torch.randn(1, M, generator=g, dtype=torch.float64, device=gpu)
    dv = torch.randn(1, M, generator=g, dtype=torch.float64, device=gpu)
    E = torch.randn(1, M, 8, generator=g, dtype=torch.float64, device=gpu)
    C = torch.empty(1, M, N, dtype=torch.float64, device=gpu)
    gemm_fused(A, B, C, row_scale=rs, addend=E, addend_cols=8, diag_col0=5, diag_vec=dv)
    ref = torch.bmm(A, B) * rs[..., None]
    ref[..., :8] += E
    i = torch.arange(min(M, N - 5), device=gpu)
    ref[0, i, i + 5] += dv[0, i]
    err = ((C - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-13, err
    del C, ref
    torch.cuda.empty_cache()
    # transposed second output (X21 = X12') across the split
    M2, N2 = 17000, 2048
    A2 = torch.randn(1, M2, K, generator=g, dtype=torch.float64, device=gpu)
    B2 = torch.randn(1, K, 16000, generator=g, dtype=torch.float64, device=gpu)
    C2 = torch.empty(1, M2, 16000, dtype=torch.float64, device=gpu)
    Ct = torch.empty(1, 16000, M2, dtype=torch.float64, device=gpu)
    # Ct is itself >= 2 GB: not splittable -> the launch must fail loudly, not write garbage
    with pytest.raises(RuntimeError):
        gemm_fused(A2, B2, C2, mirror_out=Ct)
    del C2, Ct
    torch.cuda.empty_cache()
    C3 = torch.empty(1, M2, 16000, dtype=torch.float64, device=gpu)
    Ct3 = torch.empty(1, N2, M2, dtype=torch.float64, device=gpu)
    B3 = B2[..., :N2].contiguous()
    C3v = C3[..., :N2]
    # a strided output view of 2.2 GB extent (ldc = 16000) with a 0.28 GB transposed copy
    gemm_fused(A2, B3, C3v, mirror_out=Ct3)
    ref3 = torch.bmm(A2, B3)
    assert ((C3v - ref3).abs().max() / ref3.abs().max()).item() < 1e-13
    assert torch.equal(Ct3, C3v.transpose(1, 2))


@pytest.mark.parametrize("cfg", [3, 6, 8])
def test_gemm_gathered_addend(gpu, cfg):
    """The gathered addend of the Horner steps (standardised signals formed in the epilogue):
    out = os_i (rs * (A B) + es_i * (F[rows_i] - shift) * scale on the first e_cols columns
    + the diagonal), vs the torch oracle, with rows repeated and out of order and a strided
    output row scale."""
    from pfml.ops.gemm import gemm_fused
    b, M, N, K, E = 3, 130, 202, 96, 150
    A, B = _rand(b, M, K, seed=1), _rand(b, K, N, seed=2)
    F = _rand(500, 160, seed=3)
    rows = torch.randint(0, 500, (b, 13, M), generator=torch.Generator().manual_seed(4))
    kw = dict(row_scale=_rand(b, M, seed=5), addend=F, addend_cols=E, addend_rows=rows[:, 7],
              addend_col_shift=_rand(b, 2, E, seed=6)[:, 0],
              addend_col_scale=_rand(b, 2, E, seed=6)[:, 1],
              addend_row_scale=_rand(b, 4, M, seed=7)[:, 2], diag_col0=E, diag_value=1.0,
              out_row_scale=_rand(b, 3, M, seed=8)[:, 1])    # (the next step's k-scale)
    ref = gemm_fused(A, B, torch.empty(b, M, N, dtype=torch.float64), **kw)
    kd = {k: (v.to(gpu) if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    out = gemm_fused(A.to(gpu), B.to(gpu), torch.empty(b, M, N, dtype=torch.float64, device=gpu),
                     tile_cfg=cfg, **kd).cpu()
    assert (out - ref).abs().max().item() / ref.abs().max().item() < 1e-13


@pytest.mark.parametrize("cfg", [1, 3, 6, 7, 9, 11])
@pytest.mark.parametrize("shape", [(3, 234, 256), (2, 130, 100), (2, 37, 29)])
def test_gemm_sym_and_mirror(gpu, cfg, shape):
    """Symmetric mode (only the output tiles on / below the diagonal, lower triangle mirrored:
    an exactly symmetric result) and the transposed second output of csrc/gemm_f64.hip vs
    the torch oracle of the same definition, for every square tile config."""
    from pfml.ops.gemm import gemm_fused
    b, n, K = shape
    A, B = _rand(b, n, K, seed=1), _rand(b, K, n, seed=2)
    C0 = _rand(b, n, n, seed=3)
    C0 = C0 + C0.transpose(1, 2)
    ref = gemm_fused(A, B, C0.clone(), alpha=-1.0, beta=1.0, sym=True)
    out = gemm_fused(A.to(gpu), B.to(gpu), C0.to(gpu), alpha=-1.0, beta=1.0, sym=True,
                     tile_cfg=cfg).cpu()
    assert torch.equal(out, out.transpose(1, 2))                     # exactly symmetric
    assert (out - ref).abs().max().item() / ref.abs().max().item() < 1e-13
    Bt = _rand(b, n, K, seed=4)
    ref = gemm_fused(A, Bt, C0.clone(), trans_b=True, alpha=-1.0, beta=1.0, sym=True)
    out = gemm_fused(A.to(gpu), Bt.to(gpu), C0.to(gpu), trans_b=True, alpha=-1.0, beta=1.0,
                     sym=True, tile_cfg=cfg).cpu()
    assert torch.equal(out, out.transpose(1, 2))
    assert (out - ref).abs().max().item() / ref.abs().max().item() < 1e-13
    # rectangular product with its transpose written by the same launch
    B2 = _rand(b, K, n + 6, seed=5)
    X = torch.empty(b, n, n + 6, dtype=torch.float64, device=gpu)
    Xt = torch.full((b, n + 6, n), float("nan"), dtype=torch.float64, device=gpu)
    gemm_fused(A.to(gpu), B2.to(gpu), X, alpha=-1.0, mirror_out=Xt, tile_cfg=cfg)
    ref = -(A @ B2)
    assert (X.cpu() - ref).abs().max().item() / ref.abs().max().item() < 1e-13
    assert torch.equal(Xt.cpu(), X.cpu().transpose(1, 2))


@pytest.mark.parametrize("n", [490, 257, 200])
def test_spd_inverse_sym(gpu, n):
    """Symmetric recursive SPD inverse (one-triangle Schur products, mirrored): exactly
    symmetric, and as close to the LU inverse as the two-sided form on a moderately
    conditioned batch."""
    from pfml.ops.linalg import spd_inverse, spd_inverse_sym
    g = torch.Generator().manual_seed(n)
    X = torch.randn(4, n + 40, n, generator=g, dtype=torch.float64)
    A = X.transpose(1, 2) @ X / n + 1e-3 * torch.eye(n, dtype=torch.float64)
    A = 0.5 * (A + A.transpose(1, 2))
    ref = torch.linalg.inv(A)
    st = torch.zeros(4, dtype=torch.int32, device=gpu)
    out = spd_inverse_sym(A.to(gpu).contiguous(), st).cpu()
    assert int(st.sum()) == 0
    assert torch.equal(out, out.transpose(1, 2))
    e_sym = ((out - ref).norm(dim=(1, 2)) / ref.norm(dim=(1, 2))).max().item()
    two = spd_inverse(A.to(gpu)).cpu()
    e_two = ((two - ref).norm(dim=(1, 2)) / ref.norm(dim=(1, 2))).max().item()
    assert e_sym < 1e-11 and e_sym < 4 * e_two + 1e-14, (e_sym, e_two)


@pytest.mark.parametrize("n", [490, 257, 200])
def test_spd_node_sym_bitwise(gpu, n):
    """The one-launch 65..128-row node (csrc/spd_inverse.hip spd_node_sym_kernel) is bitwise the
    GEMM + leaf launch sequence it replaces (490: nodes of 128 and 106 rows; 257: a 65-row node,
    m = 1; 200: 128 and 72), including the non-positive-pivot flags."""
    import pfml.ops.linalg as la
    g = torch.Generator().manual_seed(n + 1)
    X = torch.randn(6, n + 40, n, generator=g, dtype=torch.float64)
    A = X.transpose(1, 2) @ X / n + 1e-3 * torch.eye(n, dtype=torch.float64)
    A = 0.5 * (A + A.transpose(1, 2))
    A[5, n - 3, n - 3] = -50.0                     # not SPD: a pivot of the last node fails
    outs, sts = [], []
    for node in (True, False):
        la.SYM_NODE = node
        try:
            st = torch.zeros(6, dtype=torch.int32, device=gpu)
            outs.append(la.spd_inverse_sym(A.to(gpu).contiguous(), st).cpu())
            sts.append(st.cpu())
        finally:
            la.SYM_NODE = True
    assert torch.equal(sts[0], sts[1]) and sts[0].tolist() == [0, 0, 0, 0, 0, 1]
    assert torch.equal(outs[0][:5], outs[1][:5])
    ref = torch.linalg.inv(A[:5])
    assert ((outs[0][:5] - ref).norm(dim=(1, 2)) / ref.norm(dim=(1, 2))).max() < 1e-11


@pytest.mark.parametrize("n", [490, 257, 200])
def test_spd_inverse_sym_out_of_place_bitwise(gpu, n):
    """spd_inverse_sym(X, st, src=A) (input only read, no copy) is bitwise the in-place
    inverse of a copy of A, flags included, and leaves A untouched."""
    from pfml.ops.linalg import spd_inverse_sym
    g = torch.Generator().manual_seed(n + 7)
    X = torch.randn(5, n + 40, n, generator=g, dtype=torch.float64)
    A = X.transpose(1, 2) @ X / n + 1e-3 * torch.eye(n, dtype=torch.float64)
    A = 0.5 * (A + A.transpose(1, 2))
    A[4, 3, 3] = -20.0                             # not SPD: the first leaf's pivot fails
    Ad = A.to(gpu).contiguous()
    keep = Ad.clone()
    st1 = torch.zeros(5, dtype=torch.int32, device=gpu)
    st2 = torch.zeros(5, dtype=torch.int32, device=gpu)
    inplace = spd_inverse_sym(Ad.clone(), st1)
    out = spd_inverse_sym(torch.empty_like(Ad), st2, src=Ad)
    assert torch.equal(Ad, keep)
    assert torch.equal(st1, st2) and st1.tolist() == [0, 0, 0, 0, 1]
    assert torch.equal(out[:4], inplace[:4])


def test_segment_sums(gpu):
    from pfml.ops.ridge import segment_sums
    X = _rand(40, 7, 9, seed=7)
    st, sp = [0, 5, 5, 20], [5, 5, 20, 40]
    ref = segment_sums(X, st, sp)
    out = segment_sums(X.to(gpu), st, sp).cpu()
    assert torch.allclose(out, ref, rtol=1e-14, atol=1e-13)
    Y = _rand(11, 6, seed=8)   # even row length -> vector path
    assert torch.allclose(segment_sums(Y.to(gpu), [0, 3], [3, 11]).cpu(),
                          segment_sums(Y, [0, 3], [3, 11]), rtol=1e-14, atol=1e-13)


def _spd_stack(S, P, n_obs=40, seed=0):
    X = _rand(S, n_obs, P, seed=seed)
    return X.transpose(1, 2) @ X


@pytest.mark.parametrize("P,ns", [(9, [9, 5, 3]), (65, [65, 33, 17]), (129, [129, 65])])
def test_ridge_grid_matches_solve(gpu, P, ns):
    from pfml.ops.ridge import ridge_grid
    S = 3
    SD = _spd_stack(S, P, n_obs=max(2 * P, 40), seed=11)
    Sr = _rand(S, P, seed=12)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64)
    src = np.array([s for s in range(S) for _ in ns])
    nn = np.array([n for _ in range(S) for n in ns])
    sc = np.array([1.0 / (10 + s) for s in src])
    ref = ridge_grid(SD, Sr, src, nn, sc, lv)
    out = ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu)).cpu()
    rel = ((out - ref).norm(dim=-1) / ref.norm(dim=-1).clamp_min(1e-300)).max().item()
    assert rel < 1e-9, rel


def test_ridge_grid_production_size(gpu):
    from pfml.ops.ridge import ridge_grid
    P = 513
    SD = _spd_stack(1, P, n_obs=1200, seed=21)
    Sr = _rand(1, P, seed=22)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64)
    src, nn, sc = np.array([0, 0]), np.array([513, 257]), np.array([1e-3, 1e-3])
    ref = ridge_grid(SD, Sr, src, nn, sc, lv)
    out = ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu)).cpu()
    rel = ((out - ref).norm(dim=-1) / ref.norm(dim=-1)).max().item()
    assert rel < 1e-10, rel


def test_ridge_grid_production_rank_deficient(gpu):
    """Production size (n = 513, 257) with a RANK-DEFICIENT, indefinite window sum (400
    observations, rank 401 < 513): every lambda > 0 matches the fp64 pivoted LU (torch.linalg.solve) to 1e-10;
    at lambda = 0 the system is singular, the banded Cholesky fails and the device repairs it
    by the pivoted banded LU (PFML_Search_Coef.py:131-133 semantics).  A singular system has
    no unique solution to compare, so the lambda = 0 betas are held to np.linalg.solve's own
    guarantee instead: backward stability, |(Dbar) b - rbar| <= 1e-12 (|Dbar| |b| + |rbar|),
    with rbar in the range of Dbar (a consistent system)."""
    from pfml.ops import ridge as rg
    P = 513
    X = _rand(1, 400, P, seed=23)
    SD = X.transpose(1, 2) @ X / 400
    # one null direction turned negative: Dbar' = Dbar - 0.7 v v' stays singular (112 zero
    # eigenvalues) and is indefinite, so the banded Cholesky MUST fail at lambda = 0 (and
    # for lambda < 0.7) and every such system goes through the device repair
    e, V = torch.linalg.eigh(SD[0])
    SD[0] = SD[0] - 0.7 * torch.outer(V[:, 0], V[:, 0])
    SD[0] = 0.5 * (SD[0] + SD[0].T)
    w = _rand(1, P, seed=24)
    Sr = (SD @ w.unsqueeze(-1)).squeeze(-1)            # consistent at lambda = 0
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64)
    src, nn, sc = np.array([0, 0]), np.array([513, 257]), np.array([1.0, 1.0])
    ref = rg.ridge_grid(SD, Sr, src, nn, sc, lv)
    out = rg.ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu)).cpu()
    assert rg.repairs_done() >= 1                        # the n = 513 lambda = 0 system
    rel = ((out[:, 1:] - ref[:, 1:]).norm(dim=-1) / ref[:, 1:].norm(dim=-1)).max().item()
    assert rel < 1e-10, rel
    # n = 257 (leading block): lambda = 0 is regular here -> plain comparison
    r257 = ((out[1, 0] - ref[1, 0]).norm() / ref[1, 0].norm()).item()
    assert r257 < 1e-10, r257
    b = out[0, 0, :P]
    assert torch.isfinite(b).all()
    D0, r0 = SD[0], Sr[0]
    res = (D0 @ b - r0).norm().item()
    scale = (torch.linalg.matrix_norm(D0, ord=2) * b.norm() + r0.norm()).item()
    assert res <= 1e-12 * scale, (res, scale)


def test_quadform_utilities(gpu):
    """Utilities vs the CPU oracle for n with a split-off tail index (n - 1 a multiple of 16:
    129, 97, 65, 33, 17; csrc/quadform.hip quad_main) and without (130, 100, 1)."""
    from pfml.ops.ridge import quadform_utilities
    T, P, L = 5, 130, 101
    D = _spd_stack(T, P, n_obs=50, seed=31)
    R = _rand(T, P, seed=32)
    beta = _rand(4, L, P, seed=33)
    jc = np.array([0, 1, 2, 3, 3, 0, 1, 2, 3])
    jm = np.array([0, 1, 2, 3, 4, 4, 0, 3, 2])
    jn = np.array([130, 65, 33, 17, 130, 1, 129, 97, 100])
    ref = quadform_utilities(D, R, beta, jc, jm, jn)
    out = quadform_utilities(D.to(gpu), R.to(gpu), beta.to(gpu), jc, jm, jn).cpu()
    rel = ((out - ref).abs() / ref.abs().clamp_min(1e-12)).max().item()
    assert rel < 1e-11, rel


def test_grid_search_gpu_matches_cpu(gpu):
    from pfml.config import Config
    from pfml.models.search import PfmlReals, grid_search
    from pfml.utils.dates import mi_from_ym
    cfg = Config.default().override(["pf_ml.p_vec=[16,32]", "pf.dates.start_year=2001",
                                     "pf.dates.end_yr=2005"])
    G, P = 2, 33
    months = np.arange(mi_from_ym(1994, 3), mi_from_ym(2005, 11) + 1)
    T = len(months)
    X = _rand(G * T, 40, P, seed=41)
    D = (X.transpose(1, 2) @ X / 40).view(G, T, P, P)
    r = 0.1 * _rand(G, T, P, seed=42)
    cpu = grid_search(PfmlReals(months, r, D), cfg)
    dev = grid_search(PfmlReals(months, r.to(gpu), D.to(gpu)), cfg)
    rb = ((dev.beta.cpu() - cpu.beta).norm(dim=-1) / cpu.beta.norm(dim=-1)).max().item()
    assert rb < 1e-9
    ro = ((dev.obj.cpu() - cpu.obj).abs() / cpu.obj.abs().clamp_min(1e-12)).max().item()
    assert ro < 1e-8


@pytest.mark.parametrize("n,m,b", [(17, 5, 2), (64, 10, 2), (100, 37, 3), (490, 1028, 2),
                                   (512, 20, 1), (513, 1026, 2), (1500, 40, 2), (2900, 70, 2)])
def test_lu_solve_augmented(gpu, n, m, b):
    from pfml.ops.linalg import solve
    A = _rand(b, n, n, seed=n) + n ** 0.5 * torch.eye(n, dtype=torch.float64)
    A[:, 0, 0] = 1e-8                      # forces a row interchange in the first panel
    B = _rand(b, n, m, seed=m)
    ref = torch.linalg.solve(A, B)
    got = solve(A.to(gpu), B.to(gpu)).cpu()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 1e-10, rel


@pytest.mark.parametrize("n,m,b", [(490, 1026, 3), (512, 300, 2), (130, 70, 4), (100, 514, 2),
                                   (257, 33, 3), (700, 130, 2), (1100, 260, 2), (2100, 100, 2),
                                   (2900, 1026, 2)])
def test_lu_solve_two_level(gpu, n, m, b):
    """Two-level solve (128-wide panels, transform block Z in scratch columns, K = 128 GEMM
    updates) on the S4 layout [B | A | scratch] vs torch.linalg.solve; pivoting forced in
    the first and in a later panel.  n > 1024: the pivot panels of > 1024 rows are searched
    in registers (lu_pivot_reg_kernel, 2 and 3 row sets) - the 3000-stock stress sizes."""
    from pfml.ops.linalg import LU_PANEL_COLS, solve_augmented
    A = _rand(b, n, n, seed=n + 1) + 0.5 * n ** 0.5 * torch.eye(n, dtype=torch.float64)
    A[:, 0, 0] = 1e-8
    A[:, n // 2, n // 2] = 1e-9
    Bm = _rand(b, n, m, seed=m + 3)
    ref = torch.linalg.solve(A, Bm)
    M = torch.full((b, n, m + n + LU_PANEL_COLS), float("nan"), dtype=torch.float64)
    M[:, :, :m] = Bm
    M[:, :, m:m + n] = A
    Md = M.to(gpu)
    st = torch.zeros(b, dtype=torch.int32, device=gpu)
    got = solve_augmented(Md, n, m, a0=m, b0=0, status=st, z0=m + n).cpu()
    assert int(st.sum()) == 0
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < (1e-11 if n <= 512 else 1e-10), rel     # (rounding grows with n)


@pytest.mark.parametrize("n_obs", [1500, 400])
def test_ridge_tridiagonal_large_n(gpu, n_obs):
    """528 < n <= 1024 (p up to 1023, e.g. --set pf_ml.p_vec=[1023]) takes the blocked
    tridiagonal path (csrc/ridge.hip) with the dense device repair (csrc/ridge_repair.hip) of
    its non-SPD systems: the LU-solve oracle's betas, full-rank (n_obs = 1500, lambda = 0
    included) and rank-deficient (n_obs = 400 < n: the small lambdas repaired)."""
    from pfml.ops import ridge as rg
    P = 1024
    SD = _spd_stack(2, P, n_obs=n_obs, seed=151)
    SD = 0.5 * (SD + SD.transpose(1, 2))
    Sr = _rand(2, P, seed=152)
    lam = np.exp(np.linspace(-10, 10, 24)) if n_obs > P else np.exp(np.linspace(-2, 10, 24))
    lv = torch.tensor([0.0] + list(lam), dtype=torch.float64)
    src, nn, sc = np.array([0, 1, 0]), np.array([1024, 700, 529]), np.full(3, 1e-3)
    ref = rg.ridge_grid(SD, Sr, src, nn, sc, lv)
    out = rg.ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu)).cpu()
    assert not rg.band_path({"nmax": 1024})
    assert not torch.isnan(out).any()
    ok = slice(None) if n_obs > P else slice(1, None)         # (singular at lambda = 0)
    rel = ((out[:, ok] - ref[:, ok]).norm(dim=-1) / ref[:, ok].norm(dim=-1)).max().item()
    assert rel < 1e-9, rel


def test_ridge_dense_repair_tridiagonal_path(gpu):
    """The tridiagonal path's dense device repair (csrc/ridge_repair.hip: flag + pivoted LU,
    np.linalg.solve semantics) re-solves exactly the NaN-marked (cell, lambda) systems: betas
    of the LU oracle there, the other systems untouched."""
    from pfml.ops import ridge as rg
    P = 700
    SD = _spd_stack(2, P, n_obs=900, seed=153)
    Sr = _rand(2, P, seed=154)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-6, 6, 11))), dtype=torch.float64)
    src, nn, sc = np.array([0, 1, 1]), np.array([700, 600, 560]), np.full(3, 1e-3)
    beta = rg.ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu), repair=False)
    keep = beta.clone()
    marks = [(0, 0), (1, 5), (2, 11), (2, 3)]
    for c, l in marks:
        beta[c, l, :nn[c]] = float("nan")
    plan = rg.ridge_plan(P, len(lv), src, nn, sc)
    d_desc, = rg.upload([plan["desc"]], beta.device)
    cnt = rg.repair_launch(plan, d_desc, SD.to(gpu).contiguous(), Sr.to(gpu).contiguous(),
                           lv.to(gpu), beta)
    assert int(cnt.item()) == len(marks)
    ref = rg.ridge_grid(SD, Sr, src, nn, sc, lv)
    out = beta.cpu()
    for c, l in marks:
        rel = ((out[c, l] - ref[c, l]).norm() / ref[c, l].norm()).item()
        assert rel < 1e-9, (c, l, rel)
    untouched = torch.ones(beta.shape[:2], dtype=torch.bool)
    for c, l in marks:
        untouched[c, l] = False
    assert torch.equal(out[untouched], keep.cpu()[untouched])


@pytest.mark.parametrize("n_obs", [700, 90])
def test_band_coop_matches_lu_and_bitwise_across_k(gpu, n_obs, monkeypatch):
    """Cooperative band reduction (K workgroups per cell, the production form): for every n
    of the grid (513, 257, 129, 65) plus ragged ones (100, 17), full-rank (n_obs = 700) and
    rank-deficient (n_obs = 90: lambda = 0 repaired on the device), the betas are BITWISE
    equal for K = 1, 2, 3, 8 and 16 workgroups per cell - so the K a 1-GPU and an 8-GPU run
    choose (ops/ridge.py::coop_k) cannot change a hyper-parameter pick - and match the
    LU-solve oracle (np.linalg.solve per lambda, PFML_Search_Coef.py:131-133)."""
    from pfml.ops import ridge as rg
    P = 513
    SD = _spd_stack(3, P, n_obs=n_obs, seed=171)
    SD = 0.5 * (SD + SD.transpose(1, 2))           # exactly symmetric, like the window sums
    Sr = _rand(3, P, seed=172)
    if n_obs > P:
        lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64)
    else:
        lv = torch.tensor([0.0] + list(np.exp(np.linspace(-2, 10, 40))), dtype=torch.float64)
    for ncell in (513, 257, 129, 100, 65, 17):
        src = np.array([0, 1, 2])
        nn = np.full(3, ncell)
        sc = np.full(3, 1.5e-3)
        out = {}
        for k in ("1", "2", "3", "8", "16"):
            monkeypatch.setenv("PFML_COOP_K", k)
            out[k] = rg.ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu)).cpu()
            assert rg.coop_errors() == 0, (ncell, k)
        a = out["1"]
        for k, b in out.items():
            same = (a == b) | (torch.isnan(a) & torch.isnan(b))
            assert bool(same.all()), (ncell, k, float((a - b).abs().max()))
        ref = rg.ridge_grid(SD, Sr, src, nn, sc, lv)
        ok = slice(1, None) if n_obs <= ncell else slice(None)   # singular at lambda = 0
        rel = ((a[:, ok] - ref[:, ok]).norm(dim=-1) / ref[:, ok].norm(dim=-1)).max().item()
        assert rel < 1e-10, (ncell, rel)


def test_band_coop_mixed_launch_bitwise(gpu, monkeypatch):
    """Cells of different n in ONE cooperative launch (largest cells K > 1, the rest K = 1)
    give bitwise the betas of each cell launched alone at K = 1."""
    from pfml.ops import ridge as rg
    P = 513
    SD = _spd_stack(3, P, n_obs=700, seed=173)
    SD = 0.5 * (SD + SD.transpose(1, 2))
    Sr = _rand(3, P, seed=174)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64)
    src = np.array([0, 1, 2, 1, 0, 2, 2, 1])
    nn = np.array([513, 513, 65, 257, 129, 100, 513, 17])
    sc = np.full(len(src), 1.5e-3)
    monkeypatch.setenv("PFML_COOP_K", "4")
    mixed = rg.ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu)).cpu()
    assert rg.coop_errors() == 0
    monkeypatch.setenv("PFML_COOP_K", "1")
    for c in range(len(src)):
        one = rg.ridge_grid(SD.to(gpu), Sr.to(gpu), src[c:c + 1], nn[c:c + 1], sc[c:c + 1],
                            lv.to(gpu)).cpu()
        assert torch.equal(one[0], mixed[c]), c
    ref = rg.ridge_grid(SD, Sr, src, nn, sc, lv)
    rel = ((mixed - ref).norm(dim=-1) / ref.norm(dim=-1)).max().item()
    assert rel < 1e-10, rel


@pytest.mark.parametrize("streams", ["2", "1"])
def test_ridge_utilities_stream_groups(gpu, streams, monkeypatch):
    """ridge_utilities with the largest cells' chain on a side stream (default) or every cell
    on one stream (PFML_RIDGE_STREAMS=1) gives the CPU oracle's betas and utilities."""
    from pfml.ops.ridge import ridge_utilities
    monkeypatch.setenv("PFML_RIDGE_STREAMS", streams)
    P = 513
    SD = _spd_stack(3, P, n_obs=700, seed=65)
    Sr = _rand(3, P, seed=66)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64)
    src = np.array([0, 1, 2, 1, 0, 2, 2, 0])
    nn = np.array([513, 513, 65, 257, 513, 129, 513, 65])
    sc = np.full(len(src), 1.5e-3)
    D = _spd_stack(4, P, n_obs=600, seed=67) * 1e-3
    R = _rand(4, P, seed=68)
    jc = np.repeat(np.arange(len(src)), 2)
    jm = np.tile(np.array([1, 3]), len(src))
    jn = nn[jc]
    rb, ro = ridge_utilities(SD, Sr, src, nn, sc, lv, D, R, jc, jm, jn)
    gb, go = ridge_utilities(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu), D.to(gpu),
                             R.to(gpu), jc, jm, jn)
    torch.cuda.synchronize()
    rel = ((gb.cpu() - rb).norm(dim=-1) / rb.norm(dim=-1).clamp(min=1e-300)).max().item()
    assert rel < 1e-8, rel
    assert torch.allclose(go.cpu(), ro, rtol=1e-8, atol=1e-12 * ro.abs().max().item())


def test_backtransform_size_classes(gpu, monkeypatch):
    """The back-transform's size-class instances (2 / 4 / 4 / 8 waves for n <= 96 / 192 / 320
    / 528, csrc/ridge_band.hip ridge_band_bt_launch) against the single 8-wave form
    (PFML_BT_CLASSES=0) on a launch mixing all four classes: the same betas to rounding (the
    partial sums of V'Y run over a different wave split), and both against the CPU oracle."""
    from pfml.ops import ridge as rg
    P = 513
    SD = _spd_stack(2, P, n_obs=700, seed=95)
    Sr = _rand(2, P, seed=96)
    lv = torch.tensor([1e-4] + list(np.exp(np.linspace(-6, 6, 40))), dtype=torch.float64)
    src = np.array([0, 1, 0, 1, 0, 1, 1])
    nn = np.array([513, 257, 129, 65, 300, 96, 17])
    sc = np.full(len(src), 1.5e-3)
    out = {}
    for v in ("0", "1"):
        monkeypatch.setenv("PFML_BT_CLASSES", v)
        out[v] = rg.ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu)).cpu()
    ref = rg.ridge_grid(SD, Sr, src, nn, sc, lv)
    for v in ("0", "1"):
        rel = ((out[v] - ref).norm(dim=-1) / ref.norm(dim=-1).clamp(min=1e-300)).max().item()
        assert rel < 1e-9, (v, rel)
    rel = ((out["1"] - out["0"]).norm(dim=-1) / out["0"].norm(dim=-1).clamp(min=1e-300)).max().item()
    assert rel < 1e-12, rel


@pytest.mark.parametrize("fmt", ["bf16", "fp8"])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True)])
def test_gemm_lowp(gpu, fmt, ta, tb):
    """Low-precision MFMA GEMM (bf16 / fp8-e4m3 operands, fp32 accumulate): matches the CPU
    oracle with the same operand rounding, and the fp64 product within the format's error."""
    from pfml.ops.gemm import gemm_lowp
    b, M, N, K = 3, 100, 70, 150
    A = _rand(b, K, M, seed=71) if ta else _rand(b, M, K, seed=71)
    B = _rand(b, N, K, seed=72) if tb else _rand(b, K, N, seed=72)
    C0 = _rand(b, M, N, seed=73)
    ref = gemm_lowp(A, B, fmt, trans_a=ta, trans_b=tb, alpha=0.5, beta=0.25, out=C0.clone())
    out = gemm_lowp(A.to(gpu), B.to(gpu), fmt, trans_a=ta, trans_b=tb, alpha=0.5, beta=0.25,
                    out=C0.to(gpu)).cpu()
    scale = ref.abs().max().item()
    assert (out - ref).abs().max().item() / scale < (2e-6 if fmt == "bf16" else 2e-2)
    a = A.transpose(1, 2) if ta else A
    bb = B.transpose(1, 2) if tb else B
    exact = 0.5 * a @ bb + 0.25 * C0
    assert (out - exact).abs().max().item() / scale < (1e-2 if fmt == "bf16" else 1e-1)


def test_window_prefix_vec(gpu):
    """One-launch expanding-window sums of month vectors (r_tilde), incl. gaps and skip."""
    from pfml.ops.ridge import window_prefix_vec
    X = _rand(2, 40, 513, seed=83)
    for st, sp, skip in (([0, 7, 9, 20], [7, 9, 20, 40], 0), ([0, 10, 11], [5, 11, 40], 1)):
        ref = window_prefix_vec(X, st, sp, skip=skip)
        got = window_prefix_vec(X.to(gpu), st, sp, skip=skip).cpu()
        assert got.shape == ref.shape and got.is_contiguous()
        assert torch.allclose(got, ref, rtol=1e-13, atol=1e-13)


def test_window_prefix_sym(gpu):
    """Fused expanding-window sums over the upper triangles of symmetric month matrices."""
    from pfml.ops.ridge import window_prefix_sym
    X = _rand(2, 40, 37, 37, seed=81)
    X = X + X.transpose(-1, -2)
    st, sp = [0, 7, 9, 20], [7, 9, 20, 40]
    ref = window_prefix_sym(X, st, sp)
    out = window_prefix_sym(X.to(gpu), st, sp).cpu()
    assert torch.allclose(out, ref, rtol=1e-13, atol=1e-12)
    assert torch.equal(out, out.transpose(-1, -2))
    gap_st, gap_sp = [0, 10], [5, 40]          # months 5..9 belong to no segment
    ref2 = window_prefix_sym(X, gap_st, gap_sp)
    assert torch.allclose(window_prefix_sym(X.to(gpu), gap_st, gap_sp).cpu(), ref2,
                          rtol=1e-13, atol=1e-12)
    for skip in (1, 2):                         # prefix-only leading segments
        got = window_prefix_sym(X.to(gpu), st, sp, skip=skip).cpu()
        assert got.shape == (2, 4 - skip, 37, 37) and got.is_contiguous()
        assert torch.allclose(got, ref[:, skip:], rtol=1e-13, atol=1e-12)
        assert torch.equal(got, got.transpose(-1, -2))
    for P in (64, 513):                         # even P; P + 1 > 512 (three entries per lane)
        Y = _rand(1, 12, P, P, seed=82 + P)
        Y = Y + Y.transpose(-1, -2)
        st2, sp2 = [0, 2, 5, 11], [2, 5, 11, 12]
        ref3 = window_prefix_sym(Y, st2, sp2, skip=1)
        got = window_prefix_sym(Y.to(gpu), st2, sp2, skip=1).cpu()
        assert torch.allclose(got, ref3, rtol=1e-13, atol=1e-12)
        assert torch.equal(got, got.transpose(-1, -2))


@pytest.mark.parametrize("compat", [True, False])
def test_validation_scores_kernel(gpu, compat):
    """csrc/scores.hip (prefix mean + per-month dense rank) vs the torch path on CPU, incl.
    exact ties across (p, l) cells and a NaN."""
    from pfml.models.search import validation_scores
    g = torch.Generator().manual_seed(5)
    obj = torch.randn(37, 2, 4, 101, generator=g, dtype=torch.float64)
    obj[:, :, 1, :] = obj[:, :, 0, :]                     # exact ties
    obj[3, 1, 2, 7] = float("nan")
    for fg in (0, 1):
        ref = validation_scores(obj, fg, compat)
        got = validation_scores(obj.to(gpu), fg, compat)
        assert torch.allclose(got[0].cpu(), ref[0], rtol=0, atol=0, equal_nan=True)
        assert torch.allclose(got[1].cpu(), ref[1], rtol=1e-12, atol=1e-14, equal_nan=True)
        assert torch.equal(got[2].cpu(), ref[2])


@pytest.mark.parametrize("compat", [True, False])
@pytest.mark.parametrize("G,nP", [(2, 4), (3, 2)])
def test_validation_scores_all_frames(gpu, compat, G, nP):
    """All frames in one prefix-mean + one dense-rank launch (blockIdx.y = frame, sort width
    sized per frame) give the per-frame kernels' cum_obj and ranks bitwise, and the CPU path's."""
    from pfml.models.search import validation_scores, validation_scores_all
    g = torch.Generator().manual_seed(9)
    obj = torch.randn(29, G, nP, 101, generator=g, dtype=torch.float64)
    obj[:, :, 1, :] = obj[:, :, 0, :]                     # exact ties
    obj[2, 0, 1, 5] = float("nan")
    allf = validation_scores_all(obj.to(gpu), compat)
    for fg in range(G):
        one = validation_scores(obj.to(gpu), fg, compat)
        ref = validation_scores(obj, fg, compat)
        for a, b, c in zip(allf[fg], one, ref):
            assert torch.equal(torch.nan_to_num(a.cpu(), nan=-7.0), torch.nan_to_num(b.cpu(), nan=-7.0))
            assert torch.allclose(a.cpu(), c, rtol=1e-12, atol=1e-14, equal_nan=True)


def test_grid_search_bitwise_deterministic(gpu):
    """Replays of the device grid search are bitwise identical (fixed tilings and reduction
    orders, no float atomics; SURVEY §5.2 deterministic replay), incl. the cached-plan path."""
    from pfml.config import Config
    from pfml.models.search import PfmlReals, grid_search, validation_scores
    from pfml.utils.dates import mi_from_ym
    cfg = Config.default().override(["pf_ml.p_vec=[16,64]", "pf.dates.start_year=2001",
                                     "pf.dates.end_yr=2006"])
    G, P = 2, 65
    months = np.arange(mi_from_ym(1994, 3), mi_from_ym(2006, 11) + 1)
    T = len(months)
    X = _rand(G * T, 80, P, seed=91).to(gpu)
    D = (X.transpose(1, 2) @ X / 80).view(G, T, P, P).contiguous()
    r = (0.1 * _rand(G, T, P, seed=92)).to(gpu)
    runs = []
    for _ in range(3):
        res = grid_search(PfmlReals(months, r, D), cfg)
        runs.append((res.beta.cpu(), res.obj.cpu(), validation_scores(res.obj, 1, True)[2].cpu()))
    for b, o, k in runs[1:]:
        assert torch.equal(b, runs[0][0]) and torch.equal(o, runs[0][1])
        assert torch.equal(k, runs[0][2])


@pytest.mark.parametrize("P", [65, 513])
def test_ridge_device_repair_matches_lu(gpu, P):
    """Systems the banded Cholesky cannot factor (here an indefinite Dbar: small lambda makes
    Dbar + lambda I indefinite) are NaN-marked by the band path and re-solved on the device by
    a pivoted banded LU before the back-transform - no host round trip; betas match
    np.linalg.solve (dense pivoted LU).  P = 513: production-size cells (n = 513 / 257 / 20)."""
    from pfml.ops import ridge as rg
    X = _rand(2, max(200, 2 * P), P, seed=61)
    SD = X.transpose(1, 2) @ X / X.shape[1]
    e, V = torch.linalg.eigh(SD[1])
    SD[1] = SD[1] - (e[0] + 0.7) * torch.outer(V[:, 0], V[:, 0]) * 2.0   # one eigen < 0
    Sr = _rand(2, P, seed=62)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64)
    src, sc = np.array([0, 1, 1, 1]), np.array([1.0, 1.0, 1.0, 1.0])
    nn = np.array([P, P, (P + 1) // 2, 20])
    ref = rg.ridge_grid(SD, Sr, src, nn, sc, lv)            # CPU: LU per lambda
    out = rg.ridge_grid(SD.to(gpu), Sr.to(gpu), src, nn, sc, lv.to(gpu)).cpu()
    assert rg.repairs_done() > 0
    ok = torch.isfinite(ref).all(-1)
    rel = ((out - ref).norm(dim=-1) / ref.norm(dim=-1).clamp_min(1e-300))[ok].max().item()
    assert rel < 1e-9, rel
    assert torch.isfinite(out[ok]).all()


def test_validation_scores_nan_cells(gpu):
    """A singular cell (NaN utilities) gets NaN cum_obj until its first finite value and a NaN
    rank, and never takes rank 1 (pandas expanding().mean() / rank(method='dense'))."""
    from pfml.models.search import validation_scores
    obj = _rand(24, 2, 2, 101, seed=71)
    obj[:, 0, 1, 7] = float("nan")                        # one cell singular throughout
    obj[:5, 1, 0, 3] = float("nan")                        # another singular early on
    for compat in (True, False):
        _, c0, r0 = validation_scores(obj, 1, compat)
        _, c1, r1 = validation_scores(obj.to(gpu), 1, compat)
        c1, r1 = c1.cpu(), r1.cpu()
        assert torch.equal(torch.isnan(c0), torch.isnan(c1))
        assert torch.allclose(c0.nan_to_num(), c1.nan_to_num(), rtol=1e-13, atol=1e-15)
        assert torch.equal(torch.isnan(r0), torch.isnan(r1))
        assert torch.equal(r0.nan_to_num(-1), r1.nan_to_num(-1))
        for v in range(24):
            rv = r1[v].reshape(-1)
            fin = rv[~torch.isnan(rv)]
            assert fin.min() == 1 and torch.equal(torch.unique(fin),
                                                  torch.arange(1, int(fin.max()) + 1).double())


def test_validation_rank_ties_zeros_infs(gpu):
    """Dense rank on the device (order-preserving 64-bit sort keys) on exact ties, +0 / -0
    (one rank), +-inf and NaN, against the CPU (pandas-semantics) ranks."""
    from pfml.models.search import validation_scores
    obj = torch.round(_rand(24, 2, 2, 101, seed=72) * 4) / 4   # many exact ties
    obj[:, 0, 0, :10] = 0.0
    obj[:, 1, 0, 10:20] = -0.0
    obj[3, 0, 1, 5] = float("inf")
    obj[4, 1, 1, 6] = -float("inf")
    obj[:, 1, 1, 50] = float("nan")
    for compat in (True, False):
        _, _, r0 = validation_scores(obj, 1, compat)
        _, _, r1 = validation_scores(obj.to(gpu), 1, compat)
        assert torch.equal(r0.nan_to_num(-1), r1.cpu().nan_to_num(-1))


def _chunked_windows_all_ranks(X, R, months, years, W, dev):
    """Window sums of every rank of a W-rank run, the all-gather emulated in one process:
    each rank's chunk totals (its local months only), concatenated in canonical slot order,
    then each rank's windows.  Returns {global hp-year index: (SD, Sr)}."""
    from pfml.models.search import _search_setup, local_month_rows
    from pfml.ops.ridge import chunk_totals, chunk_windows
    G, T, P, _ = X.shape
    lv = np.array([0.0, 1.0])
    sus, tots = [], []
    for r in range(W):
        rows = local_month_rows(months, years, W, r)
        Xr = X[:, rows].contiguous().to(dev)
        Rr = R[:, rows].contiguous().to(dev)
        su = _search_setup(months, years, [16], G, len(rows), W, r,
                           torch.device(dev) if dev != "cpu" else None, lv, rows)
        totD, totR, bufs = chunk_totals(Xr, Rr, su)
        sus.append((su, Xr, Rr, bufs))
        tots.append((totD, totR))
    allD = torch.cat([t[0] for t in tots])
    allR = torch.cat([t[1] for t in tots])
    out = {}
    for su, Xr, Rr, bufs in sus:
        SD, Sr = chunk_windows(Xr, Rr, su, allD, allR, bufs)
        for k, y in enumerate(su["yl"]):
            out[int(y)] = (SD[:, k].cpu(), Sr[:, k].cpu())
    return out


def test_chunked_window_sums_world_bitwise(gpu):
    """Canonical chunked window sums (csrc/segsum.hip chunk kernels): on the device every
    hp-year window is BITWISE the same for a 1, 2, 3 and 4-rank sharding, and matches the
    CPU folds to rounding."""
    from pfml.models.search import make_plan
    from pfml.utils.dates import mi_from_ym
    G, P = 2, 37
    months = np.arange(mi_from_ym(1990, 0), mi_from_ym(2012, 11) + 1, dtype=np.int64)
    years = np.arange(1998, 2012)
    T = len(months)
    X = _rand(G, T, P, P, seed=91)
    X = X + X.transpose(-1, -2)
    R = _rand(G, T, P, seed=92)
    ref = _chunked_windows_all_ranks(X, R, months, years, 1, gpu)
    cpu = _chunked_windows_all_ranks(X, R, months, years, 1, "cpu")
    assert sorted(ref) == list(range(len(years)))
    for y in ref:
        assert torch.allclose(ref[y][0], cpu[y][0], rtol=1e-12, atol=1e-11)
        assert torch.allclose(ref[y][1], cpu[y][1], rtol=1e-12, atol=1e-11)
        assert torch.equal(ref[y][0], ref[y][0].transpose(-1, -2))
    plan = make_plan(months, years)
    last = int(plan.seg_stop[len(years) - 1])
    full = X[:, :last].sum(1)
    assert torch.allclose(ref[len(years) - 1][0], full, rtol=1e-12, atol=1e-11)
    for W in (2, 3, 4):
        got = _chunked_windows_all_ranks(X, R, months, years, W, gpu)
        assert sorted(got) == sorted(ref)
        for y in ref:
            assert torch.equal(got[y][0], ref[y][0]), (W, y)
            assert torch.equal(got[y][1], ref[y][1]), (W, y)


def test_quadform_two_months_bitwise(gpu, monkeypatch):
    """Two validation months per workgroup (shared beta tiles) give BITWISE the utilities of
    one month per workgroup (same per-month MFMA order), incl. an odd job out and n < 64."""
    from pfml.ops.ridge import quadform_utilities
    P, L = 130, 101
    D = _spd_stack(7, P, n_obs=150, seed=95) / 150
    R = _rand(7, P, seed=96)
    beta = _rand(3, L, P, seed=97)
    jc = np.array([0, 0, 0, 1, 1, 2, 2, 2, 2])
    jm = np.array([0, 1, 2, 3, 4, 5, 6, 0, 1])
    jn = np.array([130, 130, 130, 65, 65, 33, 33, 33, 33])
    args = (D.to(gpu), R.to(gpu), beta.to(gpu), jc, jm, jn)
    monkeypatch.setenv("PFML_QUAD_DIRECT", "0")
    monkeypatch.setenv("PFML_QUAD_MM", "1")
    one = quadform_utilities(*args).cpu()
    monkeypatch.setenv("PFML_QUAD_MM", "2")
    two = quadform_utilities(*args).cpu()
    assert torch.equal(one, two)
    ref = quadform_utilities(D, R, beta, jc, jm, jn)
    assert torch.allclose(two, ref, rtol=1e-11, atol=1e-11)
    # the direct-A form (default for one-month tiles): its own k order, same oracle
    monkeypatch.setenv("PFML_QUAD_MM", "1")
    monkeypatch.setenv("PFML_QUAD_DIRECT", "1")
    direct = quadform_utilities(*args).cpu()
    assert torch.allclose(direct, ref, rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize("direct", ["0", "1"])
def test_quadform_production_shape(gpu, monkeypatch, direct):
    """Both utilities forms at the production cell size (n = 513: nine row tiles, tail index
    split off) and a mixed launch (n = 257 / 129 / 65 cells), against the CPU oracle."""
    from pfml.ops.ridge import quadform_utilities
    monkeypatch.setenv("PFML_QUAD_DIRECT", direct)
    P, L = 513, 101
    D = _spd_stack(4, P, n_obs=600, seed=98) / 600
    R = _rand(4, P, seed=99)
    beta = 0.1 * _rand(4, L, P, seed=100)
    jc = np.array([0, 0, 1, 2, 3, 0])
    jm = np.array([0, 1, 2, 3, 0, 3])
    jn = np.array([513, 513, 257, 129, 65, 513])
    out = quadform_utilities(D.to(gpu), R.to(gpu), beta.to(gpu), jc, jm, jn).cpu()
    ref = quadform_utilities(D, R, beta, jc, jm, jn)
    rel = ((out - ref).abs() / ref.abs().clamp_min(1e-9)).max().item()
    assert rel < 1e-10, rel
