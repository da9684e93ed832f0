import os, sys, torch, numpy as np
sys.path.insert(0, os.getcwd())
from pfml.ops.gemm import gemm
from pfml.ops import linalg as la
dev = torch.device("cuda", 0)
torch.manual_seed(0)
B, N, K = 5, 50, 25
Xl = torch.randn(B, N, K, dtype=torch.float64, device=dev)
Xl[:, 40:] = 0
Fb = torch.randn(B, K, 300, dtype=torch.float64, device=dev); Fb = Fb @ Fb.transpose(1, 2) * 1e-4
for be in ("own", "blas"):
    S = gemm(gemm(Xl, Fb, backend=be), Xl, trans_b=True, backend=be)
    print(be, float(S.abs().sum()), float((S - Xl @ Fb @ Xl.transpose(1, 2)).abs().max()))
A = torch.randn(B, N, N, dtype=torch.float64, device=dev)
for be in ("own", "blas"):
    C = gemm(A, A, backend=be)
    print(be, float((C - A @ A).abs().max()))
    Y = gemm(A, A, alpha=0.5, backend=be)
    print(be, "alpha", float((Y - 0.5 * A @ A).abs().max()))
    Z = torch.ones_like(A); gemm(A, A, alpha=-1.0, beta=1.0, out=Z, backend=be)
    print(be, "beta", float((Z - (1 - A @ A)).abs().max()))
    W = torch.zeros(B, N, N + 8, dtype=torch.float64, device=dev)
    gemm(A[:, :, :8], A[:, :8, :8], alpha=-1.0, out=W[:, :, 3:11], backend=be)
    print(be, "strided", float((W[:, :, 3:11] + A[:, :, :8] @ A[:, :8, :8]).abs().max()))
