"""Shared body of the zero-variance factor-correlation tests (CPU and GPU forms)."""
import numpy as np
import torch


def check_zero_variance_modes(device) -> None:
    from pfml.ops.risk_kernels import ewma_factor_cov
    from pfml import reference_api as ra
    import pandas as pd
    g = torch.Generator().manual_seed(3)
    days, K, obs = 2700, 6, 2520
    fr = torch.randn(days, K, generator=g, dtype=torch.float64) * 0.01
    fr[:, 2] = 0.0                                     # zero variance in every window
    ends = np.array([2600, 2700])
    tr = np.arange(obs, 0, -1, dtype=np.float64)
    w_cor, w_var = (0.5 ** (1.0 / 378)) ** tr, (0.5 ** (1.0 / 126)) ** tr
    other = [0, 1, 3, 4, 5]
    out = {}
    for mode in (True, False):
        F, cor, var = ewma_factor_cov(fr.to(device), ends, obs, w_cor, w_var, scale=21.0,
                                      return_parts=True, nan_cor=mode)
        out[mode] = (F.cpu(), cor.cpu())
    Fc, cc = out[True]
    Fk, ck = out[False]
    assert torch.isnan(cc[:, 2, other]).all() and torch.isnan(cc[:, other, 2]).all()
    assert (cc[:, 2, 2] == 1.0).all()
    assert torch.isnan(Fc[:, 2, other]).all() and (Fc[:, 2, 2] == 0.0).all()
    assert (ck[:, 2, other] == 0.0).all() and (Fk[:, 2, :] == 0.0).all()
    assert torch.isfinite(Fk).all()
    keep = np.ix_(range(len(ends)), other, other)
    assert torch.equal(Fc[keep], Fk[keep])
    # the reference's own weighted_cor_wt on the last window: NaN pattern and values
    t = obs
    win = pd.DataFrame(fr[ends[-1] - t:ends[-1]].numpy())
    ref = ra.weighted_cor_wt(win, w_cor[obs - t:]).to_numpy()
    assert np.array_equal(np.isnan(ref), np.isnan(cc[-1].numpy()))
    fin = ~np.isnan(ref)
    assert np.allclose(cc[-1].numpy()[fin], ref[fin], rtol=1e-12, atol=1e-14)
