"""L6/L7 portfolio construction and reporting.

* ``aim_portfolios``   - PFML_aim_fun.py:130-163: December rank-1 hyper-parameters per g,
                         w_aim = s_t beta (K18), coefficients of year oos_year (quirk Q13);
* ``hps_bundle``       - PFML_hps.py: {g: {aim_pfs_list, validation, rff_w}};
* ``best_hps``         - PFML_best_hps.py:263-308: cross-g rank-first selection;
* ``pfml_weights``     - PFML_best_hps.py:137-218: value-weighted start, weight recursion (17)
                         w_t = m_t w_start + (I - m_t) w_aim: m_t batched per rank (K19), the
                         chain as device GEMVs (no per-month host round trip), one N-vector
                         hand-off between ranks;
* ``pf_ts`` / ``pf_summary`` - :220-259, :326-358 (quirks Q3, Q18);
* ``plots``            - cumulative-performance / hyper-parameter figures (matplotlib).
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd
import torch

from ..config import Config
from ..data import io
from ..ops import linalg as la
from ..ops import _native as nat
from ..ops.gemm import gemm_fused
from ..utils.dates import month_end, month_index
from ..utils.log import get_logger
from .risk import BarraCov

_P, _I, _L = nat.C.c_void_p, nat.C.c_int, nat.C.c_int64
nat.register_hip("pfml_weights_chain", [_P, _L, _L, _P, _P, _P, _P, _P, _L, _P, _I, _I, _P, _P,
                                        _P, _P])
nat.register_hip("pfml_weights_chain_max_n", [])
nat.register_hip("pfml_aim_gemv", [_P, _I, _I, _P, _L, _P, _P])
nat.register_hip("pfml_aim_job_size", [])
AIM_JOB = np.dtype([("s", "<u8"), ("ld", "<i8"), ("off", "<i8"), ("nrow", "<i4"),
                    ("nk", "<i4")])

log = get_logger("portfolio")


def _opt_hps(validation: pd.DataFrame, g: int) -> pd.DataFrame:
    v = validation[validation["g"] == g]
    er = pd.to_datetime(v["eom_ret"])
    sel = v[(er.dt.month == 12).to_numpy() & (v["rank"] == 1).to_numpy()]
    return pd.DataFrame({"hp_end": pd.to_datetime(sel["eom_ret"]).dt.year.to_numpy(),
                         "l": sel["l"].to_numpy(), "p": sel["p"].to_numpy()})


def aim_portfolios(cfg: Config, validation: pd.DataFrame, beta_years: np.ndarray,
                   beta: torch.Tensor, signal_months: np.ndarray, signal_t: list,
                   signal_ids: list, oos_months: np.ndarray) -> dict:
    """{g: {d: {'aim_pf': DataFrame(id, eom, w_aim), 'coef': ndarray}}} (internal order).

    w_aim = s_t beta (K18) for every (g, month): on the device ONE launch over all of them
    (csrc/weights.hip aim_gemv_kernel reads the S4 signal views in place; coefficients
    gathered by one index op), one host copy at the end; on the CPU one product per month."""
    G = beta.shape[0]
    p_vec = cfg.p_vec
    mpos = {int(m): i for i, m in enumerate(signal_months)}
    byear = np.asarray(beta_years)
    meta = []                                     # (g, d, i, p, l, year index, p index)
    for g in range(G):
        opt = _opt_hps(validation, g)
        sel = {int(y): (int(p), int(l)) for y, p, l in zip(opt["hp_end"], opt["p"], opt["l"])}
        for d in oos_months:
            oos_year = int(month_end(int(d) + 1).year[0])
            if oos_year - 1 not in sel:
                raise KeyError(f"no December rank-1 hyper-parameters for {oos_year - 1}")
            p, l = sel[oos_year - 1]
            hit = np.nonzero(byear == oos_year)[0]
            if len(hit) == 0:
                raise KeyError(f"coefficients of hp year {oos_year} are not on this rank")
            meta.append((g, int(d), mpos[int(d)], p, l, int(hit[0]), p_vec.index(p)))
    J = len(meta)
    out: dict = {g: {} for g in range(G)}
    if J == 0:
        return out
    gi = torch.as_tensor([m[0] for m in meta], device=beta.device)
    yi = torch.as_tensor([m[5] for m in meta], device=beta.device)
    pi = torch.as_tensor([m[6] for m in meta], device=beta.device)
    li = torch.as_tensor([m[4] for m in meta], device=beta.device)
    coefs = beta[gi, yi, pi, li].contiguous()          # [J, P], zero beyond p + 1
    sig = [signal_t[m[0]][m[2]] for m in meta]
    nrows = np.asarray([int(x.shape[0]) for x in sig], np.int64)
    offs = np.concatenate([[0], np.cumsum(nrows)[:-1]])
    if nat.is_device(beta) and all(x.is_cuda and x.stride(-1) == 1 for x in sig):
        from ..ops.ridge import upload
        if nat.hip_lib().pfml_aim_job_size() != AIM_JOB.itemsize:
            raise RuntimeError("AimJob layout mismatch between python and libpfml_hip")
        jobs = np.zeros(J, AIM_JOB)
        jobs["s"] = [x.data_ptr() for x in sig]
        jobs["ld"] = [x.stride(0) for x in sig]
        jobs["off"] = offs
        jobs["nrow"] = nrows
        jobs["nk"] = [m[3] + 1 for m in meta]
        (dj,) = upload([jobs], beta.device)
        w = torch.empty(int(nrows.sum()), dtype=torch.float64, device=beta.device)
        nat.check(nat.hip_lib().pfml_aim_gemv(dj.data_ptr(), J, int(nrows.max()),
                                              coefs.data_ptr(), coefs.shape[1], w.data_ptr(),
                                              nat.stream_of(beta)), "pfml_aim_gemv")
        w_all = w.cpu().numpy()
    else:
        w_all = torch.cat([s_[:, : m[3] + 1] @ coefs[k, : m[3] + 1].to(s_.device)
                           for k, (s_, m) in enumerate(zip(sig, meta))]).cpu().numpy()
    c_all = coefs.cpu().numpy()
    for k, (g, d, i, p, l, _, _) in enumerate(meta):
        o, n = int(offs[k]), int(nrows[k])
        out[g][d] = {"aim_pf": pd.DataFrame({"id": signal_ids[i], "eom": month_end(d)[0],
                                             "w_aim": w_all[o:o + n]}),
                     "coef": c_all[k, : p + 1].copy(), "p": p, "l": l}
    return out


def gather_aims(local: dict, cfg: Config, device) -> dict:
    """All-gather the per-rank aim portfolios (rows: g, month, id, w_aim; one coefficient
    row per (g, month)) so every rank holds the full set.  Single process: identity."""
    from ..parallel import collectives as coll
    from ..parallel.dist import env as dist_env
    if not dist_env().is_dist:
        return local
    Pm = cfg.p_max + 1
    rows, crow = [], []
    for g, per in local.items():
        for d, a in per.items():
            df = a["aim_pf"]
            n = len(df)
            rows.append(np.stack([np.full(n, g, np.float64), np.full(n, d, np.float64),
                                  df["id"].to_numpy(np.float64),
                                  df["w_aim"].to_numpy(np.float64)], axis=1))
            c = np.zeros(4 + Pm)
            c[:4] = (g, d, a["p"], a["l"])
            c[4:4 + len(a["coef"])] = a["coef"]
            crow.append(c)
    dev = torch.device(device)
    R = torch.as_tensor(np.concatenate(rows) if rows else np.zeros((0, 4)), dtype=torch.float64,
                        device=dev)
    Cc = torch.as_tensor(np.stack(crow) if crow else np.zeros((0, 4 + Pm)), dtype=torch.float64,
                         device=dev)
    R = coll.all_gather_varlen(R).cpu().numpy()
    Cc = coll.all_gather_varlen(Cc).cpu().numpy()
    out: dict = {}
    key = R[:, 0] * 1e7 + R[:, 1]
    order = np.argsort(key, kind="stable")
    R = R[order]
    bounds = np.flatnonzero(np.diff(R[:, 0] * 1e7 + R[:, 1])) + 1
    parts = np.split(R, bounds) if len(R) else []
    cmap = {(int(c[0]), int(c[1])): c for c in Cc}
    for part in parts:
        g, d = int(part[0, 0]), int(part[0, 1])
        c = cmap[(g, d)]
        p = int(c[2])
        out.setdefault(g, {})[d] = {
            "aim_pf": pd.DataFrame({"id": part[:, 2].astype(np.int64), "eom": month_end(d)[0],
                                    "w_aim": part[:, 3]}),
            "coef": c[4:4 + p + 1].copy(), "p": p, "l": int(c[3])}
    for g in out:
        out[g] = dict(sorted(out[g].items()))
    return out


def hps_bundle(aims: dict, validation: pd.DataFrame, rff_w: np.ndarray) -> dict:
    return {g: {"aim_pfs_list": aims[g], "validation": validation[validation["g"] == g],
                "rff_w": rff_w[g]} for g in aims}


def best_hps(hps: dict, oos_months: np.ndarray):
    """Cross-g selection: rank 'first' by cum_obj within eom_ret, December rank 1."""
    bh = pd.concat([h["validation"] for h in hps.values()], ignore_index=True).drop(columns="rank")
    bh["eom"] = pd.to_datetime(bh["eom"])
    bh["eom_ret"] = pd.to_datetime(bh["eom_ret"])
    bh["rank"] = bh.groupby("eom_ret")["cum_obj"].rank(ascending=False, method="first")
    bh = bh[(bh["rank"] == 1) & (bh["eom_ret"].dt.month == 12)]
    chosen, aims = {}, []
    for d in oos_months:
        oos_year = int(month_end(int(d) + 1).year[0])
        sel = bh[bh["eom_ret"].dt.year == oos_year - 1]
        g = int(sel["g"].iloc[0])
        a = hps[g]["aim_pfs_list"][int(d)]
        chosen[int(d)] = {"g": g, "p": int(sel["p"].iloc[0]), "aim": a["aim_pf"], "coef": a["coef"]}
        aims.append(a["aim_pf"])
    return bh, chosen, pd.concat(aims, ignore_index=True)


def _exact_lookup(keys: np.ndarray, q: np.ndarray, what: str) -> np.ndarray:
    """Positions of ``q`` in the sorted unique ``keys``; KeyError if any is absent."""
    if len(q) == 0:
        return np.zeros(0, np.int64)
    p = np.clip(np.searchsorted(keys, q), 0, max(len(keys) - 1, 0))
    if len(keys) == 0 or np.any(keys[p] != q):
        raise KeyError(f"{what}: missing keys")
    return p


def _month_values(frame: pd.DataFrame, col: str, months: np.ndarray) -> np.ndarray:
    mi = month_index(frame["eom"])
    o = np.argsort(mi, kind="stable")
    return frame[col].to_numpy(np.float64)[o][_exact_lookup(mi[o], np.asarray(months), col)]


def _weights_plan(cfg: Config, chars: pd.DataFrame, wealth: pd.DataFrame, aims: pd.DataFrame,
                  oos_months: np.ndarray) -> dict:
    """Host layout of the recursion, vectorised (no per-month Python loop): the valid rows of
    every OOS month in id order (only the columns the recursion reads), each month's aim
    weights aligned to them, the drift map from month t's rows to month t+1's (position of
    each id of t+1 among t's rows, or -1 for a new name), and the month of every row."""
    mi_all = month_index(chars["eom"])
    months = np.asarray(oos_months, np.int64)
    # OOS membership by a month lookup table (months are a short integer range)
    if len(months):
        lo = int(min(months.min(), mi_all.min())) if len(mi_all) else int(months.min())
        hi = int(max(months.max(), mi_all.max())) if len(mi_all) else int(months.max())
        lut = np.zeros(hi - lo + 1, bool)
        lut[months - lo] = True
        in_oos = lut[mi_all - lo]
    else:
        in_oos = np.zeros(len(mi_all), bool)
    rows = np.nonzero(in_oos & chars["valid"].to_numpy())[0]
    ids_sel = chars["id"].to_numpy(np.int64)[rows]
    # (mi, id) order: one int64 key, sorted only if the panel is not already in that order
    skey = mi_all[rows] * 10_000_000 + ids_sel
    if len(skey) > 1 and not (skey[1:] >= skey[:-1]).all():
        rows = rows[np.argsort(skey, kind="stable")]
    cols = [c for c in ("id", "me", "tr_ld1", "lambda") if c in chars.columns]
    data = pd.DataFrame({c: chars[c].to_numpy()[rows] for c in cols})
    data["mi"] = mi_all[rows]
    mi = data["mi"].to_numpy()
    starts = np.searchsorted(mi, months, "left")
    stops = np.searchsorted(mi, months, "right")
    ids_all = data["id"].to_numpy(np.int64)
    trow = np.searchsorted(months, mi)                  # month position of every row
    aim_key = month_index(aims["eom"]) * 10_000_000 + aims["id"].to_numpy(np.int64)
    ak, av = aim_key, aims["w_aim"].to_numpy(np.float64)
    if len(ak) > 1 and not (ak[1:] >= ak[:-1]).all():     # sort only if not already sorted
        order = np.argsort(aim_key, kind="stable")
        ak, av = ak[order], av[order]
    key = mi * 10_000_000 + ids_all
    p = np.clip(np.searchsorted(ak, key), 0, max(len(ak) - 1, 0))
    w_aim = np.where((len(ak) > 0) & (ak[p] == key), av[p], np.nan) if len(ak) else \
        np.full(len(key), np.nan)
    # row r of month t+1 -> row of the same id in month t (keys (t, id) are sorted)
    tk = trow * 10_000_000 + ids_all
    nxt = np.full(len(data), -1, np.int64)
    later = trow >= 1
    if later.any() and len(tk):
        qk = (trow[later] - 1) * 10_000_000 + ids_all[later]
        q = np.clip(np.searchsorted(tk, qk), 0, len(tk) - 1)
        hit = tk[q] == qk
        nxt[later] = np.where(hit, q - starts[trow[later] - 1], -1)
    return dict(data=data, months=months, starts=starts, stops=stops, ids=ids_all,
                w_aim=w_aim, nxt=nxt, trow=trow, mu=_month_values(wealth, "mu_ld1", months))


def _same_device(a: torch.device, b) -> bool:
    b = torch.device(b)
    return a.type == b.type and (b.index is None or a.index == b.index)


def m_cache_positions(m_cache: dict | None, months: np.ndarray, ns: np.ndarray, ids: list,
                      N: int, dev) -> torch.Tensor | None:
    """Rows of S4's kept m_tilde (PfmlInputs.m_keep) for S9's months, or None when the cache
    cannot stand in for S9's own m_func: a month missing, a different device or width, or a
    different universe (row count, or the ids and their order, month by month - a count match
    alone could pair another universe's m_t with this month's rows)."""
    if m_cache is None or not len(months):
        return None
    cm_ = np.asarray(m_cache["months"], np.int64)
    if not len(cm_):
        return None
    p_ = np.searchsorted(cm_, months)
    ok = (bool(np.all(p_ < len(cm_)))
          and bool(np.all(cm_[np.minimum(p_, len(cm_) - 1)] == months))
          and m_cache["mt"].shape[-1] >= N and _same_device(m_cache["mt"].device, dev))
    if not ok or not np.array_equal(np.asarray(m_cache["n"])[p_], ns):
        return None
    cids = m_cache.get("ids")
    if cids is None or not all(np.array_equal(cids[int(p)], np.asarray(i, np.int64))
                               for p, i in zip(p_, ids)):
        return None
    return torch.as_tensor(p_, device=m_cache["mt"].device)


def pfml_weights(cfg: Config, chars: pd.DataFrame, barra: BarraCov, wealth: pd.DataFrame,
                 risk_free: pd.DataFrame, aims: pd.DataFrame, oos_months: np.ndarray,
                 device, mine_months: np.ndarray | None = None,
                 m_cache: dict | None = None, n_pad: int = 0) -> pd.DataFrame | None:
    """Weight recursion (17) (PFML_best_hps.py:168-218) -> weights.csv frame (rank 0).

    Each rank takes the OOS months it owns (``mine_months``: the S4 month ownership of
    search.owned_month_rows - contiguous in time, ranks in time order; default a contiguous
    split) and needs m_t of them: from ``m_cache`` (S4's m_tilde and a of exactly these
    months, PfmlInputs.m_keep - the reference recomputes the same m_t here,
    PFML_best_hps.py:185-190) or else as batched device m_func (K19; m = diag(a) m_tilde
    diag(1/a), never formed).  It then runs its part of the sequential chain on the device -
    w_opt = w_aim + m (w_start - w_aim), the drift w_start(t+1) = w_opt (1 + tr_ld1) /
    (1 + mu_ld1) gathered through the id map, new names 0 - with no host round trip per month.
    The chain crosses ranks as ONE N-vector hand-off (point-to-point, rank r -> r+1); the
    per-row weights are gathered at the end."""
    from ..ops.ridge import _HostClock
    from ..parallel import collectives as coll
    from ..parallel.dist import env as dist_env
    th = _HostClock()
    env = dist_env()
    dev = torch.device(device)
    pf = cfg.pf_set
    gamma, mu = float(pf["gamma_rel"]), float(pf["mu"])
    tc_on = bool(cfg.settings["Transaction_Costs"])
    pl = _weights_plan(cfg, chars, wealth, aims, oos_months)
    th("s9.plan")
    data, months, starts, stops = pl["data"], pl["months"], pl["starts"], pl["stops"]
    B = len(months)
    ns = stops - starts
    # n_pad: S4's padded universe width (pfml_inputs.universe_npad) - a recomputed m_t then
    # has S4's shapes and is bitwise the cached one
    N = max(int(ns.max()) if B else 1, int(n_pad))
    K = barra.X.shape[1]
    wvals = _month_values(wealth, "wealth", months)
    rfvals = _month_values(risk_free, "rf", months)
    if mine_months is not None:
        mine = np.nonzero(np.isin(months, np.asarray(mine_months, np.int64)))[0].astype(np.int64)
    else:
        mine = np.asarray(list(coll.contiguous_split(B, env.world_size, env.rank)), np.int64)
    f64 = dict(dtype=torch.float64, device=dev)
    lam_col = data["lambda"].to_numpy(np.float64) if tc_on else None
    tr1 = data["tr_ld1"].to_numpy(np.float64)
    ids_all = pl["ids"]
    trow = pl["trow"]
    # Barra rows keyed (month, id): one sorted key array for every exact lookup below
    bkey = np.repeat(barra.months.astype(np.int64), np.diff(barra.offsets)) * 10_000_000 + \
        barra.ids.astype(np.int64)

    def rows_of(tt: np.ndarray):
        """(rows, batch index, column) of every data row of the months ``tt`` (in order)."""
        n_t = ns[tt]
        bi = np.repeat(np.arange(len(tt)), n_t)
        col = np.arange(int(n_t.sum())) - np.repeat(np.cumsum(n_t) - n_t, n_t)
        return starts[tt][bi] + col, bi, col

    # ---- m_t of this rank's months: S4's (cache) or batched m_func (K19) --------------
    Bm = len(mine)
    kpos = m_cache_positions(m_cache, months[mine], ns[mine],
                             [ids_all[starts[t]:stops[t]] for t in mine], N, dev)
    if kpos is not None:
        mt_all = m_cache["mt"].index_select(0, kpos)[:, :N, :N]   # ld = the S4 width
        a_all = m_cache["a"].index_select(0, kpos)[:, :N].contiguous()
        chunk, Bm_run = 1, 0
        log.info(f"S9: m_t of {Bm} month(s) reused from S4")
    else:
        mt_all = torch.zeros((Bm, N, N), **f64)
        a_all = torch.ones((Bm, N), **f64)
        chunk = int(cfg.run.month_batch)
        if chunk <= 0:
            from .pfml_inputs import auto_month_batch
            chunk = auto_month_batch(N, 0, dev)
        Bm_run = Bm
    for c0 in range(0, Bm_run, chunk):
        cm = mine[c0:c0 + chunk]
        Bc = len(cm)
        rows, bi, col = rows_of(cm)
        pos = _exact_lookup(bkey, months[trow[rows]] * 10_000_000 + ids_all[rows],
                            "OOS ids missing from the Barra universe")
        Xl = np.zeros((Bc, N, K))
        iv = np.ones((Bc, N))
        mask = np.zeros((Bc, N))
        Xl[bi, col], iv[bi, col], mask[bi, col] = barra.X[pos], barra.ivol[pos], 1.0
        Fb = barra.F[_exact_lookup(barra.months.astype(np.int64), months[cm], "Barra month")]
        lam = np.repeat((gamma / wvals[cm])[:, None], N, axis=1)
        lam[bi, col] = lam_col[rows] if tc_on else 1e-16
        Xd, ivd = torch.as_tensor(Xl, **f64), torch.as_tensor(iv, **f64)
        Sig = torch.empty((Bc, N, N), **f64)
        XF = torch.empty((Bc, N, K), **f64)
        gemm_fused(Xd, torch.as_tensor(Fb, **f64), XF)          # in-house GEMM, no rocBLAS
        # (as in S4: the symmetric mode's exactly symmetric Sigma, so m_t is bitwise S4's)
        gemm_fused(XF, Xd, Sig, trans_b=True, diag_col0=0, diag_vec=ivd, sym=True)
        mt, a = la.m_tilde(Sig, torch.as_tensor(lam, **f64), torch.as_tensor(wvals[cm], **f64),
                           torch.as_tensor(rfvals[cm], **f64), mu, gamma, cfg.run.iterations,
                           mask=torch.as_tensor(mask, **f64), sigma_exact_sym=True)
        mt_all[c0:c0 + Bc] = mt
        a_all[c0:c0 + Bc] = a
    th("s9.m_t")

    # ---- the sequential chain on the device ---------------------------------------------
    rows, bi, col = rows_of(mine)

    def padded(vals: np.ndarray, fill: float) -> torch.Tensor:
        out = np.full((Bm, N), fill)
        out[bi, col] = vals[rows]
        return torch.as_tensor(out, **f64)

    wa = padded(pl["w_aim"], 0.0)
    grow = padded((1.0 + tr1), 1.0) / torch.as_tensor(1.0 + pl["mu"][mine], **f64).view(Bm, 1)
    nmap = np.zeros((Bm, N), np.int64)
    hit = np.zeros((Bm, N))
    has_next = np.nonzero(mine + 1 < B)[0]
    if len(has_next):
        r1, b1, c1 = rows_of(mine[has_next] + 1)
        q = pl["nxt"][r1]
        nmap[has_next[b1], c1] = np.maximum(q, 0)
        hit[has_next[b1], c1] = q >= 0
    nmap_t, hit_t = torch.as_tensor(nmap, device=dev), torch.as_tensor(hit, **f64)
    ws0 = torch.zeros(N, **f64)
    if env.is_dist:
        ws0 = coll.recv_prev(ws0)                 # rank 0: zeros; a rank owning no month
    if Bm and mine[0] == 0:                       # passes the vector on unchanged
        g0 = np.arange(starts[0], stops[0])
        me = data["me"].to_numpy(np.float64)[g0]
        ws0 = torch.zeros(N, **f64)
        ws0[: len(g0)] = torch.as_tensor(me / me.sum(), **f64)    # value-weighted start
    Wst = torch.zeros((Bm, N), **f64)
    Wopt = torch.zeros((Bm, N), **f64)
    ws = ws0
    if nat.is_device(mt_all) and N <= int(nat.hip_lib().pfml_weights_chain_max_n()):
        # one persistent-workgroup launch for the whole chain (csrc/weights.hip)
        ws = torch.empty(N, **f64)
        if Bm:
            nat.check(nat.hip_lib().pfml_weights_chain(
                mt_all.data_ptr(), mt_all.stride(1), mt_all.stride(0), a_all.data_ptr(),
                wa.data_ptr(),
                grow.contiguous().data_ptr(), nmap_t.data_ptr(), hit_t.data_ptr(), N,
                ws0.contiguous().data_ptr(), Bm, N, Wst.data_ptr(), Wopt.data_ptr(),
                ws.data_ptr(), nat.stream_of(mt_all)), "pfml_weights_chain")
        else:
            ws.copy_(ws0)
    else:
        for i in range(Bm):
            Wst[i] = ws
            d = (ws - wa[i]) / a_all[i]
            wopt = wa[i] + a_all[i] * torch.mv(mt_all[i], d)
            Wopt[i] = wopt
            ws = (wopt * grow[i])[nmap_t[i]] * hit_t[i]             # next month's w_start
    if env.is_dist:
        coll.send_next(ws)
    th("s9.chain")
    # gather the per-row weights (rank order = month order)
    sel = torch.as_tensor(np.arange(N)[None, :] < ns[mine][:, None], device=dev)
    w_start_rows = coll.all_gather_varlen(Wst[sel])
    w_rows = coll.all_gather_varlen(Wopt[sel])
    if not env.is_main:
        return None
    w_start = w_start_rows.cpu().numpy()
    w = w_rows.cpu().numpy()
    # rows with a missing aim stay NaN like the reference's merge would leave them
    nan_aim = np.isnan(pl["w_aim"])
    w = np.where(nan_aim, np.nan, w)
    out = pd.DataFrame({"eom": month_end(data["mi"].to_numpy()),
                        "mu_ld1": pl["mu"][trow],
                        "id": ids_all, "tr_ld1": tr1, "w_start": w_start, "w": w})
    th("s9.gather+frame")
    return out


def pf_ts(weights: pd.DataFrame, chars: pd.DataFrame, wealth: pd.DataFrame,
          compat: bool = True) -> pd.DataFrame:
    """Per-month portfolio statistics (PFML_best_hps.py:220-259)."""
    comb = chars[["id", "eom", "ret_ld1", "lambda"]].merge(weights, on=["id", "eom"], how="inner")
    comb = comb.merge(wealth[["eom", "wealth"]], on="eom", how="left")
    dw = comb["w"] - comb["w_start"]
    comb = comb.assign(absw=comb["w"].abs(), shortw=comb["w"].clip(upper=0).abs(),
                       to=dw.abs(), rr=comb["w"] * comb["ret_ld1"],
                       lam_dw2=comb["lambda"] * dw * dw)
    g = comb.groupby("eom")
    res = pd.DataFrame({"inv": g["absw"].sum(), "shorting": g["shortw"].sum(),
                        "turnover": g["to"].sum(), "r": g["rr"].sum(),
                        "tc": g["wealth"].first() / 2.0 * g["lam_dw2"].sum()}).reset_index()
    if compat:
        # quirk Q3: (eom + 1M).to_period('M').to_timestamp('M') - MonthEnd(1) == eom
        res["eom_ret"] = res["eom"]
    else:
        res["eom_ret"] = res["eom"] + pd.offsets.MonthEnd(1)
    return res.drop(columns=["eom"])


def pf_summary(pf: pd.DataFrame, gamma: float) -> pd.DataFrame:
    """Annualised summary (PFML_best_hps.py:326-358; ddof = 1, quirk Q18)."""
    r, tc = pf["r"], pf["tc"]
    sd = r.std(ddof=1)
    return pd.DataFrame([{
        "type": "Portfolio-ML", "n": int(r.count()), "inv": pf["inv"].mean(),
        "shorting": pf["shorting"].mean(), "turnover_notional": pf["turnover"].mean(),
        "r": r.mean() * 12, "sd": sd * np.sqrt(12), "sr_gross": r.mean() / sd * np.sqrt(12),
        "tc": tc.mean() * 12, "r_tc": (r - tc).mean() * 12,
        "sr": (r - tc).mean() / sd * np.sqrt(12),
        "obj": (r.mean() - 0.5 * r.var(ddof=1) * gamma - tc.mean()) * 12}])


@io._io_timed                                             # (figure files: stage I/O time)
def plots(pf: pd.DataFrame, best: pd.DataFrame, gamma: float, out_dir: str) -> list[str]:
    """Cumulative performance and chosen hyper-parameters (PFML_best_hps.py:281-291,361-422)."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        log.info("matplotlib not available: plots skipped")
        return []
    os.makedirs(out_dir, exist_ok=True)
    p = pf.sort_values("eom_ret").copy()
    p["e_var_adj"] = (p["r"] - p["r"].mean()) ** 2
    p["utility_t"] = p["r"] - p["tc"] - 0.5 * p["e_var_adj"] * gamma
    fig, ax = plt.subplots(1, 3, figsize=(14, 4))
    for a, (col, title) in zip(ax, [(p["r"].cumsum(), "Gross return"),
                                    ((p["r"] - p["tc"]).cumsum(), "Return net of TC"),
                                    (p["utility_t"].cumsum(), "Return net of TC and Risk")]):
        a.plot(pd.to_datetime(p["eom_ret"]), col)
        a.set_title(title)
    f1 = os.path.join(out_dir, "cumulative_performance.png")
    fig.savefig(f1, dpi=100)
    plt.close(fig)
    fig, ax = plt.subplots(3, 1, figsize=(8, 7), sharex=True)
    for a, c in zip(ax, ["p", "l", "g"]):
        a.plot(best["eom_ret"], best[c], "o-", alpha=0.6)
        a.set_ylabel(c)
    f2 = os.path.join(out_dir, "top_hyperparameters.png")
    fig.savefig(f2, dpi=100)
    plt.close(fig)
    return [f1, f2]
