"""Typed configuration with the reference's defaults and key names.

Mirrors ``get_settings()`` / ``pf_set`` (General_functions.py:26-109) and ``get_features()``
(General_functions.py:113-170) key-for-key, so a user of the reference finds the same knobs
under the same names, and adds the framework's own run options (compat mode, precision,
device / world size, synthetic panel dimensions, artifact directory).

Overrides use dotted keys, e.g. ``--set pf_ml.p_vec=[64,128]`` or a YAML file
(``yaml.safe_load`` only).
"""
from __future__ import annotations

import copy
import hashlib
import json
from dataclasses import dataclass, field, asdict
from typing import Any

import numpy as np
import pandas as pd

# ---------------------------------------------------------------------------------------
# Feature list (General_functions.py:113-170): 154 JKP characteristics, 39 excluded -> 115.
# ---------------------------------------------------------------------------------------
_ALL_FEATURES = (
    "age aliq_at aliq_mat ami_126d at_be at_gr1 at_me at_turnover be_gr1a be_me beta_60m "
    "beta_dimson_21d betabab_1260d betadown_252d bev_mev bidaskhl_21d capex_abn capx_gr1 "
    "capx_gr2 capx_gr3 cash_at chcsho_12m coa_gr1a col_gr1a cop_at cop_atl1 corr_1260d "
    "coskew_21d cowc_gr1a dbnetis_at debt_gr3 debt_me dgp_dsale div12m_me dolvol_126d "
    "dolvol_var_126d dsale_dinv dsale_drec dsale_dsga earnings_variability ebit_bev ebit_sale "
    "ebitda_mev emp_gr1 eq_dur eqnetis_at eqnpo_12m eqnpo_me eqpo_me f_score fcf_me fnl_gr1a "
    "gp_at gp_atl1 ival_me inv_gr1 inv_gr1a iskew_capm_21d iskew_ff3_21d iskew_hxz4_21d "
    "ivol_capm_21d ivol_capm_252d ivol_ff3_21d ivol_hxz4_21d kz_index lnoa_gr1a lti_gr1a "
    "market_equity mispricing_mgmt mispricing_perf ncoa_gr1a ncol_gr1a netdebt_me netis_at "
    "nfna_gr1a ni_ar1 ni_be ni_inc8q ni_ivol ni_me niq_at niq_at_chg1 niq_be niq_be_chg1 "
    "niq_su nncoa_gr1a noa_at noa_gr1a o_score oaccruals_at oaccruals_ni ocf_at ocf_at_chg1 "
    "ocf_me ocfq_saleq_std op_at op_atl1 ope_be ope_bel1 opex_at pi_nix ppeinv_gr1a prc "
    "prc_highprc_252d qmj qmj_growth qmj_prof qmj_safety rd_me rd_sale rd5_at resff3_12_1 "
    "resff3_6_1 ret_1_0 ret_12_1 ret_12_7 ret_3_1 ret_6_1 ret_60_12 ret_9_1 rmax1_21d "
    "rmax5_21d rmax5_rvol_21d rskew_21d rvol_21d sale_bev sale_emp_gr1 sale_gr1 sale_gr3 "
    "sale_me saleq_gr1 saleq_su seas_1_1an seas_1_1na seas_11_15an seas_11_15na seas_16_20an "
    "seas_16_20na seas_2_5an seas_2_5na seas_6_10an seas_6_10na sti_gr1a taccruals_at "
    "taccruals_ni tangibility tax_gr1a turnover_126d turnover_var_126d z_score "
    "zero_trades_126d zero_trades_21d zero_trades_252d rvol_252d"
).split()

_POOR_COVERAGE = set(
    "capex_abn capx_gr2 capx_gr3 debt_gr3 dgp_dsale dsale_dinv dsale_drec dsale_dsga "
    "earnings_variability eqnetis_at eqnpo_me eqpo_me f_score iskew_hxz4_21d ivol_hxz4_21d "
    "netis_at ni_ar1 ni_inc8q ni_ivol niq_at niq_at_chg1 niq_be niq_be_chg1 niq_su "
    "ocfq_saleq_std qmj qmj_growth rd_me rd_sale rd5_at resff3_12_1 resff3_6_1 sale_gr3 "
    "saleq_gr1 saleq_su seas_16_20an seas_16_20na sti_gr1a z_score".split()
)


def get_features(exclude_poor_coverage: bool = True) -> list[str]:
    """Characteristic names used as model inputs (General_functions.py:113-170)."""
    if exclude_poor_coverage:
        return [f for f in _ALL_FEATURES if f not in _POOR_COVERAGE]
    return list(_ALL_FEATURES)


def pfml_feat_fun(p: int) -> list[str]:
    """Reference signal names for ``p`` RFFs (General_functions.py:837-844): p+1 names."""
    half = p // 2
    return (["constant"] + [f"rff{i}_cos" for i in range(1, half + 1)]
            + [f"rff{i}_sin" for i in range(1, half + 1)])


# Internal feature order.  The engine stores signals as [constant, cos1, sin1, cos2, sin2, ...]
# so that the reference's column subset pfml_feat_fun(p) is the LEADING (p+1) block of every
# P_max x P_max matrix: nested hyper-parameters become nested leading principal submatrices.
def interleaved_order(p_max: int) -> np.ndarray:
    """Map: internal position k -> reference (feat_all) column index."""
    half = p_max // 2
    order = [0]
    for i in range(half):
        order.append(1 + i)          # rff{i+1}_cos in feat_all
        order.append(1 + half + i)   # rff{i+1}_sin in feat_all
    return np.asarray(order, dtype=np.int64)


def internal_feature_names(p_max: int) -> list[str]:
    ref = pfml_feat_fun(p_max)
    return [ref[j] for j in interleaved_order(p_max)]


# ---------------------------------------------------------------------------------------
# Settings
# ---------------------------------------------------------------------------------------
def _reference_settings() -> dict:
    """Defaults of General_functions.py:26-101 (same keys, same values)."""
    return {
        "parallel": True,
        "seed_no": 1,
        "months": False,
        "Transaction_Costs": True,
        "split": {
            "train_end": pd.Timestamp("1970-12-31"),
            "test_end": pd.Timestamp("2023-12-31"),
            "val_years": 10,
            "model_update_freq": "yearly",
            "train_lookback": 1000,
            "retrain_lookback": 1000,
        },
        "feat_prank": True,
        "ret_impute": "zero",
        "feat_impute": True,
        "addition_n": 12,
        "deletion_n": 12,
        "screens": {
            "start": pd.Timestamp("1952-01-31"),
            "end": pd.Timestamp("2023-12-31"),
            "feat_pct": 0.5,
            "nyse_stocks": False,
            "size_screen": "all",   # Prepare_Data.py:449 hard-sets this
        },
        "pi": 0.1,
        "rff": {
            "p_vec": [2 ** i for i in range(1, 10)],
            "g_vec": list(np.exp(np.arange(-3, -1))),
            "l_vec": [0.0] + list(np.exp(np.linspace(-10, 10, 100))),
        },
        "pf": {
            "dates": {"start_year": 1971, "end_yr": 2023, "split_years": 10},
            "hps": {
                "cov_type": "cov_add",
                "m1": {"k": [1, 2, 3], "u": [0.25, 0.5, 1], "g": [0, 1, 2], "K": 12},
                "static": {"k": [1.0, 1 / 3, 1 / 5], "u": [0.25, 0.5, 1], "g": [0, 1, 2]},
            },
        },
        "pf_ml": {
            "g_vec": list(np.exp(np.arange(-3, -1))),
            "p_vec": [2 ** i for i in range(6, 10)],
            "l_vec": [0.0] + list(np.exp(np.linspace(-10, 10, 100))),
            "orig_feat": False,
            "scale": True,
        },
        "ef": {"wealth": [1, 1e9, 1e10, 1e11], "gamma_rel": [1, 5, 10, 20, 100]},
        "cov_set": {
            "industries": True,
            "obs": 252 * 10,
            "hl_cor": int(252 * 3 / 2),
            "hl_var": int(252 / 2),
            "hl_stock_var": int(252 / 2),
            "min_stock_obs": 252,
            "initial_var_obs": 21 * 3,
        },
        "factor_ml": {"n_pfs": 10},
    }


def _reference_pf_set() -> dict:
    """``pf_set`` of General_functions.py:103-108."""
    return {"wealth": 1e10, "gamma_rel": 10, "mu": 0.007, "lb_hor": 11}


@dataclass
class RunOptions:
    """Framework options that have no reference counterpart."""
    # compat_mode=True reproduces the reference quirks: Q1 (g ignored when the
    # RFF weight matrix is supplied), Q2 (validation rows accumulate across g), Q3
    # (pf.csv eom_ret == eom).  False gives the corrected behaviour.
    # Intentional deviation in both modes (Q19): a Barra factor with zero variance over the
    # EWMA window (no stock exposed to it, e.g. an empty FF12 industry) gets correlation 0,
    # where the reference's weighted_cor_wt (General_functions.py:827, cov / outer(sd, sd))
    # gives 0/0 = NaN when the variance is exactly 0 - which would make F, and through
    # X F X' every Sigma_t of that month, NaN.  (In practice the reference's pinv fallback
    # leaves ~1e-16 coefficient noise there, so its variance is ~1e-32, not 0, and its F
    # entries ~1e-32: the engine's exact 0 differs from that by far below every tolerance.)
    # Outputs differ only where the reference's would be NaN.
    compat_mode: bool = True
    # fp64 (production) | fp32 | bf16 | fp8: the S4 covariance (K1), RFF (K13) and risk GEMMs
    # in reduced precision (fp32 sgemm, or bf16 / fp8 MFMA with fp32 accumulation); solves
    # stay fp64 (bench --precision reports the error vs fp64)
    precision: str = "fp64"
    device: str = "auto"               # auto | cpu | cuda
    world_size: int = 1
    iterations: int = 10               # m_func fixed-point steps (hard-coded 10 in reference)
    month_batch: int = 0               # PFML months per batch (S4); 0 = sized to free memory
    data_dir: str = "Data"
    artifact_dir: str = "artifacts"
    check: bool = False                # compare device results against the CPU oracle
    profile: bool = False              # emit roctx ranges + stage timing JSONL
    plots: bool = True                 # the reference's figures as PNGs under <data_dir>/plots
    fault_inject: str = ""             # "pfml-input" / "pfml-search-coef": poison a month / a cell (tests recovery)
    synthetic: dict = field(default_factory=lambda: {
        "n_stocks": 500, "n_features": 115, "start": "1952-01-31", "end": "2023-12-31",
        "n_factors_cluster": 13, "seed": 0,
    })


class Settings(dict):
    """Nested settings dict with attribute access and dotted overrides."""

    def __getattr__(self, k):
        try:
            v = self[k]
        except KeyError as e:  # pragma: no cover - attribute protocol
            raise AttributeError(k) from e
        return Settings(v) if isinstance(v, dict) and not isinstance(v, Settings) else v

    def get_path(self, dotted: str):
        cur: Any = self
        for part in dotted.split("."):
            cur = cur[part]
        return cur

    def set_path(self, dotted: str, value) -> None:
        parts = dotted.split(".")
        cur = self
        for part in parts[:-1]:
            cur = cur.setdefault(part, {})
        cur[parts[-1]] = value


def get_settings() -> tuple[Settings, Settings]:
    """``(settings, pf_set)`` with the reference defaults."""
    return Settings(_reference_settings()), Settings(_reference_pf_set())


def _parse_value(text: str):
    import yaml
    v = yaml.safe_load(text)
    if isinstance(text, str) and len(text) >= 10 and text[4:5] == "-" and text[7:8] == "-":
        try:
            return pd.Timestamp(text)
        except ValueError:
            pass
    return v


@dataclass
class Config:
    settings: Settings
    pf_set: Settings
    run: RunOptions

    @classmethod
    def default(cls) -> "Config":
        s, p = get_settings()
        return cls(settings=s, pf_set=p, run=RunOptions())

    def override(self, assignments: list[str] | None = None, yaml_path: str | None = None) -> "Config":
        """Apply ``key=value`` overrides.  Keys are looked up in settings, pf_set, then run."""
        cfg = copy.deepcopy(self)
        items: list[tuple[str, Any]] = []
        if yaml_path:
            import yaml
            with open(yaml_path, encoding="utf-8") as f:
                doc = yaml.safe_load(f) or {}

            def walk(prefix, node):
                for k, v in node.items():
                    key = f"{prefix}.{k}" if prefix else k
                    if isinstance(v, dict) and key.split(".")[0] not in ("synthetic",) \
                            and not (key.startswith("run.synthetic")):
                        walk(key, v)
                    else:
                        items.append((key, v))
            walk("", doc)
        for a in assignments or []:
            k, _, v = a.partition("=")
            items.append((k.strip(), _parse_value(v.strip())))
        for key, val in items:
            head = key.split(".")[0]
            if head == "pf_set":
                cfg.pf_set.set_path(key[len("pf_set."):], val)
            elif head == "run":
                sub = key[len("run."):]
                if "." in sub:
                    top, rest = sub.split(".", 1)
                    getattr(cfg.run, top)[rest] = val
                else:
                    setattr(cfg.run, sub, val)
            elif head in cfg.pf_set:
                cfg.pf_set.set_path(key, val)
            elif hasattr(cfg.run, head) and head not in cfg.settings:
                setattr(cfg.run, head, val)
            else:
                cfg.settings.set_path(key, val)
        return cfg

    def to_jsonable(self) -> dict:
        def conv(o):
            if isinstance(o, dict):
                return {k: conv(v) for k, v in o.items()}
            if isinstance(o, (list, tuple)):
                return [conv(v) for v in o]
            if isinstance(o, pd.Timestamp):
                return o.isoformat()
            if isinstance(o, (np.floating, np.integer)):
                return o.item()
            return o
        return {"settings": conv(dict(self.settings)), "pf_set": conv(dict(self.pf_set)),
                "run": conv(asdict(self.run))}

    def hash(self, *sections: str) -> str:
        """Stable hash of (a subset of) the config, used to key stage artifacts."""
        doc = self.to_jsonable()
        if sections:
            doc = {s: doc["settings"].get(s, doc["pf_set"].get(s, doc["run"].get(s)))
                   for s in sections}
        blob = json.dumps(doc, sort_keys=True, default=str).encode()
        return hashlib.sha256(blob).hexdigest()[:16]

    # Convenience accessors used throughout the engine -------------------------------
    @property
    def g_vec(self) -> list[float]:
        return [float(g) for g in self.settings["pf_ml"]["g_vec"]]

    @property
    def p_vec(self) -> list[int]:
        return [int(p) for p in self.settings["pf_ml"]["p_vec"]]

    @property
    def l_vec(self) -> np.ndarray:
        return np.asarray(self.settings["pf_ml"]["l_vec"], dtype=np.float64)

    @property
    def p_max(self) -> int:
        return max(self.p_vec)

    @property
    def hp_years(self) -> np.ndarray:
        d = self.settings["pf"]["dates"]
        return np.arange(d["start_year"], d["end_yr"] + 1)
