"""Orchestrator: the reference's Main.py (exec of 8 scripts with shared globals) as a typed,
resumable stage graph.

Stages (CLI names) and the reference script each one replaces:

    get-additional-data  0_Get_Additional_Data.py   (manual in the reference; not in ``main``)
    sp500-subset         0_SP500_Subset.py          (manual in the reference; not in ``main``)
    prepare-data         Prepare_Data.py
    estimate-cov         Estimate Covariance Matrix.py
    pfml-input           PFML_Input_Data.py
    pfml-search-coef     PFML_Search_Coef.py
    pfml-hp-reals        PFML_hp_reals.py
    pfml-aim             PFML_aim_fun.py
    pfml-hps             PFML_hps.py
    pfml-best-hps        PFML_best_hps.py

State flows in memory within one process; with ``checkpoint=True`` every stage also writes
its artifact + done-marker (utils/artifacts.py) so a later run resumes from the first stage
whose inputs changed.  Multi-GPU (torchrun): pfml-input shards months and pfml-search-coef
shards hp years over ranks (RCCL), everything else runs on rank 0.
"""
from __future__ import annotations

import os
import time

import numpy as np
import pandas as pd
import torch

from .config import Config, get_features
from .data import acquire, io
from .models import portfolio, prep, risk
from .models import pfml_inputs as pin
from .models import search
from .parallel import collectives as coll
from .parallel import dist as pdist
from .utils.artifacts import ArtifactStore
from .utils.dates import month_index, pfml_date_grids
from .utils.log import COUNTERS, get_logger, metric
from .utils.trace import StageTimer

log = get_logger("pipeline")

MAIN_STAGES = ["prepare-data", "estimate-cov", "pfml-input", "pfml-search-coef",
               "pfml-hp-reals", "pfml-aim", "pfml-hps", "pfml-best-hps"]
ALL_STAGES = ["get-additional-data", "sp500-subset"] + MAIN_STAGES

# settings sections each stage's output depends on (for resume keys)
_DEPS = {
    "prepare-data": ("screens", "split", "feat_prank", "feat_impute", "addition_n", "deletion_n",
                     "pi", "pf"),
    "estimate-cov": ("cov_set",),
    "pfml-input": ("pf_ml", "Transaction_Costs", "seed_no"),
    "pfml-search-coef": ("pf_ml", "pf"),
    "pfml-hp-reals": ("pf_ml",),
    "pfml-aim": ("pf",),
    "pfml-hps": (),
    "pfml-best-hps": (),
}


class Pipeline:
    def __init__(self, cfg: Config, device: str | None = None, checkpoint: bool = False):
        self.cfg = cfg
        self.env = pdist.init(device or cfg.run.device)
        self.device = self.env.device
        self.checkpoint = checkpoint
        self.store = ArtifactStore(cfg.run.artifact_dir)
        self.state: dict = {}
        self.timer = StageTimer(self.device)
        self._keys = {}
        key = ""
        for st in ALL_STAGES:
            key = key + "|" + self.cfg.hash(*_DEPS.get(st, ())) + st
            self._keys[st] = key

    # ---------------------------------------------------------------------------------
    def run(self, stages: list[str] | None = None) -> dict:
        stages = stages or MAIN_STAGES
        for st in stages:
            if st not in ALL_STAGES:
                raise ValueError(f"unknown stage {st!r}; choose from {ALL_STAGES}")
        for st in stages:
            if self.checkpoint and self.store.is_done(st, self._keys[st]):
                log.info(f"[{st}] up to date (resume)")
                continue
            t0 = time.time()
            with self.timer(st):
                getattr(self, "_" + st.replace("-", "_"))()
            if self.checkpoint and self.env.is_main:
                self.store.mark_done(st, self._keys[st], seconds=time.time() - t0)
            pdist.barrier()
            metric(stage=st, seconds=round(time.time() - t0, 3), rank=self.env.rank,
                   world_size=self.env.world_size, fallbacks=COUNTERS.as_dict())
            log.info(f"[{st}] done in {time.time() - t0:.2f}s")
        return self.state

    # ---------------------------------------------------------------------------------
    def _get_additional_data(self):
        if self.env.is_main:
            acquire.get_additional_data(self.cfg)

    def _sp500_subset(self):
        if self.env.is_main:
            acquire.sp500_subset(self.cfg)

    def _prepare_data(self):
        if self.env.is_main:
            prep.prepare_data(self.cfg)

    def _estimate_cov(self):
        if self.env.is_main:
            dev = "cpu" if self.device.type == "cpu" else str(self.device)
            risk.estimate_cov(self.cfg, device=dev)

    def _load_common(self):
        if "chars" in self.state:
            return
        d = self.cfg.run.data_dir
        self.state["chars"] = io.read_processed_chars(d, get_features())
        self.state["barra"] = risk.BarraCov.load(os.path.join(d, "Barra_Cov.npz"))
        self.state["wealth"] = pd.read_csv(os.path.join(d, "wealth_processed.csv"),
                                           parse_dates=["eom"])
        self.state["risk_free"] = io.read_risk_free(d)
        b = self.state["barra"]
        s = self.cfg.settings
        self.state["grids"] = pfml_date_grids(int(b.months.min()), int(self.cfg.pf_set["lb_hor"]),
                                              s["split"]["test_end"],
                                              s["pf"]["dates"]["start_year"],
                                              s["pf"]["dates"]["split_years"])

    def _pfml_input(self):
        self._load_common()
        st = self.state
        m2 = st["grids"]["m2"]
        mine = np.asarray(list(coll.contiguous_split(len(m2), self.env.world_size,
                                                     self.env.rank)))
        months = m2[mine]
        res = pin.build_inputs(self.cfg, st["chars"], st["barra"], st["wealth"],
                               st["risk_free"], self.device, months=months)
        self._guard_inputs(res, months)
        R = res.reals
        G = R.G
        if self.env.is_dist:
            r_t = coll.all_gather_varlen(R.r_tilde.permute(1, 0, 2).contiguous()).permute(1, 0, 2)
            d_t = coll.all_gather_varlen(R.denom.permute(1, 0, 2, 3).contiguous()).permute(1, 0, 2, 3)
            R = search.PfmlReals(months=m2, r_tilde=r_t.contiguous(), denom=d_t.contiguous())
            sig = []
            for g in range(G):
                rows = torch.cat(res.signal_t[g]) if res.signal_t[g] else None
                sig.append(coll.all_gather_varlen(rows))
            counts = coll.all_gather_varlen(torch.as_tensor([len(x) for x in res.ids],
                                                            device=self.device)).cpu().numpy()
            ids_all = coll.all_gather_varlen(torch.as_tensor(np.concatenate(res.ids),
                                                             device=self.device)).cpu().numpy()
            offs = np.concatenate([[0], np.cumsum(counts)])
            signal_t = [[sig[g][offs[i]:offs[i + 1]] for i in range(len(m2))] for g in range(G)]
            ids = [ids_all[offs[i]:offs[i + 1]] for i in range(len(m2))]
        else:
            signal_t, ids = res.signal_t, res.ids
        st["reals"] = R
        st["signal_t"], st["signal_ids"], st["signal_months"] = signal_t, ids, m2
        st["rff_w"] = res.rff_w
        if self.checkpoint and self.env.is_main:
            payload = {"months": torch.as_tensor(R.months), "r_tilde": R.r_tilde,
                       "denom": R.denom, "rff_w": torch.as_tensor(res.rff_w),
                       "counts": torch.as_tensor([len(x) for x in ids]),
                       "ids": torch.as_tensor(np.concatenate(ids))}
            for g in range(G):
                payload[f"sig{g}"] = torch.cat(signal_t[g])
            self.store.save_tensors("pfml-input", "reals", payload)

    def _guard_inputs(self, res, months) -> None:
        """Failure detection: months whose summands are not finite are recomputed
        (once on the device, then on the fp64 CPU oracle).  ``run.fault_inject =
        "pfml-input"`` poisons the first month of every shard to exercise this path."""
        R = res.reals
        if self.cfg.run.fault_inject.startswith("pfml-input") and len(months):
            R.denom[:, 0, 0, 0] = float("nan")
            COUNTERS.add("fault_injected")
        bad = ~(torch.isfinite(R.denom).flatten(2).all(-1) & torch.isfinite(R.r_tilde).all(-1))
        bad_t = torch.nonzero(bad.any(0)).flatten().cpu().numpy()
        if len(bad_t) == 0:
            return
        st = self.state
        log.warning(f"non-finite PFML inputs in {len(bad_t)} month(s): recomputing")
        COUNTERS.add("pfml_input.recomputed_months", len(bad_t))
        for dev in (self.device, torch.device("cpu")):
            redo = pin.build_inputs(self.cfg, st["chars"], st["barra"], st["wealth"],
                                    st["risk_free"], dev, months=months[bad_t])
            ok = (torch.isfinite(redo.reals.denom).flatten(2).all(-1).all(0) &
                  torch.isfinite(redo.reals.r_tilde).all(-1).all(0))
            if bool(ok.all()):
                idx = torch.as_tensor(bad_t, device=R.denom.device)
                R.denom[:, idx] = redo.reals.denom.to(R.denom.device)
                R.r_tilde[:, idx] = redo.reals.r_tilde.to(R.r_tilde.device)
                return
        raise FloatingPointError(f"PFML inputs stay non-finite for months {months[bad_t]}")

    def _ensure_reals(self):
        if "reals" not in self.state:
            self._load_common()
            t = self.store.load_tensors("pfml-input", "reals", device=self.device)
            st = self.state
            st["reals"] = search.PfmlReals(months=t["months"].numpy(),
                                           r_tilde=t["r_tilde"], denom=t["denom"])
            counts = t["counts"].numpy()
            offs = np.concatenate([[0], np.cumsum(counts)])
            ids = t["ids"].numpy()
            G = st["reals"].G
            st["signal_t"] = [[t[f"sig{g}"][offs[i]:offs[i + 1]] for i in range(len(counts))]
                              for g in range(G)]
            st["signal_ids"] = [ids[offs[i]:offs[i + 1]] for i in range(len(counts))]
            st["signal_months"] = st["reals"].months
            st["rff_w"] = t["rff_w"].numpy()

    def _pfml_search_coef(self):
        self._ensure_reals()
        grid = search.grid_search(self.state["reals"], self.cfg)
        if self.cfg.run.check:
            metric(stage="pfml-search-coef", check=search.check_against_oracle(
                grid, self.state["reals"], self.cfg), rank=self.env.rank)
        years, beta = search.gather_beta(grid)
        self.state["grid"], self.state["beta_years"], self.state["beta"] = grid, years, beta
        if self.checkpoint and self.env.is_main:
            self.store.save_tensors("pfml-search-coef", "coef",
                                    {"years": torch.as_tensor(years), "beta": beta,
                                     "obj": grid.obj, "val_months": torch.as_tensor(grid.val_months),
                                     "val_year": torch.as_tensor(grid.val_year)})

    def _pfml_hp_reals_load(self):
        if "grid" not in self.state:
            t = self.store.load_tensors("pfml-search-coef", "coef", device=self.device)
            self.state["beta_years"], self.state["beta"] = t["years"].numpy(), t["beta"]
            self.state["grid"] = search.GridResult(
                years=self.cfg.hp_years, p_vec=self.cfg.p_vec, l_vec=self.cfg.l_vec,
                years_local=t["years"].numpy(), beta=t["beta"], val_months=t["val_months"].numpy(),
                val_year=t["val_year"].numpy(), obj=t["obj"])

    def _pfml_hp_reals(self):
        self._pfml_hp_reals_load()
        if self.env.is_main:
            val = search.validation_frame(self.state["grid"], self.cfg)
            io.write_csv(val, self.cfg.run.data_dir, "validation.csv")
            self.state["validation"] = val

    def _validation(self) -> pd.DataFrame:
        if "validation" not in self.state:
            self.state["validation"] = pd.read_csv(
                os.path.join(self.cfg.run.data_dir, "validation.csv"), parse_dates=["eom", "eom_ret"])
        return self.state["validation"]

    def _pfml_aim(self):
        if not self.env.is_main:
            return
        st = self.state
        self._load_common()
        if "signal_t" not in st:
            self._ensure_reals()
        if "beta" not in st:
            self._pfml_hp_reals_load()
        st["aims"] = portfolio.aim_portfolios(self.cfg, self._validation(), st["beta_years"],
                                              st["beta"], st["signal_months"], st["signal_t"],
                                              st["signal_ids"], st["grids"]["oos"])
        if self.checkpoint:
            rows, coefs = [], {}
            for g, per in st["aims"].items():
                for d, a in per.items():
                    rows.append(a["aim_pf"].assign(g=g, mi=d, p=a["p"], l=a["l"]))
                    coefs[f"c{g}_{d}"] = torch.as_tensor(a["coef"])
            pd.concat(rows).to_csv(self.store.path("pfml-aim", "aims.csv"), index=False)
            self.store.save_tensors("pfml-aim", "coef", coefs)

    def _load_aims(self):
        if "aims" in self.state:
            return
        df = pd.read_csv(self.store.path("pfml-aim", "aims.csv"), parse_dates=["eom"])
        coefs = self.store.load_tensors("pfml-aim", "coef")
        aims = {}
        for (g, d), sub in df.groupby(["g", "mi"], sort=True):
            aims.setdefault(int(g), {})[int(d)] = {
                "aim_pf": sub[["id", "eom", "w_aim"]].reset_index(drop=True),
                "coef": coefs[f"c{g}_{d}"].numpy(), "p": int(sub["p"].iloc[0]),
                "l": int(sub["l"].iloc[0])}
        self.state["aims"] = aims
        if "rff_w" not in self.state:
            t = self.store.load_tensors("pfml-input", "reals")
            self.state["rff_w"] = t["rff_w"].numpy()

    def _pfml_hps(self):
        if not self.env.is_main:
            return
        self._load_aims()
        self.state["hps"] = portfolio.hps_bundle(self.state["aims"], self._validation(),
                                                 self.state["rff_w"])
        if self.checkpoint:
            np.savez(self.store.path("pfml-hps", "rff_w.npz"), rff_w=self.state["rff_w"])

    def _pfml_best_hps(self):
        if not self.env.is_main:
            return
        st = self.state
        self._load_common()
        oos = st["grids"]["oos"]
        if "hps" not in st:
            self._pfml_hps()
        best, chosen, aims = portfolio.best_hps(st["hps"], oos)
        w = portfolio.pfml_weights(self.cfg, st["chars"], st["barra"], st["wealth"],
                                   st["risk_free"], aims, oos, self.device)
        d = self.cfg.run.data_dir
        io.write_csv(w, d, "weights.csv")
        pf = portfolio.pf_ts(w, st["chars"], st["wealth"], compat=self.cfg.run.compat_mode)
        io.write_csv(pf, d, "pf.csv")
        summ = portfolio.pf_summary(pf, float(self.cfg.pf_set["gamma_rel"]))
        io.write_csv(summ, d, "pf_summary.csv")
        st.update(best_hps=best, best_hps_list=chosen, weights=w, pf=pf, pf_summary=summ)
        if self.cfg.run.profile:
            portfolio.plots(pf, best, float(self.cfg.pf_set["gamma_rel"]),
                            os.path.join(d, "plots"))
        log.info("pf_summary:\n" + summ.to_string(index=False))
