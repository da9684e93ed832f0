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
whose inputs changed.

Multi-GPU (torchrun, one rank per GPU, RCCL):
  * pfml-input / pfml-search-coef: the months are cut into canonical chunks (burn-in pieces
    and groups of hp years, search.win_layout) that ranks own whole; each rank builds the S4
    summands of ITS chunks (search.s4_compute_rows) and receives the one-block validation halo
    of its last year from the next rank by one all-gather (search.complete_local_reals) -
    every month's S4 runs once, the S4 months balance, and the expanding windows need one
    all-gather of P x P chunk totals (bitwise the 1-rank sums), the utilities one.  Both stages
    keep per-rank artifacts and per-rank done markers: a resumed run recomputes only the
    shards whose marker is missing or stale.
  * pfml-aim: each rank forms the aim portfolios of the OOS months whose signals its S4
    built, with the coefficients of every hp year (one all-gather of the betas); the aims
    (N doubles per month) are all-gathered.
  * pfml-best-hps: m_t of the OOS months sharded over ranks, the recursion chained across
    ranks by one N-vector hand-off (portfolio.pfml_weights); CSVs written by rank 0.
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
from .utils.dates import month_end, month_index, pfml_date_grids
from .utils.log import COUNTERS, get_logger, metric
from .utils.trace import StageTimer

log = get_logger("pipeline")

MAIN_STAGES = ["prepare-data", "estimate-cov", "pfml-input", "pfml-search-coef",
               "pfml-hp-reals", "pfml-aim", "pfml-hps", "pfml-best-hps"]
ALL_STAGES = ["get-additional-data", "sp500-subset"] + MAIN_STAGES

# settings sections (and run options) each stage's output depends on (for resume keys);
# keys chain, so a change invalidates the stage and everything downstream
_DEPS = {
    "prepare-data": ("screens", "split", "feat_prank", "feat_impute", "addition_n", "deletion_n",
                     "pi", "pf"),
    "estimate-cov": ("cov_set",),
    "pfml-input": ("pf_ml", "Transaction_Costs", "seed_no", "compat_mode", "precision",
                   "iterations"),
    "pfml-search-coef": ("pf_ml", "pf"),
    "pfml-hp-reals": ("pf_ml", "compat_mode"),
    "pfml-aim": ("pf",),
    "pfml-hps": (),
    "pfml-best-hps": ("compat_mode", "iterations"),
}
# stages whose artifacts are per rank (resume per shard)
_SHARDED = ("pfml-input", "pfml-search-coef")
# per-rank artifact payload versions (part of the done-marker key)
_FORMAT = {"pfml-input": 2}


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
            if self.checkpoint and self._all_done(st):
                log.info(f"[{st}] up to date (resume)")
                continue
            t0 = time.time()
            io0 = io.IO_SECONDS[0]
            with self.timer(st):
                getattr(self, "_" + st.replace("-", "_"))()
            io_s = io.IO_SECONDS[0] - io0
            if self.checkpoint:
                if st in _SHARDED:
                    self.store.mark_done(st, self._rank_key(st), rank=self.env.rank,
                                         seconds=time.time() - t0)
                elif self.env.is_main:
                    self.store.mark_done(st, self._keys[st], seconds=time.time() - t0)
            pdist.barrier()
            metric(stage=st, seconds=round(time.time() - t0, 3), io_seconds=round(io_s, 3),
                   rank=self.env.rank, world_size=self.env.world_size,
                   fallbacks=COUNTERS.as_dict())
            log.info(f"[{st}] done in {time.time() - t0:.2f}s")
        return self.state

    def _rank_key(self, st: str) -> str:
        # payload format versions: a shard written by an older layout (pfml-input before
        # "signal_months" was stored) is stale and recomputed, never reinterpreted
        return f"{self._keys[st]}|w{self.env.world_size}|v{_FORMAT.get(st, 1)}"

    def _all_done(self, st: str) -> bool:
        """Resume decision, identical on every rank (stages contain collectives)."""
        if st in _SHARDED:
            mine = self.store.is_done(st, self._rank_key(st), rank=self.env.rank)
        else:
            mine = self.store.is_done(st, self._keys[st])
        return coll.all_reduce_max(0.0 if mine else 1.0, device=self.device) == 0.0

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
        # the months this rank's S4 computes (it owns them); its validation halo comes from
        # the next rank below (search.complete_local_reals)
        months = m2[search.s4_compute_rows(m2, self.cfg.hp_years, self.env.world_size,
                                           self.env.rank)]
        if self.checkpoint and self.store.is_done("pfml-input", self._rank_key("pfml-input"),
                                                  rank=self.env.rank):
            log.info(f"[pfml-input] rank {self.env.rank}: shard up to date (resume)")
            self._ensure_reals()
            if self.env.world_size > 1:
                # another rank's shard is being recomputed (else the stage would have been
                # skipped): its halo exchange is a collective, so this rank joins it with the
                # rows it computed, taken from its loaded local rows
                R = st["reals"]
                pos = torch.as_tensor(np.searchsorted(R.months, months), device=R.denom.device)
                st["reals"] = search.complete_local_reals(
                    R.r_tilde.index_select(1, pos), R.denom.index_select(1, pos), m2,
                    self.cfg.hp_years)
            return
        # S9 reuses S4's m_tilde of the OOS months this rank owns (PFML_best_hps.py:185-190
        # recomputes exactly these m_t)
        own_oos = self._owned_oos()
        keep = None if own_oos is None else np.intersect1d(own_oos, months)
        res = pin.build_inputs(self.cfg, st["chars"], st["barra"], st["wealth"],
                               st["risk_free"], self.device, months=months, keep_m=keep)
        self._guard_inputs(res, months)
        st["m_oos"] = res.m_keep
        R = search.complete_local_reals(res.reals.r_tilde, res.reals.denom, m2,
                                        self.cfg.hp_years)
        st["reals"] = R
        st["signal_t"], st["signal_ids"], st["signal_months"] = res.signal_t, res.ids, months
        st["rff_w"] = res.rff_w
        if self.checkpoint:
            payload = {"months": torch.as_tensor(R.months), "all_months": torch.as_tensor(m2),
                       "signal_months": torch.as_tensor(months),
                       "r_tilde": R.r_tilde, "denom": R.denom,
                       "rff_w": torch.as_tensor(res.rff_w),
                       "counts": torch.as_tensor([len(x) for x in res.ids]),
                       "ids": torch.as_tensor(np.concatenate(res.ids) if res.ids else
                                              np.zeros(0, np.int64))}
            for g in range(R.G):
                payload[f"sig{g}"] = (torch.cat(res.signal_t[g]) if res.signal_t[g] else
                                      torch.zeros((0, R.P), dtype=torch.float64))
            self.store.save_tensors("pfml-input", f"reals.rank{self.env.rank}", payload)

    def _owned_oos(self) -> np.ndarray | None:
        """OOS months this rank owns (search.owned_month_rows): S9's shard of the chain.  None
        (S9 falls back to a contiguous split and recomputes m_t) if the owners of the OOS
        months are not non-decreasing in time - the chain runs rank after rank."""
        g = self.state["grids"]
        m2, oos = g["m2"], g["oos"]
        W = self.env.world_size
        owner = np.full(len(oos), -1, np.int64)
        for r in range(W):
            own = m2[search.owned_month_rows(m2, self.cfg.hp_years, W, r)]
            owner[np.isin(oos, own)] = r
        if (owner < 0).any() or (np.diff(owner) < 0).any():
            return None
        return oos[owner == self.env.rank]

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
            t = self.store.load_tensors("pfml-input", f"reals.rank{self.env.rank}",
                                        device=self.device)
            st = self.state
            st["reals"] = search.PfmlReals(months=t["months"].numpy(), r_tilde=t["r_tilde"],
                                           denom=t["denom"], all_months=t["all_months"].numpy())
            counts = t["counts"].numpy()
            offs = np.concatenate([[0], np.cumsum(counts)])
            ids = t["ids"].numpy()
            G = st["reals"].G
            st["signal_t"] = [[t[f"sig{g}"][offs[i]:offs[i + 1]] for i in range(len(counts))]
                              for g in range(G)]
            st["signal_ids"] = [ids[offs[i]:offs[i + 1]] for i in range(len(counts))]
            st["signal_months"] = (t["signal_months"].numpy() if "signal_months" in t
                                   else st["reals"].months)
            st["rff_w"] = t["rff_w"].numpy()

    def _guard_grid(self, grid) -> None:
        """Failure detection for S5, run on every rank BEFORE the utilities are
        gathered: (g, year, p) cells whose coefficients are not finite after the device repair
        are re-solved with the fp64 CPU oracle on the rank's own window sums, and their
        validation utilities recomputed, so the gathered frame - and every rank's choice of
        hyper-parameters - is built from repaired rows.  Whether a cell stayed singular is
        decided collectively (one max all-reduce) so that no rank raises alone while its
        peers wait in the gather.  ``run.fault_inject = "pfml-search-coef"`` poisons one cell
        of every shard to exercise this path."""
        if self.cfg.run.fault_inject.startswith("pfml-search-coef") and grid.beta.shape[1]:
            grid.beta[0, 0, -1, len(grid.l_vec) // 2, 0] = float("nan")
            COUNTERS.add("fault_injected")
        if grid.beta.is_cuda:
            from .ops.ridge import coop_errors
            nto = coop_errors()          # cooperative hand-off timeouts: those cells are NaN
            if nto:
                COUNTERS.add("ridge.coop_timeouts", nto)
                log.warning(f"{nto} cell(s) of the cooperative band reduction timed out on rank "
                            f"{self.env.rank}: their NaN betas are recomputed below")
        bad = search.nonfinite_cells(grid)
        res = {"recomputed": 0, "singular": 0}
        if bad:
            log.warning(f"non-finite coefficients in {len(bad)} cell(s) on rank "
                        f"{self.env.rank}: recomputing on the CPU oracle")
            res = search.recompute_cells(grid, self.state["reals"], bad)
            COUNTERS.add("pfml_search.recomputed_cells", res["recomputed"])
        singular = coll.all_reduce_max(float(res["singular"]), device=self.device)
        if singular:
            COUNTERS.add("pfml_search.singular_cells", res["singular"])
            log.warning(f"{res['singular']} cell(s) on rank {self.env.rank} singular even for "
                        "pivoted LU: NaN kept (never ranked; the reference raises here)")

    def _pfml_search_coef(self):
        self._ensure_reals()
        grid = search.grid_search(self.state["reals"], self.cfg, gather=False)
        self._guard_grid(grid)
        grid = search.gather_grid(grid)
        if self.cfg.run.check:
            metric(stage="pfml-search-coef", check=search.check_against_oracle(
                grid, self.state["reals"], self.cfg), rank=self.env.rank)
        # betas stay sharded: rank r holds the coefficients of its own hp years
        self.state["grid"] = grid
        self.state["beta_years"], self.state["beta"] = grid.years_local, grid.beta
        if self.checkpoint:
            self.store.save_tensors("pfml-search-coef", f"coef.rank{self.env.rank}",
                                    {"years": torch.as_tensor(grid.years_local),
                                     "beta": grid.beta, "obj": grid.obj,
                                     "val_months": torch.as_tensor(grid.val_months),
                                     "val_year": torch.as_tensor(grid.val_year)})

    def _pfml_hp_reals_load(self):
        if "grid" not in self.state:
            t = self.store.load_tensors("pfml-search-coef", f"coef.rank{self.env.rank}",
                                        device=self.device)
            self.state["beta_years"], self.state["beta"] = t["years"].numpy(), t["beta"]
            self.state["grid"] = search.GridResult(
                years=self.cfg.hp_years, p_vec=self.cfg.p_vec, l_vec=self.cfg.l_vec,
                years_local=t["years"].numpy(), beta=t["beta"], val_months=t["val_months"].numpy(),
                val_year=t["val_year"].numpy(), obj=t["obj"])

    def _pfml_hp_reals(self):
        self._pfml_hp_reals_load()
        # every rank holds the gathered utilities: each builds the (deterministic) frame it
        # needs for the aim selection, rank 0 writes validation.csv
        val = search.validation_frame(self.state["grid"], self.cfg)
        if self.env.is_main:
            io.write_csv(val, self.cfg.run.data_dir, "validation.csv")
        self.state["validation"] = val

    def _validation(self) -> pd.DataFrame:
        if "validation" not in self.state:
            self.state["validation"] = pd.read_csv(
                os.path.join(self.cfg.run.data_dir, "validation.csv"), parse_dates=["eom", "eom_ret"])
        return self.state["validation"]

    def _pfml_aim(self):
        st = self.state
        self._load_common()
        if "signal_t" not in st:
            self._ensure_reals()
        if "beta" not in st:
            self._pfml_hp_reals_load()
        # the OOS months whose signals this rank's S4 built (the months it owns), with the
        # coefficients of their year (oos_year, quirk Q13) from any rank: one all-gather of the
        # per-year betas (the signals of a month stay where S4 computed them)
        years_b, beta_b = search.gather_beta(st["grid"])
        oos = st["grids"]["oos"]
        oos_year = month_end(oos + 1).year.to_numpy()
        mine = oos[np.isin(oos_year, np.asarray(years_b)) &
                   np.isin(oos, np.asarray(st["signal_months"]))]
        local = portfolio.aim_portfolios(self.cfg, self._validation(), years_b, beta_b,
                                         st["signal_months"], st["signal_t"],
                                         st["signal_ids"], mine)
        st["aims"] = portfolio.gather_aims(local, self.cfg, self.device)
        if self.checkpoint and self.env.is_main:
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
            t = self.store.load_tensors("pfml-input", f"reals.rank{self.env.rank}")
            self.state["rff_w"] = t["rff_w"].numpy()

    def _pfml_hps(self):
        self._load_aims()
        self.state["hps"] = portfolio.hps_bundle(self.state["aims"], self._validation(),
                                                 self.state["rff_w"])
        if self.checkpoint and self.env.is_main:
            np.savez(self.store.path("pfml-hps", "rff_w.npz"), rff_w=self.state["rff_w"])

    def _pfml_best_hps(self):
        st = self.state
        self._load_common()
        oos = st["grids"]["oos"]
        if "hps" not in st:
            self._pfml_hps()
        best, chosen, aims = portfolio.best_hps(st["hps"], oos)
        # m_t sharded over ranks, the recursion chained across them (rank 0 gets the frame)
        npad = pin.universe_npad(st["chars"], st["grids"]["m2"])
        w = portfolio.pfml_weights(self.cfg, st["chars"], st["barra"], st["wealth"],
                                   st["risk_free"], aims, oos, self.device,
                                   mine_months=self._owned_oos(), m_cache=st.get("m_oos"),
                                   n_pad=npad)
        # failure detection: the chained w_start is finite by construction (value
        # weights, drift, 0 for new names); a non-finite one means a fault in the device chain
        # -> the recursion is recomputed on the CPU (a collective decision: every rank reruns)
        bad = 0
        if self.env.is_main:
            if self.cfg.run.fault_inject.startswith("pfml-best-hps") and len(w):
                w.loc[w.index[len(w) // 2], "w_start"] = float("nan")
                COUNTERS.add("fault_injected")
            bad = int((~np.isfinite(w["w_start"].to_numpy())).sum())
        bad = coll.broadcast_object(bad) if self.env.is_dist else bad
        if bad:
            log.warning(f"non-finite w_start in {bad} row(s): weight recursion recomputed on "
                        "the CPU")
            COUNTERS.add("pfml_best_hps.recomputed", 1)
            w = portfolio.pfml_weights(self.cfg, st["chars"], st["barra"], st["wealth"],
                                       st["risk_free"], aims, oos, torch.device("cpu"),
                                       mine_months=self._owned_oos(), n_pad=npad)
            if self.env.is_main and not np.isfinite(w["w_start"].to_numpy()).all():
                raise FloatingPointError("w_start stays non-finite on the CPU recursion")
        if not self.env.is_main:
            return
        d = self.cfg.run.data_dir
        io.write_csv(w, d, "weights.csv")
        pf = portfolio.pf_ts(w, st["chars"], st["wealth"], compat=self.cfg.run.compat_mode)
        io.write_csv(pf, d, "pf.csv")
        summ = portfolio.pf_summary(pf, float(self.cfg.pf_set["gamma_rel"]))
        io.write_csv(summ, d, "pf_summary.csv")
        st.update(best_hps=best, best_hps_list=chosen, weights=w, pf=pf, pf_summary=summ)
        if self.cfg.run.plots:
            portfolio.plots(pf, best, float(self.cfg.pf_set["gamma_rel"]),
                            os.path.join(d, "plots"))
        log.info("pf_summary:\n" + summ.to_string(index=False))
