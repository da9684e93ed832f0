"""Command line: one sub-command per reference script, plus ``main`` (Main.py), synthetic data
generation and the headline benchmark.

    python -m pfml synth-data   --data-dir Data [--small] [--set run.synthetic.n_stocks=500]
    python -m pfml main         --data-dir Data [--device cuda] [--checkpoint] [--check]
    python -m pfml prepare-data | estimate-cov | pfml-input | pfml-search-coef | pfml-hp-reals
                   | pfml-aim | pfml-hps | pfml-best-hps | get-additional-data | sp500-subset
    python -m pfml stages a,b,c  (several stages in one process)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m pfml main ...   (RCCL, one rank/GPU)

Overrides: ``--set pf_ml.p_vec=[64,128]`` (dotted keys of get_settings()/pf_set/run options),
``--config file.yaml`` (yaml.safe_load).
"""
from __future__ import annotations

import argparse
import json
import sys

from .config import Config
from .pipeline import ALL_STAGES, MAIN_STAGES, Pipeline


def _cfg(a) -> Config:
    cfg = Config.default().override(a.set or [], yaml_path=a.config)
    if a.data_dir:
        cfg.run.data_dir = a.data_dir
    if a.artifact_dir:
        cfg.run.artifact_dir = a.artifact_dir
    if a.corrected:
        cfg.run.compat_mode = False
    if a.check:
        cfg.run.check = True
    if a.profile:
        cfg.run.profile = True
        from .utils import trace
        trace.enable(True)
    return cfg


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="pfml", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("command", help="main | stages | synth-data | " + " | ".join(ALL_STAGES))
    ap.add_argument("stages", nargs="?", default=None, help="comma list for `stages`")
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--artifact-dir", default=None)
    ap.add_argument("--device", default=None, help="auto | cpu | cuda")
    ap.add_argument("--set", action="append", help="dotted override key=value")
    ap.add_argument("--config", default=None, help="YAML overrides (safe_load)")
    ap.add_argument("--checkpoint", action="store_true", help="write artifacts + resume")
    ap.add_argument("--corrected", action="store_true", help="disable reference quirks Q1-Q3")
    ap.add_argument("--profile", action="store_true", help="roctx ranges + plots")
    ap.add_argument("--check", action="store_true",
                    help="compare sampled device results against the fp64 CPU oracle")
    ap.add_argument("--small", action="store_true", help="synth-data: 50-stock test panel")
    a = ap.parse_args(argv)
    cfg = _cfg(a)

    if a.command == "synth-data":
        from .data import synthetic as syn
        spec = syn.small_spec() if a.small else syn.SyntheticSpec(**{
            k: v for k, v in cfg.run.synthetic.items() if k in syn.SyntheticSpec.__dataclass_fields__})
        syn.write_raw(syn.generate(spec), cfg.run.data_dir)
        print(json.dumps({"data_dir": cfg.run.data_dir, "spec": spec.__dict__}))
        return 0
    if a.command == "main":
        stages = MAIN_STAGES
    elif a.command == "stages":
        stages = [s.strip() for s in (a.stages or "").split(",") if s.strip()]
    elif a.command in ALL_STAGES:
        stages = [a.command]
    else:
        ap.error(f"unknown command {a.command}")
        return 2
    pipe = Pipeline(cfg, device=a.device, checkpoint=a.checkpoint)
    pipe.run(stages)
    if pipe.env.is_main:
        print(json.dumps({"stages": stages, "seconds": pipe.timer.times}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
