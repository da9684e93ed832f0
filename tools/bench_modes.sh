#!/bin/bash
# headline bench under the ridge-grid execution modes
set -o pipefail
TAG=${1:-modes}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for cfg in "multi 1" "multi 2" "single 2" "single 1"; do
  set -- $cfg
  PFML_BAND_MODE=$1 PFML_RIDGE_STREAMS=$2 timeout -k 10 120 python bench.py --steps 10 --warmup 2 > $OUT/bench_$1_$2.json 2> $OUT/bench_$1_$2.err
  rc=$?; echo "$cfg: $(python -c "import json,sys; print(json.load(open('$OUT/bench_$1_$2.json'))['ms_per_step'])")"
  if [ $rc -ne 0 ]; then tail -3 $OUT/bench_$1_$2.err; exit $rc; fi
done
