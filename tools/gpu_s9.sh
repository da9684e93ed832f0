#!/bin/bash
# S9 GPU tests (golden pipeline on the device), then bench_s9 with per-section host timing.
set -o pipefail
TAG=${1:-s9}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or portfolio or weight" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest.log | head -20; exit $rc; fi
PFML_HOST_TIMING=sync timeout -k 10 300 python tools/bench_s9.py --steps 3 > $OUT/s9.txt 2>&1
rc=$?; grep -E "s9\.|metric" $OUT/s9.txt | tail -6; exit $rc
