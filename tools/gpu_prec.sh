#!/bin/bash
set -o pipefail
TAG=${1:-prec}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lowp or dgemm or mfma" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; fi
for p in bf16 fp8; do
  timeout -k 10 600 python bench.py --with-inputs --steps 1 --warmup 1 --precision $p > $OUT/bench_s4_$p.json 2> $OUT/bench_s4_$p.err
  rc=$?; cat $OUT/bench_s4_$p.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench_s4_$p.err; exit $rc; fi
done
