#!/bin/bash
# GPU tests (optionally a -k filter) + fp64 peak microbench + headline bench + rocprof of it.
# usage: tools/gpu_round.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r}; KEXPR=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$KEXPR" > $OUT/pytest_gpu.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
fi
rc=$?; tail -8 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|error" $OUT/pytest_gpu.log | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ -x tools/micro/mfma_f64_peak ]; then
  timeout -k 10 60 tools/micro/mfma_f64_peak > $OUT/mfma_f64_peak.json 2>&1
  rc=$?; cat $OUT/mfma_f64_peak.json
  if [ $rc -ne 0 ]; then echo "microbench rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err
if [ $rc -ne 0 ]; then echo "bench rc=$rc: stopping"; exit $rc; fi
PFML_HOST_TIMING=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 > $OUT/bench_host.json 2> $OUT/bench_host.err
rc=$?; if [ $rc -ne 0 ]; then echo "bench host rc=$rc: stopping"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 5 --warmup 1 > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 15 > $OUT/kernels.txt 2>&1
cat $OUT/kernels.txt
exit $rc
