#!/bin/bash
# A/B of the current kernel build against abtest/libpfml_hip_prev.so (PFML_HIP_LIB) on the
# headline step, alternating runs in one session; optional pytest -k filter first.
set -o pipefail
TAG=${1:-abprev}; KEXPR=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
if [ -n "$KEXPR" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > $OUT/pytest.log 2>&1
  rc=$?; tail -1 $OUT/pytest.log
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest.log | head; exit $rc; fi
fi
for i in 1 2 3; do
  for v in prev cur; do
    if [ $v = prev ]; then export PFML_HIP_LIB=$ROOT/abtest/libpfml_hip_prev.so; else unset PFML_HIP_LIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-inputs > $OUT/b_$v$i.json 2> $OUT/b_$v$i.err || exit 1
    echo "$v $(python -c "import json;print(json.load(open('$OUT/b_$v$i.json'))['ms_per_step'])")"
  done
done
unset PFML_HIP_LIB
