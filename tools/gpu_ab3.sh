#!/bin/bash
# Kernel tests, then A/B of an env-selected variant on the isolated kernel bench, the headline
# step and the shard rehearsal; kernel timeline of one step with the variant.
# usage: tools/gpu_ab3.sh TAG VAR=VALUE [pytest -k expr]
set -o pipefail
TAG=${1:-ab3}; VAR=${2:-PFML_QUAD_PF=1}; KEXPR=${3:-quad or ridge or band or grid}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$KEXPR" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest.log | head -20; exit $rc; fi
env $VAR timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > $OUT/pytest_var.log 2>&1
rc=$?; tail -2 $OUT/pytest_var.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest_var.log | head -20; exit $rc; fi
timeout -k 10 120 python tools/bench_quad.py > $OUT/quad_base.json 2>&1; rc=$?; cat $OUT/quad_base.json; [ $rc -ne 0 ] && exit $rc
env $VAR timeout -k 10 120 python tools/bench_quad.py > $OUT/quad_var.json 2>&1; rc=$?; cat $OUT/quad_var.json; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-inputs > $OUT/bench_base$i.json 2> $OUT/bench_base$i.err; rc=$?
  python -c "import json;d=json.load(open('$OUT/bench_base$i.json'));print('base',d['ms_per_step'])"; [ $rc -ne 0 ] && exit $rc
  env $VAR timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-inputs > $OUT/bench_var$i.json 2> $OUT/bench_var$i.err; rc=$?
  python -c "import json;d=json.load(open('$OUT/bench_var$i.json'));print('var',d['ms_per_step'])"; [ $rc -ne 0 ] && exit $rc
done
PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py 1,2,4,8 > $OUT/shard.json 2> $OUT/shard.err
rc=$?; cat $OUT/shard.json; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
env $VAR timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof1 -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-inputs > $OUT/prof1.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_timeline.py $(find $OUT/prof1 -name "*.db" | head -1) --last 32 > $OUT/timeline1.txt 2>&1
cat $OUT/timeline1.txt
exit $rc
