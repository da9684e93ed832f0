#!/bin/bash
# pipelined per-g window sums under graph replay with more hardware queues per process
set -o pipefail
TAG=${1:-pipeq}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for q in 4 8; do
  for v in 0 1; do
    GPU_MAX_HW_QUEUES=$q PFML_PIPE_SUMS=$v timeout -k 10 300 python bench.py --no-inputs --steps 20 --warmup 3 > $OUT/bench_q${q}_p${v}.json 2> $OUT/bench_q${q}_p${v}.err
    rc=$?; echo "queues=$q pipe=$v: $(python -c "import json;d=json.load(open('$OUT/bench_q${q}_p${v}.json'));print(d['ms_per_step'], d['config'].get('hip_graph'))")"
    if [ $rc -ne 0 ]; then tail -5 $OUT/bench_q${q}_p${v}.err; exit $rc; fi
  done
done
