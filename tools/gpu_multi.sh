#!/bin/bash
set -o pipefail
TAG=${1:-multi}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest.log | head; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err; python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['ms_per_step'])"
timeout -k 10 400 python tools/bench_shard.py 1,2,4,8 > $OUT/shard.json 2> $OUT/shard.err; cat $OUT/shard.json
