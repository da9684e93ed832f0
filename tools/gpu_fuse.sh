#!/bin/bash
# Band-reduction kernel tests, then the strong-scaling rehearsal with the look-ahead
# multi-workgroup reduction on (default) and off (PFML_BAND_FUSE=0), then the 1-GPU bench.
set -o pipefail
TAG=${1:-fuse}; KEXPR=${2:-band or ridge}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "$KEXPR" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest.log | head -20; exit $rc; fi
PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py 1,2,4,8 > $OUT/shard_fuse.json 2> $OUT/shard_fuse.err
rc=$?; cat $OUT/shard_fuse.json; if [ $rc -ne 0 ]; then tail -3 $OUT/shard_fuse.err; exit $rc; fi
PFML_BAND_FUSE=0 PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py 2,4,8 > $OUT/shard_nofuse.json 2> $OUT/shard_nofuse.err
rc=$?; cat $OUT/shard_nofuse.json; if [ $rc -ne 0 ]; then tail -3 $OUT/shard_nofuse.err; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-inputs > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof8 -o run -- python3 $ROOT/tools/bench_shard.py 8 3 7 > $OUT/prof8.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_timeline.py $(find $OUT/prof8 -name "*.db" | head -1) --last 100 > $OUT/timeline8.txt 2>&1
exit $rc
