#!/bin/bash
# CholeskyQR2 panel path: band/ridge GPU tests, band-mode timings for both panel QRs,
# headline bench, shard rehearsal (W = 8).
set -o pipefail
TAG=${1:-cqr}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "band or ridge" > $OUT/pytest_band.log 2>&1
rc=$?; tail -3 $OUT/pytest_band.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_band.log | head -20; exit $rc; fi
for q in cqr householder; do
  PFML_BAND_QR=$q timeout -k 10 200 python tools/bench_band.py 1,14,106 > $OUT/band_${q}.json 2> $OUT/band_${q}.err
  rc=$?; echo "$q: $(cat $OUT/band_${q}.json)"; if [ $rc -ne 0 ]; then tail -3 $OUT/band_${q}.err; exit $rc; fi
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench.err; exit $rc; fi
PFML_BAND_QR=householder timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench_hh.json 2> $OUT/bench_hh.err
rc=$?; cat $OUT/bench_hh.json; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_shard.py > $OUT/shard.json 2> $OUT/shard.err
rc=$?; cat $OUT/shard.json; tail -2 $OUT/shard.err
exit $rc
