#!/bin/bash
# Strong-scaling rehearsal: per-rank step with the small cells on their own stream (one
# workgroup per cell) next to the multi-workgroup big cells, vs one stream.
set -o pipefail
timeout -k 10 300 python -u tools/bench_shard.py 4,8 5 > gpurun_out/sh1.log 2>&1 || exit 1
echo "streams=1 $(tail -1 gpurun_out/sh1.log)"
PFML_RIDGE_STREAMS=2 timeout -k 10 300 python -u tools/bench_shard.py 4,8 5 > gpurun_out/sh2.log 2>&1 || exit 1
echo "streams=2 $(tail -1 gpurun_out/sh2.log)"
