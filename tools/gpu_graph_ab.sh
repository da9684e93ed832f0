#!/bin/bash
# A/B: eager launches vs a captured HIP graph of the grid step.
set -o pipefail
for m in eager graph eager graph; do
  f="--no-graph"; [ "$m" = graph ] && f="--graph"
  timeout -k 10 120 python -u bench.py --no-inputs --steps 20 --warmup 3 $f > gpurun_out/g_$m.log 2>&1 || exit 1
  echo "$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/g_$m.log) $(grep -o '"hip_graph": [a-z]*' gpurun_out/g_$m.log) $(grep -o '"outputs_finite": [a-z]*' gpurun_out/g_$m.log)"
  grep "graph capture failed" gpurun_out/g_$m.log || true
done
