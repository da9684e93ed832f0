#!/bin/bash
# A/B of the quadform row tile (64 vs 128 rows per workgroup) on the headline step.
set -o pipefail
for r in 64 128 64 128; do
  PFML_QUAD_ROWS=$r timeout -k 10 120 python -u bench.py --no-inputs --steps 20 --warmup 3 > gpurun_out/qd_$r.log 2>&1 || exit 1
  echo "rows=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/qd_$r.log)"
done
