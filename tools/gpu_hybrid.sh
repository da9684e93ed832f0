#!/bin/bash
# A/B of PFML_BAND_HYBRID (big cells in the multi-workgroup reduction) on the headline step.
set -o pipefail
for k in 0 16 32 48; do
  PFML_BAND_HYBRID=$k timeout -k 10 120 python -u bench.py --no-inputs --steps 20 --warmup 3 > gpurun_out/hy_$k.log 2>&1 || exit 1
  echo "hybrid=$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hy_$k.log)"
done
