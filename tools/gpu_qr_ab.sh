#!/bin/bash
# A/B of the band-reduction panel QR (Householder default vs CholeskyQR2) on the headline step.
set -o pipefail
for q in householder cqr householder cqr; do
  PFML_BAND_QR=$q timeout -k 10 120 python -u bench.py --no-inputs --steps 20 --warmup 3 > gpurun_out/qr_$q.log 2>&1 || exit 1
  echo "qr=$q $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/qr_$q.log)"
done
