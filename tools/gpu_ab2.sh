#!/bin/bash
# A/B of the headline bench: current kernels vs abtest/libpfml_hip_prev.so (alternating)
set -o pipefail
TAG=${1:-ab2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for v in cur alt cur2 alt2; do
  if [ "${v:0:3}" = "alt" ]; then export PFML_HIP_LIB=$ROOT/abtest/libpfml_hip_prev.so; else unset PFML_HIP_LIB; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit 1
  echo "$v $(python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print(d['ms_per_step'])")"
  timeout -k 10 200 python tools/bench_band.py 106 > $OUT/band_$v.json 2> $OUT/band_$v.err || exit 1
  echo "$v $(cat $OUT/band_$v.json)"
done
