#!/bin/bash
# A/B of two builds of the HIP library on one GPU box: the GEMM shape table and the S4+S5+S6
# bench under each (PFML_HIP_LIB selects the library; arms alternate A B A B).
#   bash tools/gpu_ab_lib.sh TAG <lib A .so> <lib B .so> [shapes]
# Outputs gpurun_out/TAG/{A,B}{1,2}_shapes.log and the bench ms lines.
set -o pipefail
TAG=$1; LA=$2; LB=$3; SH=${4:-horner,inv_W,inv_S_sym,inv_X11_sym,inv_X12_mirror,db_prod}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for arm in A B; do
    lib=$LA; [ $arm = B ] && lib=$LB
    PFML_HIP_LIB=$lib PFML_DGEMM_CFGS=${PFML_DGEMM_CFGS:-7,8} PFML_DGEMM_SHAPES=$SH timeout -k 10 300 \
      python tools/micro/dgemm_shapes.py 5 > $OUT/${arm}${rep}_shapes.log 2>&1 || exit $?
    PFML_HIP_LIB=$lib timeout -k 10 600 python bench.py --with-inputs --steps 2 --warmup 1 \
      > $OUT/${arm}${rep}_s4.json 2> $OUT/${arm}${rep}_s4.err || { tail -3 $OUT/${arm}${rep}_s4.err; exit 1; }
    echo "$arm$rep $(grep -o '"ms_per_step": [0-9.]*' $OUT/${arm}${rep}_s4.json)"
  done
done
for f in $OUT/A1_shapes.log $OUT/B1_shapes.log $OUT/A2_shapes.log $OUT/B2_shapes.log; do
  echo "== $f"; grep -v "^{" $f | grep -v amdgpu.ids
done
