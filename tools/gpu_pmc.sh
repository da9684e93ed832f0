#!/bin/bash
set -o pipefail
TAG=${1:-pmc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $OUT/p1 -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 > $OUT/p1.log 2>&1
rc=$?
cd $ROOT
python tools/pmc_summary.py $OUT/p1 --top 10 > $OUT/pmc1.txt 2>&1; cat $OUT/pmc1.txt
exit $rc
