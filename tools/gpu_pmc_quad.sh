#!/bin/bash
set -o pipefail
TAG=${1:-pmcq}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 $ROOT/tools/bench_quad.py > $OUT/p1.log 2>&1
rc=$?
cd $ROOT
python tools/pmc_summary.py $OUT/p1 --top 6 > $OUT/pmc1.txt 2>&1; cat $OUT/pmc1.txt
exit $rc
