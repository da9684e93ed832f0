#!/bin/bash
# rsq/rcp accuracy microbench + two PMC passes over one grid step (bench.py --no-inputs)
set -o pipefail
TAG=${1:-pmc2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
if [ -x tools/micro/rsq_acc ]; then
  timeout -k 10 60 tools/micro/rsq_acc > $OUT/rsq_acc.json 2>&1
  rc=$?; cat $OUT/rsq_acc.json; if [ $rc -ne 0 ]; then exit $rc; fi
fi
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/pA -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-inputs --no-graph > $OUT/pA.log 2>&1
rc=$?; if [ $rc -ne 0 ]; then tail -5 $OUT/pA.log; exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pB -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-inputs --no-graph > $OUT/pB.log 2>&1
rc=$?
cd $ROOT
python tools/pmc_summary.py $OUT/pA --top 14 > $OUT/pmcA.txt 2>&1; cat $OUT/pmcA.txt
python tools/pmc_summary.py $OUT/pB --top 14 > $OUT/pmcB.txt 2>&1; cat $OUT/pmcB.txt
exit $rc
