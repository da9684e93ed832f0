#!/bin/bash
# A/B of PFML_* env switches on one GPU box: per arm the PFML_KTEST-selected GPU tests and the
# S4+S5+S6 bench (tools/gpu_run.sh ktest,s4b) under that arm's environment.
#   PFML_KTEST="m_tilde or db_sqrt" bash tools/gpu_ab.sh TAG "" "PFML_DB_SYM=0 PFML_DB_SYMPROD=0"
# Outputs gpurun_out/TAG_a<i>/.  Stops at the first failing arm.  AB_STEPS: other steps.
set -o pipefail
TAG=$1; shift
i=0
for arm in "$@"; do
  echo "== arm $i: ${arm:-default}"
  env $arm bash tools/gpu_run.sh ${TAG}_a$i ${AB_STEPS:-ktest,s4b} || exit $?
  i=$((i + 1))
done
