set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_quick.sh q12 || exit 1
cd /tmp && export TMPDIR=/tmp
for d in 1; do
  PFML_BAND_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/q12/p$d -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/q12/log$d.txt 2>&1 || exit 1
  python3 $R/tools/rocprof_summary.py $(find $R/gpurun_out/q12/p$d -name "*.db" | head -1) --top 6
done
