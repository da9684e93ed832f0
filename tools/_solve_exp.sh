set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-q13}
mkdir -p $R/gpurun_out/$T
timeout -k 10 300 python $R/tools/debug_ridge.py 17 65 513 > $R/gpurun_out/$T/dbg.txt 2>&1 && DEBUG_INDEF=1 timeout -k 10 300 python $R/tools/debug_ridge.py 33 129 >> $R/gpurun_out/$T/dbg.txt 2>&1 && grep -v amdgpu $R/gpurun_out/$T/dbg.txt | grep "{" && bash $R/tools/gpu_quick.sh $T || exit 1
timeout -k 10 120 python $R/tools/bench_ridge.py --timing > $R/gpurun_out/$T/timing.txt 2>&1; python3 $R/tools/rocprof_timeline.py $(find $R/gpurun_out/$T/prof -name "*.db" | head -1) --last 60 > $R/gpurun_out/$T/timeline.txt
