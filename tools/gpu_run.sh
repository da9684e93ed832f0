#!/bin/bash
# GPU session driver (run through gpurun): bash tools/gpu_run.sh TAG step1,step2,...
# Every step writes under gpurun_out/TAG, runs under its own time limit and stops the chain on
# failure.  Steps:
#   suite      pytest -m gpu + smoke()          bench     headline bench (one JSON line)
#   timeline   kernel timeline of one grid step shard     one-GPU per-rank strong-scaling rehearsal
#   peak       fp64 MFMA / VALU roofline anchor dgemm     library vs in-house DGEMM rate
#   coop       cooperative band reduction: tests, per-phase timing, time vs #cells
#   cooptime   per-phase timing at K = 1 / 2       benchk    headline bench at auto K and K = 1
#   qr         panel-QR micro-benchmark        ktest     pytest -m gpu -k "$PFML_KTEST"
#   e2e        production-shape `main` end to end (synthetic raw data, S0 stages, 8 stages)
#   s4         S4+S5+S6 bench + S4 kernel stats stress    3000-stock S4 stress (BASELINE config 4)
#   s4roof     S4 roofline (kernel trace + work ledger)   dgemmpmc  in-house DGEMM TF/s + PMC
#   stressprof kernel stats of the stress    prec bf16 / fp8 S4 GEMMs (BASELINE config 5)  pmc     PMC counters of one grid step
#   shards4    per-rank S4 + grid step of W = 1 / 2 / 4 / 8 rank shards on this GPU
#   multiproc  2, 4 and 8 ranks sharing the GPU (gloo), utilities bitwise vs 1 rank
#   rccl1      RCCL collectives + segmented-capture check and the distributed bench at a forced world of one
#   segtl      kernel timeline of the segmented (multi-rank form) grid step under RCCL at world one
set -o pipefail
TAG=${1:-r03}
MODE=${2:-suite}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for step in ${MODE//,/ }; do
  case $step in
    peak)
      timeout -k 10 120 ./tools/micro/mfma_f64_peak > $OUT/mfma_peak.json 2>&1
      rc=$?; cat $OUT/mfma_peak.json; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    s4tile)
      # S4 with the 128 x 128 GEMM tile forced vs the auto choice (A / B / A)
      for tc in 0 1 0 1; do
        PFML_GEMM_TILE=$tc timeout -k 10 400 python bench.py --with-inputs --steps 1 --warmup 1 > $OUT/bench_s4_tile$tc.json 2> $OUT/bench_s4_tile$tc.err
        rc=$?; echo "tile $tc: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_s4_tile$tc.json)"
        if [ $rc -ne 0 ]; then tail -3 $OUT/bench_s4_tile$tc.err; exit $rc; fi
      done ;;
    rccl1)
      # RCCL itself on a one-GPU box: the collectives check and the bench's distributed path
      # (graph segments between RCCL collectives) as a forced world of one rank
      PFML_DIST_FORCE=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 tools/rccl_check.py > $OUT/rccl_check.log 2>&1
      rc=$?; grep '^{' $OUT/rccl_check.log; if [ $rc -ne 0 ]; then tail -20 $OUT/rccl_check.log; exit $rc; fi
      PFML_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29562 bench.py --no-inputs > $OUT/bench_rccl1.json 2> $OUT/bench_rccl1.err
      rc=$?; grep '^{' $OUT/bench_rccl1.json | cut -c1-200; grep -o '"dist_backend": "[a-z]*"\|"hip_graph": [a-z]*' $OUT/bench_rccl1.json; if [ $rc -ne 0 ]; then tail -5 $OUT/bench_rccl1.err; exit $rc; fi ;;
    s4cap)
      # S4 months per batch: the default cap (256) vs all 731 months in one batch (A / B / A / B)
      for cap in 256 1024 256 1024; do
        PFML_S4_BATCH_CAP=$cap timeout -k 10 400 python bench.py --with-inputs --steps 1 --warmup 1 > $OUT/bench_s4_cap$cap.json 2> $OUT/bench_s4_cap$cap.err
        rc=$?; echo "cap $cap: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_s4_cap$cap.json) $(grep -o 'months per batch[^"]*' $OUT/bench_s4_cap$cap.err | head -1)"
        if [ $rc -ne 0 ]; then tail -3 $OUT/bench_s4_cap$cap.err; exit $rc; fi
      done ;;
    gemm2)
      timeout -k 10 400 python tools/bench_gemm2.py > $OUT/gemm2.log 2>&1
      rc=$?; tail -1 $OUT/gemm2.log | cut -c1-3000; if [ $rc -ne 0 ]; then tail -5 $OUT/gemm2.log; exit $rc; fi ;;
    dgemm)
      timeout -k 10 200 python tools/micro/dgemm_rate.py > $OUT/dgemm_rate.json 2>&1
      rc=$?; tail -4 $OUT/dgemm_rate.json; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    s4roof)
      # S4 roofline: ONE eager S4 of all 731 months on one stream (per-kernel times do not
      # overlap; the work ledger counts the same launches) under a kernel trace
      (cd /tmp && export TMPDIR=/tmp PFML_S4_STREAMS=1 PFML_WORK_LEDGER=$OUT/work_ledger.json && timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/prof_s4r -o run -- python3 $ROOT/bench.py --s4-stress 731 --stocks 500 --warmup 0 > $OUT/prof_s4r.log 2>&1)
      rc=$?; tail -1 $OUT/prof_s4r.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -5 $OUT/prof_s4r.log; exit $rc; fi
      python tools/roofline_s4.py $(find $OUT/prof_s4r -name "*.db" | head -1) $OUT/work_ledger.json > $OUT/roofline_s4.md 2>&1
      rc=$?; cat $OUT/roofline_s4.md | head -30; python tools/rocprof_summary.py $(find $OUT/prof_s4r -name "*.db" | head -1) --top 40 > $OUT/kernels_s4r.txt 2>&1; rm -rf $OUT/prof_s4r; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    stressroof)
      # roofline of the 3000-stock stress: one eager S4 of 16 months on one stream
      (cd /tmp && export TMPDIR=/tmp PFML_S4_STREAMS=1 PFML_WORK_LEDGER=$OUT/work_ledger_stress.json && timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/prof_sr -o run -- python3 $ROOT/bench.py --s4-stress 16 --stocks 3000 --warmup 0 > $OUT/prof_sr.log 2>&1)
      rc=$?; tail -1 $OUT/prof_sr.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -5 $OUT/prof_sr.log; exit $rc; fi
      python tools/roofline_s4.py $(find $OUT/prof_sr -name "*.db" | head -1) $OUT/work_ledger_stress.json > $OUT/roofline_stress.md 2>&1
      rc=$?; head -40 $OUT/roofline_stress.md; python tools/rocprof_summary.py $(find $OUT/prof_sr -name "*.db" | head -1) --top 40 > $OUT/kernels_sr.txt 2>&1; rm -rf $OUT/prof_sr; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    dgemmpmc)
      # in-house DGEMM on the Horner shape / large squares: TF/s, then one PMC pass
      timeout -k 10 200 python tools/micro/dgemm_shapes.py 5 > $OUT/dgemm_shapes.log 2>&1
      rc=$?; tail -1 $OUT/dgemm_shapes.log; if [ $rc -ne 0 ]; then tail -5 $OUT/dgemm_shapes.log; exit $rc; fi
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/dgemm_pmc -o run -- python3 $ROOT/tools/micro/dgemm_shapes.py 2 > $OUT/dgemm_pmc.log 2>&1)
      rc=$?; python tools/pmc_summary.py $OUT/dgemm_pmc --top 8 > $OUT/dgemm_pmc.txt 2>&1; cat $OUT/dgemm_pmc.txt; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    invab)
      # SPD-inverse kernels: bitwise A/B against a saved build (lib_ab/old.so) + node latency
      PFML_HIP_LIB=$ROOT/lib_ab/old.so timeout -k 10 200 python tools/micro/inverse_ab.py save $OUT/inv_old.sha > $OUT/inv_old.json 2>&1
      rc=$?; tail -1 $OUT/inv_old.json | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi
      timeout -k 10 200 python tools/micro/inverse_ab.py save $OUT/inv_new.sha > $OUT/inv_new.json 2>&1
      rc=$?; tail -1 $OUT/inv_new.json | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi
      python tools/micro/inverse_ab.py cmp $OUT/inv_old.sha $OUT/inv_new.sha | tee $OUT/inv_cmp.json
      PFML_HIP_LIB=$ROOT/lib_ab/old.so timeout -k 10 200 python tools/micro/node_timing.py 36 715 > $OUT/node_timing_old.jsonl 2>&1
      rc=$?; grep '^{' $OUT/node_timing_old.jsonl | cut -c1-300; if [ $rc -ne 0 ]; then tail -3 $OUT/node_timing_old.jsonl; exit $rc; fi
      timeout -k 10 200 python tools/micro/node_timing.py 36 715 > $OUT/node_timing.jsonl 2>&1
      rc=$?; grep '^{' $OUT/node_timing.jsonl | cut -c1-300; if [ $rc -ne 0 ]; then tail -3 $OUT/node_timing.jsonl; exit $rc; fi ;;
    gemmtest)
      # GEMM / SPD-inverse kernel tests only (fast numerics check of a kernel change)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "gemm or spd_inverse or mfma" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gemm.log 2>&1
      rc=$?; tail -2 $OUT/pytest_gemm.log
      if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_gemm.log | head -20; exit $rc; fi ;;
    gemmclk)
      # Horner / DB-product GEMMs: effective clock and MFMA-pipe busy (one PMC pass)
      (cd /tmp && export TMPDIR=/tmp && PFML_DGEMM_SHAPES=${PFML_DGEMM_SHAPES:-horner,db_prod} PFML_DGEMM_CFGS=${PFML_DGEMM_CFGS:-3,8} timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/gemmclk -o run -- python3 $ROOT/tools/micro/dgemm_shapes.py 3 > $OUT/gemmclk.log 2>&1)
      rc=$?; python tools/pmc_summary.py $OUT/gemmclk --top 8 > $OUT/gemmclk.txt 2>&1; cat $OUT/gemmclk.txt
      if [ $rc -ne 0 ]; then tail -5 $OUT/gemmclk.log; exit $rc; fi ;;
    shapes)
      timeout -k 10 400 python tools/micro/dgemm_shapes.py 5 > $OUT/shapes.log 2>&1
      rc=$?; grep -v '^{' $OUT/shapes.log; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    suite)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -2 $OUT/pytest_gpu.log
      if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; fi
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; tail -1 $OUT/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    bench)
      timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; grep '^{' $OUT/bench.json | cut -c1-400; if [ $rc -ne 0 ]; then tail -5 $OUT/bench.err; exit $rc; fi ;;
    repair)
      # lambda = 0 repair load on the production grid: collinear summands (every window rank
      # <= 200) vs the clean step on the same box
      timeout -k 10 300 python bench.py --no-inputs --steps 20 --warmup 5 > $OUT/bench_clean.json 2> $OUT/bench_clean.err
      rc=$?; grep '^{' $OUT/bench_clean.json | cut -c1-300; if [ $rc -ne 0 ]; then tail -5 $OUT/bench_clean.err; exit $rc; fi
      timeout -k 10 300 python bench.py --no-inputs --steps 20 --warmup 5 --collinear 200 > $OUT/bench_collinear.json 2> $OUT/bench_collinear.err
      rc=$?; grep '^{' $OUT/bench_collinear.json | cut -c1-300; if [ $rc -ne 0 ]; then tail -5 $OUT/bench_collinear.err; exit $rc; fi ;;
    qr)
      # panel QR in isolation (band_panel_factor): cycles per panel, Householder vs CholeskyQR2
      timeout -k 10 200 python tools/bench_qr.py 497 241 > $OUT/qr_bench.jsonl 2> $OUT/qr_bench.err
      rc=$?; cat $OUT/qr_bench.jsonl; if [ $rc -ne 0 ]; then tail -5 $OUT/qr_bench.err; exit $rc; fi ;;
    cooptime)
      for k in 1 2; do
        PFML_COOP_K=$k timeout -k 10 120 python tools/bench_ridge.py --timing > $OUT/coop_timing_k$k.json 2>&1
        rc=$?; grep -E '"(X_partials|C_sums_W|update|lookahead_qr|U|sync_wait|end_sync)"|total' $OUT/coop_timing_k$k.json; if [ $rc -ne 0 ]; then cat $OUT/coop_timing_k$k.json; exit $rc; fi
      done
      PFML_BENCH_CELLS=1,13,106 timeout -k 10 300 python tools/bench_ridge.py > $OUT/coop_cells.log 2>&1
      rc=$?; tail -1 $OUT/coop_cells.log; if [ $rc -ne 0 ]; then exit $rc; fi
      PFML_COOP_K=1 PFML_BENCH_CELLS=1,106 timeout -k 10 300 python tools/bench_ridge.py > $OUT/coop_cells_k1.log 2>&1
      rc=$?; tail -1 $OUT/coop_cells_k1.log; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    benchk)
      # headline bench with the cooperative reduction at auto K and at K = 1 (every cell one WG);
      # PFML_BENCHK overrides the list (e.g. "1 2 1 2")
      for k in ${PFML_BENCHK:-auto 1}; do
        if [ $k = auto ]; then unset PFML_COOP_K; else export PFML_COOP_K=$k; fi
        timeout -k 10 300 python bench.py --no-inputs > $OUT/bench_k$k.json 2> $OUT/bench_k$k.err
        rc=$?; echo "K=$k: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_k$k.json)"; if [ $rc -ne 0 ]; then tail -5 $OUT/bench_k$k.err; exit $rc; fi
      done
      unset PFML_COOP_K ;;
    coop)
      # cooperative band reduction: tests (oracle + bitwise across K), per-phase timing of
      # one n = 513 cell at K = 1 / 2 / 4, wall time vs #cells (auto K)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -k "coop" > $OUT/pytest_coop.log 2>&1
      rc=$?; tail -3 $OUT/pytest_coop.log
      if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_coop.log | head -20; exit $rc; fi
      for k in 1 2 4; do
        PFML_COOP_K=$k timeout -k 10 120 python tools/bench_ridge.py --timing > $OUT/coop_timing_k$k.json 2>&1
        rc=$?; cat $OUT/coop_timing_k$k.json; if [ $rc -ne 0 ]; then exit $rc; fi
      done
      PFML_BENCH_CELLS=1,13,106 timeout -k 10 300 python tools/bench_ridge.py > $OUT/coop_cells.log 2>&1
      rc=$?; tail -1 $OUT/coop_cells.log; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    abmm)
      # utilities: one vs two validation months per workgroup (shared beta tiles), A/B/A/B
      for mm in 1 2 1 2; do
        PFML_QUAD_MM=$mm timeout -k 10 200 python bench.py > $OUT/bench_mm$mm.json 2> $OUT/bench_mm$mm.err
        rc=$?; echo "mm $mm: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_mm$mm.json)"; if [ $rc -ne 0 ]; then tail -5 $OUT/bench_mm$mm.err; exit $rc; fi
      done ;;
    shardk)
      # W-rank rehearsal (PFML_SHARDW, default 8) with the big cells' K forced (PFML_SHARDK
      # list, default "auto 8 4")
      W=${PFML_SHARDW:-8}
      for k in ${PFML_SHARDK:-auto 8 4}; do
        if [ $k = auto ]; then unset PFML_COOP_K; else export PFML_COOP_K=$k; fi
        PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py $W > $OUT/shard${W}_k$k.json 2> $OUT/shard${W}_k$k.err
        rc=$?; echo "W=$W K=$k: $(grep -o '"w[0-9]*_max_ms": [0-9.]*' $OUT/shard${W}_k$k.json)"; if [ $rc -ne 0 ]; then tail -3 $OUT/shard${W}_k$k.err; exit $rc; fi
      done
      unset PFML_COOP_K ;;
    shardtl)
      # kernel timeline of the last rank's grid step of a W = 8 rehearsal (graph replay)
      (cd /tmp && export TMPDIR=/tmp PFML_SHARD_GRAPH=1 && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof8 -o run -- python3 $ROOT/tools/bench_shard.py 8 3 > $OUT/prof8.log 2>&1)
      rc=$?; if [ $rc -ne 0 ]; then tail -3 $OUT/prof8.log; exit $rc; fi
      python tools/rocprof_timeline.py $(find $OUT/prof8 -name "*.db" | head -1) --last 40 > $OUT/timeline8.txt 2>&1
      rm -rf $OUT/prof8; tail -34 $OUT/timeline8.txt ;;
    timeline)
      # kernel timeline of the last full 1-GPU grid step
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof1 -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-inputs > $OUT/prof1.log 2>&1)
      rc=$?; if [ $rc -ne 0 ]; then tail -3 $OUT/prof1.log; exit $rc; fi
      python tools/rocprof_timeline.py $(find $OUT/prof1 -name "*.db" | head -1) --last 40 > $OUT/timeline1.txt 2>&1
      tail -32 $OUT/timeline1.txt ;;
    shards4)
      # per-rank S4 + S5 + S6 of W = 1, 2, 4, 8 rank shards on this GPU (whole-node projection)
      timeout -k 10 900 python tools/bench_shard.py --with-inputs 1,2,4,8 5 > $OUT/shard_s4.json 2> $OUT/shard_s4.err
      rc=$?; cat $OUT/shard_s4.json; if [ $rc -ne 0 ]; then tail -5 $OUT/shard_s4.err; exit $rc; fi ;;
    shard8)
      # per-rank S4 + step of the W = 8 shards only (PFML_* A/B switches from the caller)
      timeout -k 10 600 python tools/bench_shard.py --with-inputs 8 2 > $OUT/shard8_s4.json 2> $OUT/shard8_s4.err
      rc=$?; cat $OUT/shard8_s4.json; if [ $rc -ne 0 ]; then tail -5 $OUT/shard8_s4.err; exit $rc; fi ;;
    shard8prof)
      # kernel stats of rank 0's S4 + step at W = 8 on one stream (serial: the latency floor)
      (cd /tmp && export TMPDIR=/tmp PFML_S4_STREAMS=1 && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_sh8 -o run -- python3 $ROOT/tools/bench_shard.py --with-inputs 8 1 0 > $OUT/prof_sh8.log 2>&1)
      rc=$?; tail -2 $OUT/prof_sh8.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi
      python tools/rocprof_summary.py $(find $OUT/prof_sh8 -name "*.db" | head -1) --top 45 > $OUT/kernels_sh8.txt 2>&1; rm -rf $OUT/prof_sh8; cat $OUT/kernels_sh8.txt ;;
    segtl)
      # kernel timeline of the segmented (multi-rank form) grid step: RCCL at a forced world of
      # one, the process group from the env (no launcher under the profiler)
      (cd /tmp && export TMPDIR=/tmp PFML_DIST_FORCE=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/profseg -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-inputs > $OUT/profseg.log 2>&1)
      rc=$?; grep '^{' $OUT/profseg.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -3 $OUT/profseg.log; exit $rc; fi
      python tools/rocprof_timeline.py $(find $OUT/profseg -name "*.db" | head -1) --last 80 > $OUT/timeline_seg.txt 2>&1
      tail -45 $OUT/timeline_seg.txt ;;
    shard)
      PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py 1,2,4,8 > $OUT/shard.json 2> $OUT/shard.err
      rc=$?; cat $OUT/shard.json; if [ $rc -ne 0 ]; then tail -3 $OUT/shard.err; exit $rc; fi ;;
    shardserial)
      # fault hunt: serialised launches, so a memory fault surfaces at the launching call
      AMD_SERIALIZE_KERNEL=3 PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py 1,2,4,8 2 > $OUT/shard_serial.json 2> $OUT/shard_serial.err
      rc=$?; cat $OUT/shard_serial.json; if [ $rc -ne 0 ]; then grep -v "^frame" $OUT/shard_serial.err | tail -25; exit $rc; fi ;;
    ktest)
      # targeted GPU tests: PFML_KTEST = pytest -k expression
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${PFML_KTEST}" > $OUT/pytest_k.log 2>&1
      rc=$?; tail -3 $OUT/pytest_k.log
      if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_k.log | cut -c1-300 | head -20; exit $rc; fi ;;
    e2e)
      # production-shape end-to-end run of `main` (SURVEY §7 north star): synthetic raw data of
      # the production shape (500 stocks, 1952-2023), the two S0 stages, then the 8 stages of
      # Main.py on the GPU; per-stage JSONL metrics
      D=/tmp/pfml_e2e_data; AD=/tmp/pfml_e2e_art
      rm -rf $D $AD
      timeout -k 10 400 python -u -m pfml synth-data --data-dir $D > $OUT/e2e_synth.log 2>&1
      rc=$?; tail -1 $OUT/e2e_synth.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi
      PFML_METRICS=$OUT/e2e_metrics.jsonl timeout -k 10 600 python -u -m pfml stages get-additional-data,sp500-subset --data-dir $D --artifact-dir $AD --device cuda > $OUT/e2e_s0.log 2>&1
      rc=$?; tail -2 $OUT/e2e_s0.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi
      PFML_METRICS=$OUT/e2e_metrics.jsonl timeout -k 10 900 python -u -m pfml main --data-dir $D --artifact-dir $AD --device cuda > $OUT/e2e_main.log 2>&1
      rc=$?; tail -3 $OUT/e2e_main.log | cut -c1-300; cat $OUT/e2e_metrics.jsonl | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    s4)
      timeout -k 10 600 python bench.py --with-inputs --steps 1 --warmup 1 > $OUT/bench_s4.json 2> $OUT/bench_s4.err
      rc=$?; grep '^{' $OUT/bench_s4.json | cut -c1-300; if [ $rc -ne 0 ]; then tail -3 $OUT/bench_s4.err; exit $rc; fi
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_s4 -o run -- python3 $ROOT/bench.py --with-inputs --steps 1 --warmup 0 > $OUT/prof_s4.log 2>&1)
      rc=$?; if [ $rc -ne 0 ]; then tail -3 $OUT/prof_s4.log; exit $rc; fi
      python tools/rocprof_summary.py $(find $OUT/prof_s4 -name "*.db" | head -1) --top 30 > $OUT/kernels_s4.txt 2>&1
      rm -rf $OUT/prof_s4; cat $OUT/kernels_s4.txt ;;
    s4b)
      # S4+S5+S6 bench only (A/B of an env switch: PFML_* set by the caller)
      timeout -k 10 600 python bench.py --with-inputs --steps 2 --warmup 1 > $OUT/bench_s4b.json 2> $OUT/bench_s4b.err
      rc=$?; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_s4b.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench_s4b.err; exit $rc; fi ;;
    stress)
      timeout -k 10 900 python -u bench.py --s4-stress 48 --stocks 3000 --warmup 1 > $OUT/stress3000.json 2> $OUT/stress3000.err
      rc=$?; cat $OUT/stress3000.json; tail -2 $OUT/stress3000.err; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    stressprof)
      # kernel stats of the 3000-stock stress (12 months)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_stress -o run -- python3 $ROOT/bench.py --s4-stress 12 --stocks 3000 --warmup 0 > $OUT/prof_stress.log 2>&1)
      rc=$?; if [ $rc -ne 0 ]; then tail -3 $OUT/prof_stress.log; exit $rc; fi
      python tools/rocprof_summary.py $(find $OUT/prof_stress -name "*.db" | head -1) --top 20 > $OUT/kernels_stress.txt 2>&1
      rm -rf $OUT/prof_stress; cat $OUT/kernels_stress.txt ;;
    prec)
      for pr in bf16 fp8; do
        timeout -k 10 600 python bench.py --with-inputs --steps 1 --warmup 1 --precision $pr > $OUT/bench_s4_$pr.json 2> $OUT/bench_s4_$pr.err
        rc=$?; grep '^{' $OUT/bench_s4_$pr.json | cut -c1-300; if [ $rc -ne 0 ]; then tail -3 $OUT/bench_s4_$pr.err; exit $rc; fi
      done ;;
    pmc)
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $OUT/pmc -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-inputs > $OUT/pmc.log 2>&1)
      rc=$?; python tools/pmc_summary.py $OUT/pmc --top 10 > $OUT/pmc.txt 2>&1; cat $OUT/pmc.txt; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    pmcmem)
      # HBM bytes per grid-step kernel: FETCH_SIZE and WRITE_SIZE in passes of their own
      # (3 + 2 TCC counters), with the kernel durations from the same runs
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAVES --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-inputs > $OUT/pmc_fetch.log 2>&1)
      rc=$?; python tools/pmc_summary.py $OUT/pmc_fetch --top 14 > $OUT/pmc_fetch.txt 2>&1; cat $OUT/pmc_fetch.txt; if [ $rc -ne 0 ]; then exit $rc; fi
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_WAVES --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-inputs > $OUT/pmc_write.log 2>&1)
      rc=$?; python tools/pmc_summary.py $OUT/pmc_write --top 14 > $OUT/pmc_write.txt 2>&1; cat $OUT/pmc_write.txt; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    multiproc)
      timeout -k 10 900 bash tools/gpu_multiproc.sh $TAG ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
