#!/bin/bash
# The one GPU driver (run through gpurun from the repo root):
#     T=r05a scripts/gpu.sh tests smoke driver long prof
# Each named step runs under its own time limit and writes
# gpurun_out/${T}_<step>.txt (rocprof output under gpurun_out/${T}_<step>/).
# The run stops at the first failing step: nothing more touches the GPU after
# a fault, abort, segfault or time limit.
#   tests      full GPU pytest suite           window  BA window / harness tests
#   corrtests  corr + golden GPU tests         large   large-graph / global / sharded BA tests
#   smoke      __graft_entry__.smoke()
#   driver     bench.py exactly as the driver runs it (--steps 20 --warmup 5)
#   long       bench.py --steps 300 --warmup 10 (no CPU baseline)
#   bench      bench.py $BENCH_ARGS (full default run, CPU baseline included)
#   prof       rocprofv3 --kernel-trace --stats over a 200-step bench (kernel table printed)
#   profdrv    the same over the driver's 20-step command
#   proff16    the same over a 200-step bench with fp16 features
#   phases     BA window phase tables: cfg2 2 iterations, DPVO windows E=9850 / 3940 1 iteration
#   probe      host enqueue time per call of a step, first after a sync vs steady
#   stale      the stale-granule regression test; staledemo: its A/B on the round-4 tree
#   launchprof rocprof kernel durations of the fused start-of-update launch and its parts
#   launchtrace per-workgroup timeline of that launch inside the bench step (scripts/launch_trace.py)
#   corrvar    A-CORR product kernel times, fp32 and fp16 (scripts/corr_variants.py)
#   corrab     A/B of builds copied to scratch_ab/<v> (VARIANTS, scripts/corr_ab.sh)
#   dropin     per-level NCHW / channels-last drop-in calls (scripts/corr_dropin_bench.py)
#   benchf16   bench.py --features f16 (the fork's MIXED_PRECISION rings)
#   spdbench   training-path dense solve vs torch/rocSOLVER (scripts/spd_solve_bench.py)
#   dpvoprof   rocprofv3 over the fork's live BA call at E = 9850 (scripts/dpvo_window_call.py)
#   corrpmc    SQ / TCC counter passes over scripts/corr_variants.py (scripts/pmc_corrvar.sh)
#   corrwide   the channels-last corr tests incl. the wide-dynamic-range ones
#   cfg4       bench.py --sharded (cfg4 global BA, one rank)
#   cfg4prof   rocprofv3 over the cfg4 bench
#   pmcsq      BA/corr SQ + LDS counter passes (scripts/pmc.sh with PMC_GROUPS)
#   traffic    corr FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${T:-run}
mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
run() {  # run <name> <limit-s> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/${T}_$name.txt 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  tail -4 $O/${T}_$name.txt
  [ $rc -eq 0 ] || exit $rc
}
prof() {  # prof <name> <bench args...>
  local name=$1; shift
  run $name 400 rocprofv3 --kernel-trace --stats -d $O/${T}_$name -o run --output-format csv \
    -- python bench.py --no-cpu-baseline "$@"
  local f
  f=$(find $O/${T}_$name -name "*kernel_stats.csv" | head -1)
  python scripts/kstats.py "$f" 8 | tee $O/${T}_${name}_kstats.txt
}
for s in "$@"; do
  case $s in
    tests) run tests 900 $PYT tests ;;
    window) run window 400 $PYT tests/test_ba_window_gpu.py tests/test_ba_gpu.py tests/test_update_harness_gpu.py ;;
    corrtests) run corrtests 400 $PYT tests/test_corr_gpu.py tests/test_golden_gpu.py ;;
    large) run large 500 $PYT tests/test_ba_large_gpu.py tests/test_global_ba_gpu.py tests/test_sharded_hip_gpu.py ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    driver) run driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    long) run long 300 python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline ;;
    bench) run bench 400 python -u bench.py ${BENCH_ARGS:-} ;;
    prof) prof prof --steps 200 --warmup 10 ;;
    profdrv) prof profdrv --steps 20 --warmup 5 ;;
    proff16) prof proff16 --steps 200 --warmup 10 --features f16 ;;
    phases)
      run phases_cfg2 300 python -u scripts/ba_window_phases.py cfg2 2
      run phases_dpvo25_1 300 python -u scripts/ba_window_phases.py 25 1
      run phases_dpvo10_1 300 python -u scripts/ba_window_phases.py 10 1 ;;
    probe) run probe 300 python -u scripts/host_enqueue_probe.py ;;
    staledemo) run staledemo 400 python -u scripts/stale_granule_demo.py _r04tree . ;;
    stale) run stale 400 $PYT tests/test_granule_stale_gpu.py ;;
    launchprof)  # kernel durations of the update's first launch and its parts
      run launchprof 300 rocprofv3 --kernel-trace --stats -d $O/${T}_launchprof -o run --output-format csv \
        -- python scripts/reproject_launch_bench.py cfg2 dpvo25
      python scripts/kstats.py "$(find $O/${T}_launchprof -name '*kernel_stats.csv' | head -1)" 12 \
        | tee $O/${T}_launchprof_kstats.txt ;;
    spdbench) run spdbench 200 python -u scripts/spd_solve_bench.py ;;
    launchtrace) run launchtrace 200 python -u scripts/launch_trace.py ;;
    corrvar) run corrvar 200 python -u scripts/corr_variants.py ${CORRVAR_ARGS:-} ;;
    corrpmc) run corrpmc 700 bash scripts/pmc_corrvar.sh ;;
    corrab) run corrab 400 bash scripts/corr_ab.sh ;;
    dropin) run dropin 300 python -u scripts/corr_dropin_bench.py ;;
    benchf16) run benchf16 300 python -u bench.py --features f16 --no-cpu-baseline ;;
    dpvoprof)
      run dpvocall 200 python -u scripts/dpvo_window_call.py
      run dpvoprof 300 rocprofv3 --kernel-trace --stats -d $O/${T}_dpvoprof -o run --output-format csv \
        -- python scripts/dpvo_window_call.py
      python scripts/kstats.py "$(find $O/${T}_dpvoprof -name '*kernel_stats.csv' | head -1)" 8 \
        | tee $O/${T}_dpvoprof_kstats.txt ;;
    corrwide) run corrwide 300 $PYT tests/test_corr_gpu.py -k "wide_range or channels_last" ;;
    cfg4) run cfg4 300 python -u bench.py --sharded --steps 5 --warmup 2 ;;
    cfg4prof) prof cfg4prof --sharded --steps 3 --warmup 1 ;;
    pmcsq) run pmcsq 600 env SQ_EXTRA="${SQ_EXTRA:-SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE}" bash scripts/pmc_sq.sh ;;
    traffic) run traffic 400 env PMC_GROUPS="FETCH_SIZE WRITE_SIZE" bash scripts/pmc.sh ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
