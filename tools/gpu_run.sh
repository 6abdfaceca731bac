#!/bin/bash
# One parameterised GPU lease script (run through gpurun); replaces the per-experiment
# tools/gpu_r0*.sh scripts of rounds 3-4.  Steps run in order, each under its own time limit; the
# first failing step ends the call (no GPU step runs after a failure).
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# STEP is one of
#   smoke                 __graft_entry__.smoke()
#   tests[=EXPR]          pytest -m gpu (EXPR: a -k expression)
#   bench[=ARGS]          python bench.py ARGS (default: the driver's command line)
#   ab=T1,T2[,..]         interleaved A/B of the training step (tools/variant_step.py), two rounds;
#                         Ti = a list of rr_set_tuning key=value (or variant_step.py --options)
#                         joined by '+', or 'base'
#   abv=V1,V2[,..]        the same over librain_raster.so variants (tools/build_variant.py names)
#   abl=V1,V2[,..]        the same over librain_loss.so variants (build_variant.py --lib librain_loss.so)
#   prof[=ARGS]           rocprofv3 kernel trace + stats of the bench (default arguments + ARGS), timed-window summary
#   stalls=PATTERN        one SQ stall-counter pass, summarised for the kernels matching PATTERN
#   pbprof                phase-B kernel durations per view vs the open-tile region (tools/phaseb_profile.py)
#   fwdtrace              per-wave forward-blend timelines (tools/fwd_trace.py, gpurun_variants/trace.so)
#   hostprobe[=ARGS]      host time of the training step under cProfile (tools/host_probe.py ARGS)
#   owner                 owner-kernel time of the sharded step for N = 1, 2, 4, 8 (tools/owner_bench.py)
#   pmc                   PMC passes (tools/profile_round.sh without the trace) -> pmc_traffic.json
# Output: gpurun_out/TAG_*.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
for STEP in "$@"; do
  case "$STEP" in
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > ${OUT}_smoke.log 2>&1 || { tail -20 ${OUT}_smoke.log; exit 1; }
      tail -2 ${OUT}_smoke.log ;;
    tests|tests=*)
      K=(); [ "$STEP" != tests ] && K=(-k "${STEP#tests=}")
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
        > ${OUT}_gpu_tests.log 2>&1; rc=$?; tail -3 ${OUT}_gpu_tests.log
      [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" ${OUT}_gpu_tests.log | head -30; exit $rc; } ;;
    bench|bench=*)
      A="--gpus 1 --steps 20 --warmup 5"; [ "$STEP" != bench ] && A="${STEP#bench=}"
      timeout -k 10 600 python3 bench.py $A > ${OUT}_bench.json 2> ${OUT}_bench.err \
        || { tail -20 ${OUT}_bench.err; exit 1; }
      cat ${OUT}_bench.json ;;
    ab=*)
      IFS=',' read -ra VS <<< "${STEP#ab=}"
      for r in 1 2; do
        for v in "${VS[@]}"; do
          TUNE=""
          if [ "$v" != base ]; then
            IFS='+' read -ra KV <<< "$v"
            for kv in "${KV[@]}"; do
              case "$kv" in -*) TUNE="$TUNE $kv" ;; *) TUNE="$TUNE --tune $kv" ;; esac
            done
          fi
          timeout -k 10 300 python3 -u tools/variant_step.py --tag="$v" $TUNE >> ${OUT}_ab.jsonl 2>> ${OUT}_ab.err \
            || { tail -20 ${OUT}_ab.err; exit 1; }
        done
      done
      cat ${OUT}_ab.jsonl ;;
    abv=*)
      IFS=',' read -ra VS <<< "${STEP#abv=}"
      for r in 1 2; do
        for v in "${VS[@]}"; do
          LIB=""; [ "$v" != base ] && LIB=gpurun_variants/$v.so
          RAIN_RASTER_LIB=$LIB timeout -k 10 300 python3 -u tools/variant_step.py --tag="$v" >> ${OUT}_ab.jsonl \
            2>> ${OUT}_ab.err || { tail -20 ${OUT}_ab.err; exit 1; }
        done
      done
      cat ${OUT}_ab.jsonl ;;
    abl=*)
      IFS=',' read -ra VS <<< "${STEP#abl=}"
      for r in 1 2; do
        for v in "${VS[@]}"; do
          LIB=""; [ "$v" != base ] && LIB=gpurun_variants/$v.so
          RAIN_LOSS_LIB=$LIB timeout -k 10 300 python3 -u tools/variant_step.py --tag="$v" >> ${OUT}_ab.jsonl \
            2>> ${OUT}_ab.err || { tail -20 ${OUT}_ab.err; exit 1; }
        done
      done
      cat ${OUT}_ab.jsonl ;;
    binstats)
      # per-bin run lengths of three bench frames (tools/bin_stats.py)
      timeout -k 10 300 python3 -u tools/bin_stats.py > ${OUT}_bin_stats.json 2> ${OUT}_bin_stats.err \
        || { tail -20 ${OUT}_bin_stats.err; exit 1; }
      cat ${OUT}_bin_stats.json ;;
    pbprof|pbprof=*)
      # phase-B kernel durations per view against the open-tile region (tools/phaseb_profile.py);
      # pbprof=V: with the library variant gpurun_variants/V.so
      V=""; P=${OUT}_pbp; [ "$STEP" != pbprof ] && { V=gpurun_variants/${STEP#pbprof=}.so; P=${OUT}_pbp_${STEP#pbprof=}; }
      RAIN_RASTER_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace -d $P -o run --output-format csv \
        -- python3 tools/phaseb_profile.py run --views 64 > ${P}_views.jsonl 2> ${P}.err \
        || { tail -20 ${P}.err; exit 1; }
      python3 tools/phaseb_profile.py join $P ${P}_views.jsonl > ${P}_profile.jsonl
      grep -v '"open_tiles": 0,' ${P}_profile.jsonl | head -40 ;;
    fwdtrace)
      # per-wave forward-blend timelines of 6 bench frames (gpurun_variants/trace.so, -DRR_FWD_TRACE=1)
      RAIN_RASTER_LIB=gpurun_variants/trace.so timeout -k 10 300 python3 -u tools/fwd_trace.py --frames 6 \
        > ${OUT}_fwd_trace.txt 2> ${OUT}_fwd_trace.err || { tail -20 ${OUT}_fwd_trace.err; exit 1; }
      cat ${OUT}_fwd_trace.txt ;;
    hostprobe|hostprobe=*)
      # host (Python + driver) time of the training step under cProfile (tools/host_probe.py)
      A=""; [ "$STEP" != hostprobe ] && A="${STEP#hostprobe=}"
      RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29532 timeout -k 10 400 \
        python3 -u tools/host_probe.py $A > ${OUT}_host_probe.txt 2> ${OUT}_host_probe.err \
        || { tail -20 ${OUT}_host_probe.err; exit 1; }
      head -60 ${OUT}_host_probe.txt ;;
    owner)
      # owner-kernel time of the Gaussian-sharded step by N (tools/owner_bench.py)
      timeout -k 10 400 python3 -u tools/owner_bench.py > ${OUT}_owner.jsonl 2> ${OUT}_owner.err \
        || { tail -20 ${OUT}_owner.err; exit 1; }
      cat ${OUT}_owner.jsonl ;;
    prof|prof=*)
      # one rank in this process (the launcher's variables set here): bench.py must not spawn a
      # child under the profiler
      A=""; [ "$STEP" != prof ] && A="${STEP#prof=}"
      RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d ${OUT}_prof -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline $A > ${OUT}_prof_bench.json 2> ${OUT}_prof.err \
        || { tail -20 ${OUT}_prof.err; exit 1; }
      python3 tools/step_breakdown.py ${OUT}_prof --window > ${OUT}_timed_kernels.txt 2>&1
      python3 tools/step_breakdown.py ${OUT}_prof --window --seq | tail -40 > ${OUT}_launch_sequence.txt 2>&1
      head -32 ${OUT}_timed_kernels.txt; cat ${OUT}_launch_sequence.txt ;;
    stalls=*)
      # SQ stall counters (one pass, its own run) over the bench's training step, summarised for the
      # kernels matching the pattern (tools/pmc_stalls.py)
      timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
        --kernel-trace -d ${OUT}_stall -o run --output-format csv -- python3 tools/pmc_workload.py \
        > ${OUT}_stall.log 2>&1 || { tail -20 ${OUT}_stall.log; exit 1; }
      python3 tools/pmc_stalls.py ${OUT}_stall --match "${STEP#stalls=}" | tee ${OUT}_stalls.txt
      python3 tools/pmc_stalls.py ${OUT}_stall --match "${STEP#stalls=}" --min-us 30 > ${OUT}_stalls_long.txt ;;
    pmc)
      bash tools/profile_round.sh ${OUT}_pmcdir pmc-only || exit 1
      head -60 ${OUT}_pmcdir/pmc_traffic.json ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
