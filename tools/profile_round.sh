#!/bin/bash
# Profiling passes for one round (run on the GPU box through gpurun):
#   1. kernel trace + stats of the default bench command  -> $OUT/bench/
#   2. three counter passes over tools/pmc_workload.py (FETCH_SIZE, WRITE_SIZE, SQ VALU activity),
#      each in its own run with --kernel-trace only (no sys/runtime tracing with --pmc)
#   3. tools/pmc_traffic.py -> profiles/pmc_traffic.json
# Usage: bash tools/profile_round.sh gpurun_out/prof_rNN [pmc-only]
set -e -o pipefail
OUT=${1:-gpurun_out/prof}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "$OUT"
if [ "$2" != pmc-only ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/bench" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv \
    -- python3 tools/pmc_workload.py > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv \
    -- python3 tools/pmc_workload.py > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU --kernel-trace -d "$OUT/pmc_sq" -o run \
    --output-format csv -- python3 tools/pmc_workload.py > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-trace \
    -d "$OUT/pmc_inst" -o run --output-format csv -- python3 tools/pmc_workload.py > "$OUT/inst.log" 2>&1
# transcendental VALU instructions (v_exp / v_rcp / v_sqrt issue at twice a v_fma's cost), so the
# issue fraction of the blends can price them; optional: a counter this ROCm does not know fails fast
TRANS=""
if timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES --kernel-trace \
    -d "$OUT/pmc_trans" -o run --output-format csv -- python3 tools/pmc_workload.py > "$OUT/trans.log" 2>&1; then
  TRANS="--trans-dir $OUT/pmc_trans"
else
  echo "transcendental counter pass failed (see $OUT/trans.log)"
fi
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --sq-dir "$OUT/pmc_sq" --inst-dir "$OUT/pmc_inst" \
    $TRANS --out "$OUT/pmc_traffic.json" > /dev/null
echo "profile passes done: $OUT"
