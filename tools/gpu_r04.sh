# Round-4 GPU runs (gpurun): bash tools/gpu_r04.sh TAG STEP...
#   suite  full -m gpu suite          smoke   __graft_entry__.smoke()
#   bench  default bench.py line      prof    rocprofv3 kernel trace + stats of bench.py, timed-window summary
#   multi  only the multi-rank tests  fwdprof rocprofv3 of a short bench (K=30) for quick per-kernel A/B
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in "$@"; do
  case $s in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
      tail -2 gpurun_out/${TAG}_gpu_tests.log ;;
    multi)
      timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread \
        > gpurun_out/${TAG}_multi.log 2>&1 || { tail -30 gpurun_out/${TAG}_multi.log; exit 1; }
      tail -2 gpurun_out/${TAG}_multi.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -1 gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
        || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${TAG}_bench.json ;;
    prof)
      cd /tmp && cd - > /dev/null
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err \
        || { tail -20 gpurun_out/${TAG}_prof_bench.err; exit 1; }
      python3 tools/step_breakdown.py gpurun_out/${TAG}_prof --window --json gpurun_out/${TAG}_timed_kernels.json \
        > gpurun_out/${TAG}_timed_kernels.txt && head -40 gpurun_out/${TAG}_timed_kernels.txt
      python3 tools/step_breakdown.py gpurun_out/${TAG}_prof --window --seq | tail -45 > gpurun_out/${TAG}_launch_sequence.txt
      python3 tools/bench_summary.py gpurun_out/${TAG}_prof_bench.json ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
