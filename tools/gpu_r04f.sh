# one rocprofv3 kernel trace of a short bench run (per-kernel durations of the step) + the fused tests
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
  -- python3 bench.py --steps 30 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err \
  || { tail -20 gpurun_out/${TAG}_prof_bench.err; exit 1; }
python3 tools/step_breakdown.py gpurun_out/${TAG}_prof --window > gpurun_out/${TAG}_timed_kernels.txt 2>&1
python3 tools/step_breakdown.py gpurun_out/${TAG}_prof --window --seq | tail -45 > gpurun_out/${TAG}_launch_sequence.txt 2>&1
head -40 gpurun_out/${TAG}_timed_kernels.txt
cat gpurun_out/${TAG}_launch_sequence.txt
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_fused_tests.log 2>&1; tail -3 gpurun_out/${TAG}_fused_tests.log
