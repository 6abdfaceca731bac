# native densification statistics: tests, API-path trace, bench
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_densify_gpu.py tests/test_fused_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_api -o run --output-format csv \
  -- python3 tools/api_trace.py > gpurun_out/${TAG}_api.log 2> gpurun_out/${TAG}_api.err || { tail -20 gpurun_out/${TAG}_api.err; exit 1; }
cat gpurun_out/${TAG}_api.log
python3 tools/step_breakdown.py gpurun_out/${TAG}_api --window > gpurun_out/${TAG}_api_kernels.txt 2>&1
python3 tools/step_breakdown.py gpurun_out/${TAG}_api --window --seq | tail -60 > gpurun_out/${TAG}_api_seq.txt 2>&1
head -40 gpurun_out/${TAG}_api_kernels.txt
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
