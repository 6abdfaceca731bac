set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sharded_gpu.py tests/test_multirank_gpu.py -k "not cfg4" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_pv_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03_pv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/owner_bench.py > gpurun_out/r03_owner3.json 2> gpurun_out/r03_owner3.err || { tail -20 gpurun_out/r03_owner3.err; exit 1; }
cat gpurun_out/r03_owner3.json
