set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_sharded_gpu.py tests/test_multirank_gpu.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r03_wire_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|rel L1|passed|failed" gpurun_out/r03_wire_tests.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/owner_bench.py > gpurun_out/r03_owner4.json 2> gpurun_out/r03_owner4.err || { tail -20 gpurun_out/r03_owner4.err; exit 1; }
cat gpurun_out/r03_owner4.json
