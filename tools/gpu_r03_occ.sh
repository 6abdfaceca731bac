set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/owner_bench.py > gpurun_out/r03_owner2.json 2> gpurun_out/r03_owner2.err || { tail -20 gpurun_out/r03_owner2.err; exit 1; }
cat gpurun_out/r03_owner2.json
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_sharded_gpu.py tests/test_parity_gpu.py tests/test_fused_gpu.py -k "not cfg4" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_occ_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03_occ_tests.log; exit $rc
