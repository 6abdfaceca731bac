set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_sharded_gpu.py -k "not cfg4" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_chunk.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|rel L1|passed|failed" gpurun_out/r03_chunk.log | tail -20
exit $rc
