set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_multirank_gpu.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r03_t2.log 2>&1 || { grep -E "rel L1|PASS|FAIL|Error|error" gpurun_out/r03_t2.log | head -30; tail -60 gpurun_out/r03_t2.log; exit 1; }
grep -E "rel L1|PASSED|FAILED|passed|failed" gpurun_out/r03_t2.log | cut -c1-300
