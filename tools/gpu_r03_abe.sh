set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_densify_gpu.py tests/test_native_abi.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_abe.log 2>&1; rc=$?
tail -15 gpurun_out/r03_abe.log; exit $rc
