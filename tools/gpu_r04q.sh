# early-stop + parity tests, then the bench kernel trace
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_early_stop_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04f.sh $TAG
