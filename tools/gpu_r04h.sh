# kernel trace of the bench step + parity/fused GPU tests + sortexpand LDS-capacity A/B
set -o pipefail
TAG=$1
bash tools/gpu_r04f.sh $TAG || exit 1
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_parity_tests.log 2>&1; tail -3 gpurun_out/${TAG}_parity_tests.log
bash tools/gpu_ab.sh $TAG "sx4096 sx2048"
