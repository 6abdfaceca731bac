set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_mr.log 2>&1 || { tail -60 gpurun_out/t_mr.log; exit 1; }
tail -5 gpurun_out/t_mr.log
