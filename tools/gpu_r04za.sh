# k_gauss_bwd compact SH gradients (parameters from LDS): full -m gpu suite, then an interleaved A/B
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for o in gauss_bwd_compact=1 gauss_bwd_compact=0; do
    timeout -k 10 300 python -u tools/variant_step.py --tag $o --tune $o \
      >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
  done
done
cat gpurun_out/${TAG}_ab.jsonl
