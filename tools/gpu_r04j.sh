# phase-B gather path: early-stop tests (both phase-B paths) + full -m gpu suite, A/B of the two
# phase-B paths on the bench step, bench kernel trace
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_early_stop_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_early_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_early_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for o in phase_b_gather=1 phase_b_gather=0; do
    timeout -k 10 300 python -u tools/variant_step.py --tag $o --tune $o \
      >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
  done
done
cat gpurun_out/${TAG}_ab.jsonl
bash tools/gpu_r04f.sh $TAG
