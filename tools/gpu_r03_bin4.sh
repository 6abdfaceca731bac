set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_bin4_suite.log 2>&1; rc=$?; tail -15 gpurun_out/r03_bin4_suite.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base bin4; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 40 >> gpurun_out/r03_bin4.jsonl 2>> gpurun_out/r03_bin4.err || { tail -20 gpurun_out/r03_bin4.err; exit 1; }
  done
done
cat gpurun_out/r03_bin4.jsonl
