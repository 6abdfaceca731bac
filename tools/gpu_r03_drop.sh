set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in base drop; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 60 >> gpurun_out/r03_drop.jsonl 2>> gpurun_out/r03_drop.err || { tail -20 gpurun_out/r03_drop.err; exit 1; }
  done
done
cat gpurun_out/r03_drop.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_drop_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r03_drop_suite.log; exit $rc
