set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in base bl; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 60 >> gpurun_out/r03_bl.jsonl 2>> gpurun_out/r03_bl.err || { tail -20 gpurun_out/r03_bl.err; exit 1; }
  done
done
cat gpurun_out/r03_bl.jsonl
RAIN_RASTER_LIB=gpurun_variants/bl.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_fused_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_bl_parity.log 2>&1; tail -3 gpurun_out/r03_bl_parity.log
