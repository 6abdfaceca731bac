set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python -u tools/variant_step.py --tag base >> gpurun_out/r03_v1.jsonl 2>/dev/null || exit 1
  RAIN_RASTER_LIB=gpurun_variants/rcp1.so timeout -k 10 200 python -u tools/variant_step.py --tag rcp1 >> gpurun_out/r03_v1.jsonl 2>/dev/null || exit 1
done
cat gpurun_out/r03_v1.jsonl
RAIN_RASTER_LIB=gpurun_variants/rcp1.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py::test_cfg3_api_and_fused_paths_match_oracle -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_v1_parity.log 2>&1; tail -3 gpurun_out/r03_v1_parity.log
