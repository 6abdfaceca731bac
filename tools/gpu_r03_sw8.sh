set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in base sw8; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 40 >> gpurun_out/r03_sw8.jsonl 2>> gpurun_out/r03_sw8.err || { tail -20 gpurun_out/r03_sw8.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_sw8.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms_per_step"], d["stages_ms"]["depth_sort"], d["stages_ms"]["tile_sort"], d["stages_ms"]["duplicate"])
P
for v in sw8; do
RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_fused_gpu.py tests/test_early_stop_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_${v}_parity.log 2>&1 || { tail -5 gpurun_out/r03_${v}_parity.log; exit 1; }
tail -1 gpurun_out/r03_${v}_parity.log
done
