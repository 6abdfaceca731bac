set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in base du1 du2 du4; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 40 >> gpurun_out/r03_du.jsonl 2>> gpurun_out/r03_du.err || { tail -20 gpurun_out/r03_du.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_du.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms_per_step"], d["stages_ms"]["duplicate"])
P
RAIN_RASTER_LIB=gpurun_variants/du4.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_early_stop_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_du_parity.log 2>&1; rc=$?; tail -2 gpurun_out/r03_du_parity.log; exit $rc
