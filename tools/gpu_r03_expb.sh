set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in base expb; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 40 >> gpurun_out/r03_expb.jsonl 2>> gpurun_out/r03_expb.err || { tail -20 gpurun_out/r03_expb.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_expb.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms_per_step"], d["stages_ms"]["ranges"])
P
RAIN_RASTER_LIB=gpurun_variants/expb.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_early_stop_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_expb_parity.log 2>&1; rc=$?; tail -2 gpurun_out/r03_expb_parity.log; exit $rc
