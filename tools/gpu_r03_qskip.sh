set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in base qskip; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 40 >> gpurun_out/r03_qskip.jsonl 2>> gpurun_out/r03_qskip.err || { tail -20 gpurun_out/r03_qskip.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_qskip.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms_per_step"], d["stages_ms"]["blend_bwd"])
P
RAIN_RASTER_LIB=gpurun_variants/qskip.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_fused_gpu.py tests/test_early_stop_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_qskip_parity.log 2>&1; rc=$?; tail -2 gpurun_out/r03_qskip_parity.log; exit $rc
