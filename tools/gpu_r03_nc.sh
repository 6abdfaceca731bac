# A/B: next-pass digit counts fused into the radix scatter (nc) vs count launches (base)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in base nc; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 60 >> gpurun_out/r03_nc.jsonl 2>> gpurun_out/r03_nc.err || { tail -20 gpurun_out/r03_nc.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_nc.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s["depth_sort"], s["tile_sort"], s["duplicate"])
P
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fused_gpu.py tests/test_early_stop_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_nc_parity.log 2>&1 || { tail -30 gpurun_out/r03_nc_parity.log; exit 1; }
tail -1 gpurun_out/r03_nc_parity.log
