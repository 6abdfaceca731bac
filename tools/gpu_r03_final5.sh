# A/B of the backward blend's per-pair reduction without the empty-pair skip (noskip), then the
# final validation of the tree: -m gpu suite, smoke, default bench, rocprofv3 stats + PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in base noskip; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 60 >> gpurun_out/r03_noskip.jsonl 2>> gpurun_out/r03_noskip.err || { tail -20 gpurun_out/r03_noskip.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_noskip.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s.get("blend_bwd"))
P
bash tools/gpu_r03_final4.sh
