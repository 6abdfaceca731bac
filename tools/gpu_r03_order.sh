# backward prologue with / without the tile-order workgroup (what bounds the prologue)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 240 python -u tools/variant_step.py --tag order --steps 40 >> gpurun_out/r03_order.jsonl 2>> gpurun_out/r03_order.err || { tail -20 gpurun_out/r03_order.err; exit 1; }
  RAIN_BWD_TILE_ORDER=0 timeout -k 10 240 python -u tools/variant_step.py --tag noorder --steps 40 >> gpurun_out/r03_order.jsonl 2>> gpurun_out/r03_order.err || { tail -20 gpurun_out/r03_order.err; exit 1; }
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_order.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s.get("memset"), s.get("blend_bwd"))
P
