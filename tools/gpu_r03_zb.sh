# backward prologue: clear workgroups 2048 (base) / 512 / 256 / 128 beside the tile-order workgroup
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in base zb512 zb256 zb128; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 40 >> gpurun_out/r03_zb.jsonl 2>> gpurun_out/r03_zb.err || { tail -20 gpurun_out/r03_zb.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_zb.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s.get("memset"), s.get("blend_bwd"), s.get("gauss_bwd"))
P
