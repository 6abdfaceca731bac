set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in base pre5 pre6; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 40 >> gpurun_out/r03_pre.jsonl 2>> gpurun_out/r03_pre.err || { tail -20 gpurun_out/r03_pre.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_pre.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms_per_step"], d["stages_ms"]["preprocess"])
P
