set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in base shco shno; do
    RAIN_RASTER_LIB=gpurun_variants/$v.so timeout -k 10 240 python -u tools/variant_step.py --tag $v --steps 40 >> gpurun_out/r03_shprobe.jsonl 2>> gpurun_out/r03_shprobe.err || { tail -20 gpurun_out/r03_shprobe.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_shprobe.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms_per_step"], d["stages_ms"]["preprocess"])
P
