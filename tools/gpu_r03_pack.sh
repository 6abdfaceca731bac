set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 240 python -u tools/variant_step.py --tag sep --steps 40 >> gpurun_out/r03_pack.jsonl 2>> gpurun_out/r03_pack.err || { tail -20 gpurun_out/r03_pack.err; exit 1; }
  timeout -k 10 240 python -u tools/variant_step.py --tag packed --pack --steps 40 >> gpurun_out/r03_pack.jsonl 2>> gpurun_out/r03_pack.err || { tail -20 gpurun_out/r03_pack.err; exit 1; }
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_pack.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms_per_step"], d["stages_ms"]["gauss_bwd"], d["stages_ms"]["preprocess"])
P
