# sort unit-size A/B with the 8-wave scatter (rr_set_tuning knobs through tools/variant_step.py --tune)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { timeout -k 10 240 python -u tools/variant_step.py --steps 40 "$@" >> gpurun_out/r03_units.jsonl 2>> gpurun_out/r03_units.err || { tail -20 gpurun_out/r03_units.err; exit 1; }; }
for i in 1 2; do
  run --tag d256_t1024
  run --tag d512 --tune sort_min_units=512
  run --tag d128 --tune sort_min_units=128
  run --tag t512 --tune sort_min_units_tile=512
  run --tag t2048 --tune sort_min_units_tile=2048
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_units.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s["depth_sort"], s["duplicate"], s["tile_sort"])
P
