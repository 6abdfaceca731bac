# backward-blend waves per tile (1 / 2 / 4) on the current kernels + per-tile tile_max of three bench views
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/tile_stats.py gpurun_out/r03_tile_max.npz > gpurun_out/r03_tile_stats.json 2> gpurun_out/r03_tile_stats.err || { tail -20 gpurun_out/r03_tile_stats.err; exit 1; }
for i in 1 2; do
  for nw in 1 2 4; do
    timeout -k 10 240 python -u tools/variant_step.py --tag nw$nw --tune bwd_waves=$nw --steps 40 >> gpurun_out/r03_nw.jsonl 2>> gpurun_out/r03_nw.err || { tail -20 gpurun_out/r03_nw.err; exit 1; }
  done
done
python3 - <<'P'
import json
for l in open("gpurun_out/r03_nw.jsonl"):
    d = json.loads(l); s = d["stages_ms"]; print(d["tag"], d["ms_per_step"], s["blend_bwd"])
P
