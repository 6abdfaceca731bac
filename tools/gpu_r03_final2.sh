set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --force-dist --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03_final2_dist.json 2> gpurun_out/r03_final2_dist.err || { tail -20 gpurun_out/r03_final2_dist.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r03_final2_dist.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(d["value"], d["ms_per_step"], d["config"]["parallelism"], "densify", d.get("densify_iter_ms"))
print({k: r[k] for k in ("kernel", "achieved", "frac", "ms_per_launch", "launches_per_step", "algorithmic_bytes_per_launch")})
print({k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()})
P
bash tools/profile_round.sh gpurun_out/prof_r03b && python3 tools/step_breakdown.py gpurun_out/prof_r03b/bench > gpurun_out/prof_r03b/step_breakdown.txt 2>&1
head -5 gpurun_out/prof_r03b/step_breakdown.txt
