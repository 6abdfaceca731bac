set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_b2.json 2> gpurun_out/r03_b2.err || { tail -20 gpurun_out/r03_b2.err; exit 1; }
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_b2f.json 2> gpurun_out/r03_b2f.err || { tail -20 gpurun_out/r03_b2f.err; exit 1; }
python3 - <<'P'
import json
for f in ("gpurun_out/r03_b2.json", "gpurun_out/r03_b2f.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["config"]["parallelism"], "densify", d["densify_iter_ms"], d["ordinary_iter_ms_alone"], "api", d["api_iters_per_s"])
    print({k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()})
P
