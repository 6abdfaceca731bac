# final tree: cfg5 (5M @ 4K, depth + normal) bench and the sharded step forced at world 1 over RCCL
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --points 5000000 --width 3840 --height 2160 --aux-normal --steps 30 --no-cpu-baseline > gpurun_out/r03d_cfg5.json 2> gpurun_out/r03d_cfg5.err || { tail -20 gpurun_out/r03d_cfg5.err; exit 1; }
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29537 bench.py --force-dist --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03d_dist.json 2> gpurun_out/r03d_dist.err || { tail -20 gpurun_out/r03d_dist.err; exit 1; }
python3 - <<'P'
import json
for f in ("gpurun_out/r03d_cfg5.json", "gpurun_out/r03d_dist.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["config"]["parallelism"], d["config"]["gaussians"], d["config"]["width"])
P
