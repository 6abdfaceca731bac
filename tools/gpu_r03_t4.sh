set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_multirank_gpu.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r03_t4.log 2>&1 || { grep -E "rel L1|PASS|FAIL|Error|error" gpurun_out/r03_t4.log | head -30; tail -40 gpurun_out/r03_t4.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03_t4.log | cut -c1-200
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_b4f.json 2> gpurun_out/r03_b4f.err || { tail -20 gpurun_out/r03_b4f.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r03_b4f.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["config"]["parallelism"], "densify", d["densify_iter_ms"], d["ordinary_iter_ms_alone"])
print({k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()})
P
