# round-3 final: full -m gpu suite, smoke, default bench, forced-dist (RCCL one-rank) bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03_final_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r03_final_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_final_smoke.log 2>&1 || { tail -20 gpurun_out/r03_final_smoke.log; exit 1; }
tail -1 gpurun_out/r03_final_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03_final_bench.json 2> gpurun_out/r03_final_bench.err || { tail -20 gpurun_out/r03_final_bench.err; exit 1; }
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03_final_bench_dist.json 2> gpurun_out/r03_final_bench_dist.err || { tail -20 gpurun_out/r03_final_bench_dist.err; exit 1; }
python3 - <<'P'
import json
for f in ("gpurun_out/r03_final_bench.json", "gpurun_out/r03_final_bench_dist.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], d["config"]["parallelism"], "densify", d.get("densify_iter_ms"), "api", d["api_iters_per_s"], d.get("api_torch_adam_iters_per_s"))
    print("  ", {k: r[k] for k in ("kernel", "achieved", "frac", "measured_copy_GBps", "measured_rmw_GBps", "frac_of_measured_rmw")})
    print("  ", {k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()})
P
