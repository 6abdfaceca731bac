set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r03_b3.json 2> gpurun_out/r03_b3.err || { tail -20 gpurun_out/r03_b3.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r03_b3.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(d["value"], d["ms_per_step"], "densify", d.get("densify_iter_ms"), "api", d["api_iters_per_s"], d["api_torch_adam_iters_per_s"])
print({k: r[k] for k in ("kernel", "achieved", "frac", "measured_copy_GBps", "measured_rmw_GBps", "frac_of_measured_rmw", "ms_per_launch")})
print({k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()})
print("cpu", d["cpu_baseline"])
P
