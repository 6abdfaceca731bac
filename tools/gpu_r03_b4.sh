set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/r03_b4.json 2> gpurun_out/r03_b4.err || { tail -20 gpurun_out/r03_b4.err; exit 1; }
timeout -k 10 600 python -u bench.py --points 5000000 --width 3840 --height 2160 --aux-normal --steps 30 --no-cpu-baseline > gpurun_out/r03_b4_cfg5.json 2> gpurun_out/r03_b4_cfg5.err || { tail -20 gpurun_out/r03_b4_cfg5.err; exit 1; }
python3 - <<'P'
import json
for f in ("gpurun_out/r03_b4.json", "gpurun_out/r03_b4_cfg5.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], "densify", d.get("densify_iter_ms"), "api", d["api_iters_per_s"], d.get("api_torch_adam_iters_per_s"), "fwd", d["forward_mpix_per_s"])
    print("  ", {k: r[k] for k in ("kernel", "achieved", "frac", "measured_copy_GBps", "measured_rmw_GBps", "frac_of_measured_rmw")})
    print("  ", {k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()})
P
