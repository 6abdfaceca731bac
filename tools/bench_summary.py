"""One-screen summary of a bench.py JSON line: python tools/bench_summary.py gpurun_out/x_bench.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(f"value {d['value']} it/s  ms/step {d['ms_per_step']}  1in100 {d.get('iters_per_s_1in100')}  "
      f"densify {d.get('densify_iter_ms')} / ordinary {d.get('ordinary_iter_ms_alone')} ms  api {d.get('api_iters_per_s')}  "
      f"bracket {d.get('bracket_iters_per_s')}  fwd Mpix/s {d.get('forward_mpix_per_s')}")
print({k: r.get(k) for k in ("kernel", "achieved", "frac", "ms_per_launch", "measured_rmw_GBps", "frac_of_measured_rmw")})
print({k: round(v["ms_per_step"], 4) for k, v in d.get("kernels", {}).items()})
c = d.get("cpu_baseline")
if c:
    print("cpu", {k: c.get(k) for k in ("value", "unit", "cores", "kind")})
