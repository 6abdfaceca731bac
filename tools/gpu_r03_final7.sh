# final tree: smoke + default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03e_smoke.log 2>&1 || { tail -20 gpurun_out/r03e_smoke.log; exit 1; }
tail -1 gpurun_out/r03e_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err || { tail -20 gpurun_out/r03e_bench.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r03e_bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(d["value"], d["ms_per_step"], "densify", d.get("densify_iter_ms"), d.get("ordinary_iter_ms_alone"), "api", d["api_iters_per_s"])
print({k: r[k] for k in ("kernel", "achieved", "frac", "measured_rmw_GBps")})
print({k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()})
P
