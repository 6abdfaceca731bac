# round-3 continuation final: -m gpu suite, smoke, default bench, rocprofv3 kernel stats + PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03d_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r03d_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_smoke.log 2>&1 || { tail -20 gpurun_out/r03d_smoke.log; exit 1; }
tail -1 gpurun_out/r03d_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || { tail -20 gpurun_out/r03d_bench.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r03d_bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(d["value"], d["ms_per_step"], "densify", d.get("densify_iter_ms"), d.get("ordinary_iter_ms_alone"), "api", d["api_iters_per_s"], "cpu", d["cpu_baseline"]["value"])
print({k: r[k] for k in ("kernel", "achieved", "frac", "measured_copy_GBps", "measured_rmw_GBps")})
print({k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()})
P
bash tools/profile_round.sh gpurun_out/prof_r03d && python3 tools/step_breakdown.py gpurun_out/prof_r03d/bench > gpurun_out/prof_r03d/step_breakdown.txt 2>&1 && python3 tools/step_breakdown.py gpurun_out/prof_r03d/bench --seq > gpurun_out/prof_r03d/launch_sequence.txt 2>&1
head -4 gpurun_out/prof_r03d/step_breakdown.txt
