set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02v5_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02v5_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02v5_gpu_tests.log
for v in head prev head prev; do
  if [ $v = prev ]; then export RAIN_RASTER_LIB=$PWD/gpurun_variants/prev.so; else unset RAIN_RASTER_LIB; fi
  rm -rf /tmp/ab_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/ab_$v -o run -- python3 bench.py --steps 300 --warmup 30 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 - "$v" /tmp/ab_$v gpurun_out/ab_$v.json <<'PY'
import sys, json, glob, csv
v, d, j = sys.argv[1:]
b = json.loads(open(j).read().strip().splitlines()[-1])
out = [f"{v}: {b['value']:.1f} it/s"]
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("k_duplicate", "k_preprocess", "k_expand")):
            out.append(f"{r['Name'][:40]} calls {r['Calls']} avg {float(r['AverageNs'])/1e3:.2f} us")
print("; ".join(out))
PY
  mkdir -p gpurun_out/ab_stats_$v && cp $(find /tmp/ab_$v -name '*kernel_stats.csv') gpurun_out/ab_stats_$v/ 2>/dev/null
done
unset RAIN_RASTER_LIB
bash tools/profile_round.sh gpurun_out/prof_r02v5 || exit 1
python3 tools/step_breakdown.py gpurun_out/prof_r02v5/bench > gpurun_out/prof_r02v5/step_breakdown.txt
timeout -k 10 300 python bench.py > gpurun_out/r02v5_bench_full.json 2> gpurun_out/r02v5_bench_full.err || exit 1
tail -1 gpurun_out/r02v5_bench_full.json | cut -c1-200
du -sh gpurun_out
