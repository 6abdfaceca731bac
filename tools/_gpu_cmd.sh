set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
for v in head prev head prev; do
  if [ $v = prev ]; then export RAIN_RASTER_LIB=$PWD/gpurun_variants/prev.so; else unset RAIN_RASTER_LIB; fi
  rm -rf /tmp/ab_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ab_$v -o run -- python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 - "$v" /tmp/ab_$v gpurun_out/ab_$v.json <<'PY'
import sys, json, glob, csv
v, d, j = sys.argv[1:]
b = json.loads(open(j).read().strip().splitlines()[-1])
k = b['kernels']
out = [f"{v}: {b['value']:.1f} it/s " + " ".join(f"{n} {k[n]['ms_per_step']*1e3:.1f}" for n in ("preprocess","depth_sort","scan","duplicate"))]
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("k_rs_count<unsigned int", "k_publish")):
            out.append(f"  {r['Name'][:48]} calls {r['Calls']} avg {float(r['AverageNs'])/1e3:.2f} us")
print("\n".join(out))
PY
done
