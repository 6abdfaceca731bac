set -o pipefail
mkdir -p gpurun_out/apitrace
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/apitrace -o run --output-format csv -- python3 tools/api_profile.py --steps 20 > gpurun_out/apitrace/log.txt 2>&1
python3 - <<'P'
import csv, glob, collections
f = glob.glob("gpurun_out/apitrace/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last 20 API steps + 10 synced + 10 profiled = 40 steps: take the window after the first 5 warmup steps
agg = collections.defaultdict(lambda: [0, 0])
n = len(rows)
tail = rows[int(n * 0.5):]
span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
busy = 0
for r in tail:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy += d
    k = r["Kernel_Name"][:100]
    agg[k][0] += d
    agg[k][1] += 1
print(f"window {span:.1f} us, busy {busy:.1f} us")
for k, (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:30]:
    print(f"{d:10.1f} us {c:5d}  {k}")
P
