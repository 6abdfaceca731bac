"""Per-training-step kernel breakdown from a rocprofv3 kernel trace (csv).

Steps are delimited by the backward blend kernel; prints the mean step period and the mean time
per step of every kernel name, heaviest first.  The defaults cover bench.py's timed loop of the
default run (10 warmup + 20 stage-profiled steps, then the 100 timed ones; the bracket and
reference-API legs that follow run different kernels).

    python tools/step_breakdown.py gpurun_out/prof_x [--first 100 --count 80]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--first", type=int, default=30)
    ap.add_argument("--count", type=int, default=99)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
    idx = [i for i, x in enumerate(rows) if "k_blend_bwd" in x["Kernel_Name"]]
    agg = collections.defaultdict(float)
    period = 0.0
    steps = 0
    for s in range(a.first, min(a.first + a.count, len(idx) - 1)):
        seg = rows[idx[s] + 1: idx[s + 1] + 1]
        period += (int(rows[idx[s + 1]]["End_Timestamp"]) - int(rows[idx[s]]["End_Timestamp"])) / 1000
        steps += 1
        for x in seg:
            agg[x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]] += (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000
    busy = sum(agg.values()) / steps
    print(f"steps {steps}  period {period / steps:.1f} us  busy {busy:.1f} us")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"{v / steps:8.1f}  {k}")


if __name__ == "__main__":
    main()
