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
    ap.add_argument("--seq", action="store_true", help="per launch position of a step: mean duration and gap")
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
    if a.seq:  # steps with the modal launch count: mean duration / gap before each launch position
        segs = [rows[idx[s] + 1: idx[s + 1] + 1] for s in range(a.first, min(a.first + a.count, len(idx) - 1))]
        n = collections.Counter(len(g) for g in segs).most_common(1)[0][0]
        segs = [g for g in segs if len(g) == n]
        prev_end = [int(rows[idx[a.first + i]]["End_Timestamp"]) for i in range(len(segs))]
        print(f"launch sequence over {len(segs)} steps of {n} launches (us: duration, gap before)")
        for j in range(n):
            d = sum(int(g[j]["End_Timestamp"]) - int(g[j]["Start_Timestamp"]) for g in segs) / len(segs) / 1000
            gp = sum(int(g[j]["Start_Timestamp"]) - (int(g[j - 1]["End_Timestamp"]) if j else 0) for g in segs) / len(segs) / 1000 if j else 0.0
            nm = segs[0][j]["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
            print(f"{j:3d} {d:8.1f} {gp:7.1f}  {nm}")
    busy = sum(agg.values()) / steps
    print(f"steps {steps}  period {period / steps:.1f} us  busy {busy:.1f} us")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"{v / steps:8.1f}  {k}")


if __name__ == "__main__":
    main()
