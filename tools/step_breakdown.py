"""Per-training-step kernel breakdown from a rocprofv3 kernel trace (csv).

Default: steps are delimited by the backward blend kernel; prints the mean step period and the mean
time per step of every kernel name, heaviest first.

--window: only the launches between bench.py's trace markers (k_trace_mark_begin / k_trace_mark_end,
rt_trace_marker: the K steps of the timed loop and nothing else — no warm-up, no profiled window,
no bracket / API / forward-only legs).  Prints, per kernel name, the calls, total, average, min and
max duration over that window (the rocprofv3 --stats columns restricted to the timed loop) and the
per-step figures; --json writes the same as a file.  bench.py's roofline `ms_per_launch` (HIP events
around the same launches) should agree with the average printed for its kernel.

    python tools/step_breakdown.py gpurun_out/prof_x [--first 100 --count 80] [--seq]
    python tools/step_breakdown.py gpurun_out/prof_x --window [--json profiles/r04_timed_kernels.json]
"""
import argparse
import collections
import csv
import glob
import json
import os


def _name(x):
    return x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]


def _dur(x):
    return (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000.0  # us


def window(rows, json_out=None):
    b = [i for i, x in enumerate(rows) if "k_trace_mark_begin" in x["Kernel_Name"]]
    e = [i for i, x in enumerate(rows) if "k_trace_mark_end" in x["Kernel_Name"]]
    if not b or not e:
        raise SystemExit("no trace markers in this trace (bench.py of round 4 or later emits them)")
    i0 = b[-1]
    i1 = min(j for j in e if j > i0)
    seg = rows[i0 + 1:i1]
    span = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["End_Timestamp"])) / 1000.0
    steps = sum(1 for x in seg if "k_blend_bwd" in x["Kernel_Name"])
    st = collections.OrderedDict()
    for x in seg:
        d = _dur(x)
        s = st.setdefault(_name(x), {"calls": 0, "total_us": 0.0, "min_us": 1e30, "max_us": 0.0})
        s["calls"] += 1
        s["total_us"] += d
        s["min_us"] = min(s["min_us"], d)
        s["max_us"] = max(s["max_us"], d)
    busy = sum(s["total_us"] for s in st.values())
    out = {"window": "launches between k_trace_mark_begin and k_trace_mark_end (bench.py timed loop)",
           "steps": steps, "launches": len(seg), "span_us": round(span, 1),
           "us_per_step": round(span / max(steps, 1), 2), "busy_us_per_step": round(busy / max(steps, 1), 2),
           "kernels": {}}
    print(f"timed window: {steps} steps, {len(seg)} launches, span {span:.1f} us = {span / max(steps, 1):.1f} us/step, "
          f"kernel-busy {busy / max(steps, 1):.1f} us/step")
    print(f"{'calls':>6} {'total_us':>10} {'avg_us':>8} {'min_us':>8} {'max_us':>8} {'us/step':>8}  kernel")
    for k, s in sorted(st.items(), key=lambda kv: -kv[1]["total_us"]):
        s["avg_us"] = s["total_us"] / s["calls"]
        s["us_per_step"] = s["total_us"] / max(steps, 1)
        out["kernels"][k] = {kk: round(v, 3) if isinstance(v, float) else v for kk, v in s.items()}
        print(f"{s['calls']:6d} {s['total_us']:10.1f} {s['avg_us']:8.2f} {s['min_us']:8.2f} {s['max_us']:8.2f} "
              f"{s['us_per_step']:8.2f}  {k}")
    if json_out:
        with open(json_out, "w") as f:
            json.dump(out, f, indent=1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--first", type=int, default=30)
    ap.add_argument("--count", type=int, default=99)
    ap.add_argument("--seq", action="store_true", help="per launch position of a step: mean duration and gap")
    ap.add_argument("--window", action="store_true", help="only bench.py's timed loop (trace markers)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
    if a.window:
        window(rows, a.json)
        if not a.seq:
            return
        b = max(i for i, x in enumerate(rows) if "k_trace_mark_begin" in x["Kernel_Name"])
        e = min(i for i, x in enumerate(rows) if "k_trace_mark_end" in x["Kernel_Name"] and i > b)
        rows = rows[b + 1:e]
        a.first, a.count = 0, 10 ** 9
    idx = [i for i, x in enumerate(rows) if "k_blend_bwd" in x["Kernel_Name"]]
    agg = collections.defaultdict(float)
    period = 0.0
    steps = 0
    for s in range(a.first, min(a.first + a.count, len(idx) - 1)):
        seg = rows[idx[s] + 1: idx[s + 1] + 1]
        period += (int(rows[idx[s + 1]]["End_Timestamp"]) - int(rows[idx[s]]["End_Timestamp"])) / 1000
        steps += 1
        for x in seg:
            agg[_name(x)[:70]] += _dur(x)
    if a.seq:  # steps with the modal launch count: mean duration / gap before each launch position
        segs = [rows[idx[s] + 1: idx[s + 1] + 1] for s in range(a.first, min(a.first + a.count, len(idx) - 1))]
        n = collections.Counter(len(g) for g in segs).most_common(1)[0][0]
        segs = [g for g in segs if len(g) == n]
        print(f"launch sequence over {len(segs)} steps of {n} launches (us: duration, gap before)")
        for j in range(n):
            d = sum(_dur(g[j]) for g in segs) / len(segs)
            gp = sum(int(g[j]["Start_Timestamp"]) - int(g[j - 1]["End_Timestamp"]) for g in segs) / len(segs) / 1000 if j else 0.0
            print(f"{j:3d} {d:8.1f} {gp:7.1f}  {_name(segs[0][j])[:60]}")
    if a.window:
        return
    busy = sum(agg.values()) / steps
    print(f"steps {steps}  period {period / steps:.1f} us  busy {busy:.1f} us")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"{v / steps:8.1f}  {k}")


if __name__ == "__main__":
    main()
