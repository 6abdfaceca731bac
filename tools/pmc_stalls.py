#!/usr/bin/env python3
"""Where a kernel's wave cycles go, from one rocprofv3 SQ counter pass:

    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \\
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \\
        --kernel-trace -d gpurun_out/pmc_stall -o run --output-format csv -- python3 tools/pmc_workload.py
    python tools/pmc_stalls.py gpurun_out/pmc_stall [--match blend]

Per (kernel, grid size), medians over dispatches:
  occupancy   mean resident waves per SIMD = SQ_WAVE_CYCLES x 4 / (duration x clock x 1024 SIMDs)
  wait / issue_stall / active   shares of wave cycles (SQ_WAIT_ANY: parked on s_waitcnt or a barrier;
              SQ_WAIT_INST_ANY: ready but not issued; SQ_ACTIVE_INST_ANY: issuing) — they add to ~1
  valu / lds  SQ_ACTIVE_INST_VALU / _LDS per SIMD cycle (x4 quad-cycles / SIMDs)
  clock_GHz   GRBM_GUI_ACTIVE / 8 XCDs / duration (reads high on short dispatches)
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics

SIMDS = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--json", default=None)
    ap.add_argument("--min-us", type=float, default=0.0, help="only dispatches at least this long")
    a = ap.parse_args()
    per = {}
    for fn in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if a.match and not re.search(a.match, name):
                    continue
                key = (re.sub(r"\(.*", "", name)[:80], int(row["Grid_Size"]))
                d = per.setdefault(key, {}).setdefault((fn, row["Dispatch_Id"]), {})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                d["dur_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    out = {}
    for (kname, grid), disp in sorted(per.items(), key=lambda kv: -sum(d["dur_ns"] for d in kv[1].values())):
        rows = []
        for d in disp.values():
            dur = d["dur_ns"]
            if dur <= 0 or dur < a.min_us * 1e3:
                continue
            clk = d.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 / dur if d.get("GRBM_GUI_ACTIVE") else 2.1
            cyc = dur * clk
            wc = d.get("SQ_WAVE_CYCLES", 0.0)
            r = {"dur_us": dur / 1e3, "clock_GHz": clk, "occupancy": wc * 4 / (cyc * SIMDS) if cyc else None}
            if wc:
                r["wait"] = d.get("SQ_WAIT_ANY", 0.0) / wc
                r["issue_stall"] = d.get("SQ_WAIT_INST_ANY", 0.0) / wc
                r["active"] = d.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
                r["lds_issue_stall"] = d.get("SQ_WAIT_INST_LDS", 0.0) / wc
            if cyc:
                r["valu"] = d.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / (cyc * SIMDS)
                r["lds"] = d.get("SQ_ACTIVE_INST_LDS", 0.0) * 4 / (cyc * SIMDS)
                r["busy"] = d.get("SQ_BUSY_CYCLES", 0.0) * 4 / cyc / 8 if d.get("SQ_BUSY_CYCLES") else None
            rows.append(r)
        if not rows:
            continue
        med = {k: statistics.median([r[k] for r in rows if r.get(k) is not None])
               for k in rows[0] if any(r.get(k) is not None for r in rows)}
        med["dispatches"] = len(rows)
        out[f"{kname} grid={grid}"] = {k: round(v, 4) if isinstance(v, float) else v for k, v in med.items()}
    for k, v in out.items():
        print(k)
        print("   ", "  ".join(f"{kk}={vv}" for kk, vv in v.items()))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
