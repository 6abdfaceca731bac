#!/usr/bin/env python3
"""Turn two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE; separate runs because the TCC slots
cannot hold both) over tools/pmc_workload.py into profiles/pmc_traffic.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE, both in KiB as rocprofv3 reports them
(MI355X_MICROARCH.md, HBM section: on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
reads; WRITE_SIZE is exact for 16-B stores and dword atomics).  Infinity-Cache hits are counted,
so this is memory-side fabric traffic, an upper bound of HBM bytes.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics

STAGES = [  # kernel-name pattern -> bench.py stage name
    (r"k_blend_bwd", "blend_bwd"),
    (r"k_rs_scatter", "sort_scatter"),
    (r"k_rs_count", "sort_count"),
    (r"k_blend_fwd", "blend_fwd"),
    (r"k_preprocess", "preprocess"),
    (r"k_gauss_bwd", "gauss_bwd"),
    (r"k_duplicate", "duplicate"),
    (r"k_ranges", "ranges"),
]


def _stage(name):
    for pat, st in STAGES:
        if re.search(pat, name):
            return st
    return None


def _read(dirname, counter):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {dirname}")
    per = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                st = _stage(row.get("Kernel_Name", ""))
                if st is None:
                    continue
                key = (fn, row.get("Dispatch_Id"))
                per.setdefault(st, {}).setdefault(key, 0.0)
                per[st][key] += float(row["Counter_Value"])  # summed over XCD / instance rows
    return {st: list(d.values()) for st, d in per.items()}


SIMDS = 256 * 4       # MI355X: 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4       # peak engine clock (MI355X_MICROARCH.md)


def _valu_busy(dirname):
    """Fraction of SIMD issue cycles with a VALU instruction, per kernel: sum over waves of
    SQ_ACTIVE_INST_VALU (quad-cycles, x4) / (kernel duration x SIMDs x clock)."""
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    out = {}
    for fn in files:
        per = {}
        with open(fn) as f:
            for row in csv.DictReader(f):
                st = _stage(row.get("Kernel_Name", ""))
                if st is None:
                    continue
                key = row.get("Dispatch_Id")
                d = per.setdefault((st, key), {"dur": None})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                if row.get("End_Timestamp") and row.get("Start_Timestamp"):
                    d["dur"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        for (st, _), d in per.items():
            if d.get("dur") and "SQ_ACTIVE_INST_VALU" in d:
                o = out.setdefault(st, [0.0, 0.0])
                o[0] += 4.0 * d["SQ_ACTIVE_INST_VALU"]
                o[1] += d["dur"] * CLOCK_GHZ * SIMDS
    # time-weighted over the launches of a name (both forward-blend phases, whose durations and
    # occupancy differ a lot, count by their share of the time)
    return {st: v[0] / v[1] for st, v in out.items() if v[1] > 0}


def _inst_mix(dirname):
    """Per kernel (median over launches): wave-level VALU / SALU / LDS instruction counts, and (time-
    weighted over launches) the
    VALU issue fraction = SQ_INSTS_VALU x 2 cycles (a wave64 VALU op occupies a SIMD-32 for two
    cycles; transcendentals longer, so this is a lower bound) / (duration x 1024 SIMDs x clock)."""
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    acc = {}
    for fn in files:
        per = {}
        with open(fn) as f:
            for row in csv.DictReader(f):
                st = _stage(row.get("Kernel_Name", ""))
                if st is None:
                    continue
                d = per.setdefault((st, row.get("Dispatch_Id")), {"dur": None})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                if row.get("End_Timestamp") and row.get("Start_Timestamp"):
                    d["dur"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        for (st, _), d in per.items():
            if not d.get("dur") or "SQ_INSTS_VALU" not in d:
                continue
            r = acc.setdefault(st, {})
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES"):
                if k in d:
                    r.setdefault(k, []).append(d[k])
            r.setdefault("_valu_cycles", []).append(2.0 * d["SQ_INSTS_VALU"])
            r.setdefault("_simd_cycles", []).append(d["dur"] * CLOCK_GHZ * SIMDS)
    res = {}
    for st, r in acc.items():
        res[st] = {k.lower(): round(statistics.median(v), 0) for k, v in r.items() if not k.startswith("_")}
        res[st]["valu_issue_frac"] = round(sum(r["_valu_cycles"]) / sum(r["_simd_cycles"]), 4)  # time-weighted
    return res


def _trans(dirname):
    """Per kernel, time-weighted over launches: VALU issue fraction with transcendentals priced at
    twice a plain VALU op (MI355X_MICROARCH.md constants: v_exp / v_rcp / v_sqrt 8 cycles vs
    v_fma 4 for one wave's stream), (2 (VALU - TRANS) + 4 TRANS) cycles / (duration x SIMDs x clock),
    and the transcendental share of the VALU instructions."""
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    acc = {}
    for fn in files:
        per = {}
        with open(fn) as f:
            for row in csv.DictReader(f):
                st = _stage(row.get("Kernel_Name", ""))
                if st is None:
                    continue
                d = per.setdefault((st, row.get("Dispatch_Id")), {"dur": None})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                if row.get("End_Timestamp") and row.get("Start_Timestamp"):
                    d["dur"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        for (st, _), d in per.items():
            if not d.get("dur") or "SQ_INSTS_VALU" not in d or "SQ_INSTS_VALU_TRANS_F32" not in d:
                continue
            r = acc.setdefault(st, [0.0, 0.0, 0.0, 0.0])
            v, t = d["SQ_INSTS_VALU"], d["SQ_INSTS_VALU_TRANS_F32"]
            r[0] += 2.0 * (v - t) + 4.0 * t
            r[1] += d["dur"] * CLOCK_GHZ * SIMDS
            r[2] += t
            r[3] += v
    return {st: {"valu_issue_frac_trans_weighted": round(r[0] / r[1], 4),
                 "trans_share_of_valu": round(r[2] / r[3], 4) if r[3] else None}
            for st, r in acc.items() if r[1] > 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--sq-dir", default=None, help="a third pass with SQ_ACTIVE_INST_VALU (VALU busy)")
    ap.add_argument("--inst-dir", default=None, help="a pass with SQ_INSTS_VALU/SALU/LDS and SQ_WAVES")
    ap.add_argument("--trans-dir", default=None, help="a pass with SQ_INSTS_VALU and SQ_INSTS_VALU_TRANS_F32")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = _read(a.fetch_dir, "FETCH_SIZE")
    write = _read(a.write_dir, "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE over tools/pmc_workload.py "
                     "(the bench training step: 1M Gaussians, SH 3, 1920x1080, fused Adam); hbm = 2*FETCH + WRITE (gfx950 correction)",
           "unit": "bytes per launch (median over launches)", "kernels": {}}
    for st in sorted(set(fetch) | set(write)):
        f = statistics.median(fetch[st]) * 1024.0 if st in fetch else None
        w = statistics.median(write[st]) * 1024.0 if st in write else None
        out["kernels"][st] = {
            "launches": len(fetch.get(st, [])),
            "fetch_bytes_raw": f, "write_bytes": w,
            "hbm_bytes_per_launch": (2 * f + w) if (f is not None and w is not None) else None,
        }
    if a.sq_dir:
        out["valu_busy_note"] = ("sum of SQ_ACTIVE_INST_VALU quad-cycles x4 / (kernel duration x 1024 SIMDs x "
                                 f"{CLOCK_GHZ} GHz): fraction of SIMD cycles issuing a VALU op")
        for st, v in _valu_busy(a.sq_dir).items():
            out["kernels"].setdefault(st, {})["valu_busy"] = round(v, 3)
    if a.inst_dir:
        out["inst_note"] = ("wave-level instruction counts per launch (SQ_INSTS_*); valu_issue_frac = "
                            f"SQ_INSTS_VALU x 2 cycles / (duration x 1024 SIMDs x {CLOCK_GHZ} GHz)")
        for st, v in _inst_mix(a.inst_dir).items():
            out["kernels"].setdefault(st, {}).update(v)
    if a.trans_dir:
        out["trans_note"] = ("valu_issue_frac_trans_weighted = (2 x non-transcendental + 4 x transcendental "
                             f"VALU wave instructions) cycles / (duration x 1024 SIMDs x {CLOCK_GHZ} GHz)")
        for st, v in _trans(a.trans_dir).items():
            out["kernels"].setdefault(st, {}).update(v)
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
