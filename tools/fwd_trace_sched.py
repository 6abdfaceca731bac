#!/usr/bin/env python3
"""Offline analysis of forward-blend wave timelines (tools/fwd_trace.py's gpurun_out/fwd_trace*.npy):
how long phase A drains, and how much a dispatch order by a per-tile predictor known before the
blend would recover, by list-scheduling the measured workgroup durations (a tile's workgroup runs
as long as its slower wave) on the observed concurrency.

    python tools/fwd_trace_sched.py gpurun_out/fwd_trace*.npy [--gx 120]
"""
import argparse
import heapq

import numpy as np


def phase_records(rec, phase):
    r = rec[(rec[:, 7] & 0xFF) == phase]
    return r[(r[:, 0] | r[:, 1]) != 0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--gx", type=int, default=120)
    a = ap.parse_args()
    for f in a.files:
        rec = np.load(f)
        r = phase_records(rec, 1)
        if len(r) == 0:
            r = phase_records(rec, 0)
        start = (r[:, 1].astype(np.uint64) << np.uint64(32)) | r[:, 0].astype(np.uint64)
        end = (r[:, 3].astype(np.uint64) << np.uint64(32)) | r[:, 2].astype(np.uint64)
        t0 = start.min()
        s = (start - t0).astype(np.float64) * 0.01
        e = (end - t0).astype(np.float64) * 0.01
        tile = r[:, 4].astype(np.int64)
        walked, n = r[:, 5].astype(np.int64), r[:, 6].astype(np.int64)
        # per tile (workgroup): start, end, list length, pairs walked by its slower wave
        tiles = np.unique(tile)
        idx = {t: i for i, t in enumerate(tiles)}
        ws = np.full(len(tiles), np.inf)
        we = np.zeros(len(tiles))
        wn = np.zeros(len(tiles), np.int64)
        ww = np.zeros(len(tiles), np.int64)
        for k in range(len(r)):
            i = idx[tile[k]]
            ws[i] = min(ws[i], s[k])
            we[i] = max(we[i], e[k])
            wn[i] = n[k]
            ww[i] = max(ww[i], walked[k])
        d = we - ws
        span = we.max()
        edges = np.linspace(0, span, 41)
        live = np.array([int(((ws <= t) & (we > t)).sum()) for t in edges[:-1] + (edges[1] - edges[0]) / 2])
        slots = int(live.max())

        def sched(order):
            h = [0.0] * slots
            for i in order:
                t = heapq.heappop(h)
                heapq.heappush(h, t + d[i])
            return max(h)

        ty = tiles // a.gx
        tx = tiles % a.gx
        preds = {
            "launch order": np.argsort(ws, kind="stable"),
            "longest list": np.argsort(-wn, kind="stable"),
            "shortest list": np.argsort(wn, kind="stable"),
            "bottom rows first": np.argsort(-ty, kind="stable"),
            "top rows first": np.argsort(ty, kind="stable"),
            "oracle": np.argsort(-d, kind="stable"),
        }
        # fraction of the span with fewer than half the peak workgroups running
        drain = float((live < 0.5 * slots).mean()) * span
        print(f"{f}: {len(tiles)} tiles, span {span:.1f} us, peak {slots} workgroups, "
              f"< half-peak for {drain:.1f} us; duration p50 {np.median(d):.1f} p99 {np.percentile(d, 99):.1f} "
              f"max {d.max():.1f} us")
        print("  " + ", ".join(f"{k} {sched(v):.1f}" for k, v in preds.items()))
        for name, x in (("list length", wn), ("walked", ww), ("tile row", ty), ("tile col", tx)):
            print(f"  corr(duration, {name}) {np.corrcoef(d, x)[0, 1]:+.2f}")
        # duration by tile row band (8 bands)
        bands = np.array_split(np.argsort(ty, kind="stable"), 8)
        print("  mean duration by row band (top..bottom): " + " ".join(f"{d[b].mean():.1f}" for b in bands))
        q = np.argsort(-d)[: max(1, len(d) // 20)]
        print(f"  slowest 5%: mean list {wn[q].mean():.0f} (all {wn.mean():.0f}), mean walked {ww[q].mean():.0f} "
              f"(all {ww.mean():.0f}), mean row {ty[q].mean():.1f} (all {ty.mean():.1f}), "
              f"walked == list in {100 * float((ww[q] >= wn[q]).mean()):.0f}% (all {100 * float((ww >= wn).mean()):.0f}%)")


if __name__ == "__main__":
    main()
