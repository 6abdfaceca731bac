#!/usr/bin/env python3
"""Per-pair instruction budget of the backward blend's pair loop (k_blend_bwd), from the
gfx950 assembly of rain_amd/csrc/rr_blend.hip.

The pair loop is the innermost loop of the kernel.  Its basic blocks are sorted into roles:
  * pixel body q  — a block entered under a per-pixel exec mask that holds the pixel's v_rcp_f32
                    (the transmittance recovery and the gradient terms of one pixel of the lane);
  * per-pair      — every other block of the loop (record reads from LDS, the four alphas, the
                    nine per-lane sums, the wave reduction, the LDS store of the reduced values,
                    and the exec-mask set-up of the four pixel bodies).
Instructions are classed by opcode (VALU arithmetic, transcendental, DPP / permlane cross-lane,
compare / select, LDS, SALU, branch, wait / nop).  The per-pair blocks run once per (tile, pair);
a pixel body runs when any lane of the wave has that pixel active.  With the measured VALU
instructions per (tile, pair) from the PMC pass (SQ_INSTS_VALU / L_eff) the number of pixel
bodies a pair executes on average follows:  valu = per_pair_valu + k * body_valu.

    python tools/isa_budget.py [--valu-per-pair 158.6] [--define MACRO=VALUE] [--out FILE]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KERNEL = "_ZN2rr11k_blend_bwdENS_12BlendBwdArgsE"


def opclass(op):
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait/nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("v_permlane", "v_readlane", "v_writelane")) or op.endswith("_dpp"):
        return "xlane"
    if op.startswith(("v_exp", "v_rcp", "v_sqrt", "v_rsq", "v_log")):
        return "trans"
    if op.startswith(("v_cmp", "v_cndmask")):
        return "cmp/sel"
    if op.startswith("v_"):
        return "valu"
    return "other"


def assemble(defines):
    from rain_amd import _build as B

    out = os.path.join(tempfile.mkdtemp(), "blend.s")
    cmd = [B.HIPCC, *B.CXXFLAGS, *B.EXTRA["rr_blend.hip"], *[f"-D{d}" for d in defines], "--offload-device-only",
           "-S", os.path.join(B.CSRC, "rr_blend.hip"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    with open(out) as f:
        return f.read().splitlines()


def loop_blocks(lines):
    """Basic blocks of the kernel's innermost loop: [(label, [(op, text)])]."""
    start = next(i for i, l in enumerate(lines) if l.startswith(KERNEL + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end + 1]
    blocks, cur = [], None
    for l in body:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?", l)
        if m:
            cur = [m.group(1), l, []]
            blocks.append(cur)
            continue
        s = l.strip()
        if cur is not None and not cur[2] and s.startswith(";"):
            cur[1] += " " + s  # the label's loop annotation continues on comment lines
            continue
        if not s or s.startswith(";") or s.startswith(".") or cur is None:
            continue
        op = s.split()[0]
        cur[2].append((op, s))
    # innermost loop: blocks annotated "in Loop: Header=BBx Depth=2" (or the header itself)
    hdr = next(b for b in blocks if "Inner Loop Header" in b[1])
    m = re.search(r"Loop Header: Depth=(\d+)", hdr[1])
    depth = m.group(1)
    hname = hdr[0].replace(".LBB", "BB")
    inloop = [b for b in blocks if b is hdr or (f"Header={hname} Depth={depth}" in b[1])]
    return inloop


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--valu-per-pair", type=float, default=None,
                    help="measured VALU instructions per (tile, pair): SQ_INSTS_VALU per launch / L_eff")
    ap.add_argument("--define", action="append", default=[])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    blocks = loop_blocks(assemble(a.define))
    per_pair, body = Counter(), Counter()
    nbodies = 0
    rows = []
    for label, _, ins in blocks:
        c = Counter(opclass(op) for op, _ in ins)
        is_body = any(op.startswith("v_rcp") for op, _ in ins)
        if is_body:
            nbodies += 1
            body += c
        else:
            per_pair += c
        rows.append((label, "pixel body" if is_body else "per-pair", len(ins), dict(c)))
    classes = ["valu", "trans", "xlane", "cmp/sel", "lds", "salu", "branch", "wait/nop"]
    out = []
    out.append(f"k_blend_bwd<1,3> pair loop ({'; '.join(a.define) or 'default build'}): {len(blocks)} basic blocks, "
               f"{nbodies} pixel bodies")
    out.append("")
    out.append(f"{'block':<14} {'role':<11} {'instrs':>6}  " + " ".join(f"{c:>8}" for c in classes))
    for label, role, n, c in rows:
        out.append(f"{label:<14} {role:<11} {n:>6}  " + " ".join(f"{c.get(k, 0):>8}" for k in classes))
    out.append("")
    vb = body["valu"] + body["trans"] + body["xlane"] + body["cmp/sel"]
    vp = per_pair["valu"] + per_pair["trans"] + per_pair["xlane"] + per_pair["cmp/sel"]
    bodies = max(nbodies, 1)
    out.append("per (tile, pair), static:")
    out.append("  per-pair blocks : " + ", ".join(f"{k} {per_pair.get(k, 0)}" for k in classes) + f"  (VALU-class {vp})")
    out.append("  one pixel body  : " + ", ".join(f"{k} {body.get(k, 0) / bodies:.1f}" for k in classes)
               + f"  (VALU-class {vb / bodies:.1f})")
    out.append(f"  VALU-class if all {nbodies} bodies run: {vp + vb}")
    if a.valu_per_pair:
        k = (a.valu_per_pair - vp) / (vb / bodies)
        out.append(f"measured VALU per (tile, pair) {a.valu_per_pair:.1f} -> pixel bodies executed per pair "
                   f"k = {k:.2f} of {nbodies}")
        out.append(f"  -> per pair: {vp} per-pair VALU ({100 * vp / a.valu_per_pair:.0f} %), "
                   f"{k * vb / bodies:.1f} pixel-body VALU ({100 * k * vb / bodies / a.valu_per_pair:.0f} %)")
        xl = per_pair["xlane"]
        out.append(f"  of the per-pair VALU: cross-lane reduction {xl}, alpha / record set-up and sums "
                   f"{per_pair['valu'] + per_pair['trans']}, compares {per_pair['cmp/sel']}")
    text = "\n".join(out)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
