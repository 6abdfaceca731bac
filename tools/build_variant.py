#!/usr/bin/env python3
"""Build an A/B variant of librain_raster.so with extra compile definitions, into
gpurun_variants/<name>.so (git-ignored; travels to the GPU box with the snapshot).

    python tools/build_variant.py nostage -DRR_STAGE_SH=0
    python tools/build_variant.py prev --rev HEAD      (the sources of a git revision)
    python tools/build_variant.py probe --src DIR -DX  (sources from DIR/rain_amd/csrc, DIR/include)
    python tools/build_variant.py ilp @rr_blend.hip=-mllvm,-amdgpu-sched-strategy=max-ilp
                                                       (flags for one source only)
    python tools/build_variant.py lossx --lib librain_loss.so -DX   (another library of rain_amd/_build.py;
                                                       RAIN_LOSS_LIB selects it)
"""
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rain_amd import _build as B  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    csrc = B.CSRC
    if flags[:1] == ["--rev"]:
        rev, flags = flags[1], flags[2:]
        tmp = tempfile.mkdtemp(prefix="rr_rev_")
        arc = subprocess.run(["git", "-C", ROOT, "archive", rev, "rain_amd/csrc", "include"],
                             capture_output=True, check=True).stdout
        subprocess.run(["tar", "-x", "-C", tmp], input=arc, check=True)
        csrc, inc = os.path.join(tmp, "rain_amd", "csrc"), os.path.join(tmp, "include")
    elif flags[:1] == ["--src"]:
        tmp, flags = flags[1], flags[2:]
        csrc, inc = os.path.join(tmp, "rain_amd", "csrc"), os.path.join(tmp, "include")
    lib = "librain_raster.so"
    if flags[:1] == ["--lib"]:
        lib, flags = flags[1], flags[2:]
    per_file = {}  # @source=flag,flag: extra flags for that source only
    for f in [f for f in flags if f.startswith("@")]:
        src, _, fl = f[1:].partition("=")
        per_file.setdefault(src, []).extend(fl.split(","))
    flags = [f for f in flags if not f.startswith("@")]
    pre = ["-I", inc, "-I", csrc] if csrc != B.CSRC else []  # ahead of the tree's own include dirs
    out = os.path.join(ROOT, "gpurun_variants")
    objdir = os.path.join(out, name + "_obj")
    os.makedirs(objdir, exist_ok=True)
    srcs = B.LIBS[lib]

    def cc(s):
        src = os.path.join(csrc, s)
        obj = os.path.join(objdir, s.replace(".hip", ".o"))
        cmd = [B.HIPCC, *pre, *B.CXXFLAGS, *B.EXTRA.get(s, []), *flags, *per_file.get(s, []), "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr)
        return obj

    with ThreadPoolExecutor(max_workers=6) as ex:
        objs = list(ex.map(cc, srcs))
    target = os.path.join(out, name + ".so")
    r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", target, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    print(target)


if __name__ == "__main__":
    main()
