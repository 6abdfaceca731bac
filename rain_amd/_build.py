"""Ahead-of-time build of the HIP rasterizer (replaces the reference's import-time JIT,
submodules/diff_gaussian_rasterization/setup.py:8-19).

Compiles rain_amd/csrc/*.hip for gfx950 with hipcc and links ``rain_amd/lib/librain_raster.so``
(C ABI: include/rain_raster.h).  The .so lives in-tree so it travels to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(PKG, "lib", "obj")

ARCH = os.environ.get("RAIN_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
CXXFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
            "-I", os.path.join(ROOT, "include"), "-I", CSRC]

LIBS = {
    "librain_raster.so": ["rr_forward.hip", "rr_bin.hip", "rr_blend_fwd_s.hip", "rr_blend.hip", "rr_backward.hip",
                          "rr_sort.hip", "rr_api.hip"],
    "librain_loss.so": ["loss.hip"],
    "librain_knn.so": ["knn.hip"],
    "librain_train.so": ["train.hip", "densify.hip"],
}


# Per-source extra device flags.  rr_blend.hip: no packed-fp32 (v_pk_*) formation — in the blend
# loops hipcc pairs unrelated scalars into v_pk ops and pays for it with v_mov shuffles and ~30
# extra VGPRs (measured: 132 vs 166 VGPRs, 537 vs 602 instructions in k_blend_bwd<1>).
# loss.hip: the SSIM kernels' band loop must unroll fully (compile-time ring / queue slots) and is
# larger than clang's default pragma-unroll size limit; packed-fp32 formation is off for the same
# reason as rr_blend.hip (it pairs unrelated scalars: 940 v_mov, 244 VGPRs in k_ssim_fwd).
# rr_forward.hip / rr_backward.hip: floating-point contraction only inside one source expression
# (llvm.fmuladd), not across statements by the backend — the forward preprocess and the next
# frame's preprocess inside the per-Gaussian backward (rr_preprocess.hpp, include/rain_raster.h
# rr_next_frame) then compile the same arithmetic to the same fma sequence in both kernels, so the
# fused geometry is bitwise the forward's.
# rr_blend.hip / rr_backward.hip: LLVM's max-ILP machine scheduler instead of the default
# occupancy-driven one (same VGPR budget here: both kernels' occupancy is set elsewhere — the
# backward blend's 4 waves, the Gaussian backward's LDS rows); it interleaves the independent chains
# of a pair's alphas and a row's terms further: blend bwd 0.227 -> 0.221 ms, Gaussian bwd 0.326 ->
# 0.324, step -8 us (profiles/r06ah_sched_ilp_ab.jsonl; on the forward blend, the binning and the
# SSIM sources it measured neutral or slower, r06ag / r06ah)
MAX_ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
CONTRACT_ON = ["-ffp-contract=on"]
EXTRA = {
    "rr_forward.hip": CONTRACT_ON,
    "rr_backward.hip": CONTRACT_ON + MAX_ILP,
    # rr_blend_fwd_s.hip: machine sinking would move the software-pipelined next-group record loads
    # below the blend (next to their use in the loop latch), serialising them again
    "rr_blend_fwd_s.hip": ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "-mllvm", "-disable-machine-sink"],
    "rr_blend.hip": ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"] + MAX_ILP,
    "loss.hip": ["-mllvm", "-pragma-unroll-threshold=200000",
                 "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"],
}


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    hs += [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    return hs


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src, obj, verbose):
    cmd = [HIPCC, *CXXFLAGS, *EXTRA.get(os.path.basename(src), []), "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False) -> dict:
    os.makedirs(OBJDIR, exist_ok=True)
    headers = _headers()
    jobs = []
    for lib, srcs in LIBS.items():
        for s in srcs:
            src = os.path.join(CSRC, s)
            if not os.path.exists(src):
                continue
            obj = os.path.join(OBJDIR, s.replace(".hip", ".o"))
            if force or _stale(obj, [src, *headers, os.path.abspath(__file__)]):  # flags live here
                jobs.append((src, obj))
    if jobs:
        with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            list(ex.map(lambda j: _compile(j[0], j[1], verbose), jobs))
    out = {}
    for lib, srcs in LIBS.items():
        objs = [os.path.join(OBJDIR, s.replace(".hip", ".o")) for s in srcs if os.path.exists(os.path.join(CSRC, s))]
        if not objs:
            continue
        target = os.path.join(LIBDIR, lib)
        if force or _stale(target, objs):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", target, *objs]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed for {lib}:\n{r.stdout}\n{r.stderr}")
        out[lib] = target
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
