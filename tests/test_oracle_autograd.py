"""The oracle's hand-written backward (restating backward.cu) against float64 autograd of a
differentiable restatement of its own forward (oracle/torch_ref.py), on small scenes.  Together
with tests/test_golden.py this pins the oracle that the GPU parity tests trust."""
import numpy as np
import pytest

from oracle import torch_ref
from tests.common import make_scene, oracle_run, rel_l1

CASES = {
    "sh3": dict(P=250, W=48, H=40, sh_degree=3),
    "sh1": dict(P=250, W=48, H=40, sh_degree=3, active_degree=1),
    "white_bg_mod": dict(P=200, W=40, H=32, sh_degree=2, bg=(1.0, 0.5, 0.25), scale_modifier=0.8),
    "colors_precomp": dict(P=200, W=40, H=32, sh_degree=3, precomp_colors=True),
    "cov3D_precomp": dict(P=200, W=40, H=32, sh_degree=3, precomp_cov=True),
    "low_pass_big": dict(P=60, W=48, H=40, sh_degree=3, low_pass=20.0),
    "frustum_clamp": dict(P=300, W=48, H=40, sh_degree=3, extent=3.0, radius=3.2),
}


@pytest.mark.parametrize("case", list(CASES))
def test_oracle_backward_equals_autograd(oracle, case):
    inp, st = make_scene(**CASES[case])
    rng = np.random.default_rng(3)
    dpix = rng.standard_normal((3, st["image_height"], st["image_width"])).astype(np.float32)
    ref = oracle_run(oracle, inp, st, dL_dpix=dpix, nthreads=1)
    lists = ref["state"].blend_lists()
    stn = {k: (v.numpy() if hasattr(v, "numpy") else v) for k, v in st.items()}
    ag = torch_ref.render_autograd(stn, {k: v.numpy() for k, v in inp.items()}, lists, ref["radii"] > 0, dpix)
    # forward image agrees (float32 oracle vs float64 restatement)
    assert rel_l1(ref["color"], ag["image"]) < 1e-5
    g = ref["grads"]
    vis = ref["radii"] > 0
    for k in ag:
        if k == "image":
            continue
        a, b = g[k], ag[k]
        if k == "dL_dsh":
            K = (st["sh_degree"] + 1) ** 2
            assert np.abs(a[:, K:]).sum() == 0  # coefficients beyond the active degree get nothing
            a, b = a[:, :K], b[:, :K]
        if k == "dL_dcov3D":  # the reference only writes it for visible Gaussians
            a, b = a[vis], b[vis]
        if np.abs(b).sum() == 0:
            assert np.abs(a).max() < 1e-9, k
            continue
        r = rel_l1(a, b)
        assert r < 1e-4, f"{k}: rel L1 {r:.3e}"
    # Gaussians the forward did not keep get exactly zero gradient (backward.cu:146,357)
    for k in ("dL_dmeans3D", "dL_dscales", "dL_drotations", "dL_dopacity", "dL_dcov3D"):
        assert np.abs(g[k][~vis]).sum() == 0, k
