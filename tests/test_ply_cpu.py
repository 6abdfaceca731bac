"""PLY save/load and the checkpoint tuple (gaussian_model.py:51-83,167-246).
The byte layout is pinned against a header and record layout written out by hand from the
reference's construct_list_of_attributes / plyfile's binary_little_endian format."""
import numpy as np
import torch

from rain_amd import synthetic
from rain_amd.gaussian_model import GaussianModel, OptimizationParams
from rain_amd.ply import read_elements, write_vertices


def _model(P=500, deg=3, seed=0):
    g = GaussianModel(deg, device="cpu")
    g.set_params(synthetic.random_gaussians(P, sh_degree=deg, seed=seed, bench=True))
    g.active_sh_degree = 1
    return g


def test_ply_layout_matches_reference(tmp_path):
    g = _model(7, 3)
    path = str(tmp_path / "pc" / "point_cloud.ply")
    g.save_ply(path)
    raw = open(path, "rb").read()
    names = ["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)] + \
        [f"f_rest_{i}" for i in range(45)] + ["opacity"] + [f"scale_{i}" for i in range(3)] + \
        [f"rot_{i}" for i in range(4)]
    header = "ply\nformat binary_little_endian 1.0\nelement vertex 7\n" + \
        "".join(f"property float {n}\n" for n in names) + "end_header\n"
    assert raw.startswith(header.encode())
    body = np.frombuffer(raw[len(header):], dtype="<f4").reshape(7, len(names))
    # channel-major SH: f_dc_c = dc[c]; f_rest_{c*15 + k} = rest[k][c]
    dc = g._features_dc.detach().numpy()[:, 0, :]
    rest = g._features_rest.detach().numpy()
    assert np.array_equal(body[:, 6:9], dc)
    assert np.array_equal(body[:, 9:54].reshape(7, 3, 15), rest.transpose(0, 2, 1))
    assert np.array_equal(body[:, 3:6], np.zeros((7, 3), np.float32))
    assert np.array_equal(body[:, 54], g._opacity.detach().numpy()[:, 0])
    assert np.array_equal(body[:, 58:62], g._rotation.detach().numpy())


def test_ply_round_trip(tmp_path):
    g = _model(300, 3, seed=4)
    path = str(tmp_path / "a.ply")
    g.save_ply(path)
    h = GaussianModel(3, device="cpu")
    h.load_ply(path)
    for a, b in zip(g.params(), h.params()):
        assert a.shape == b.shape and torch.equal(a.detach(), b.detach())
    assert h.active_sh_degree == 3


def test_ply_reader_ascii_and_big_endian(tmp_path):
    p = tmp_path / "a.ply"
    p.write_text("ply\nformat ascii 1.0\ncomment x\nelement vertex 2\nproperty float x\nproperty uchar c\n"
                 "end_header\n1.5 3\n-2 255\n")
    v = read_elements(str(p))["vertex"]
    assert v["x"].tolist() == [1.5, -2.0] and v["c"].tolist() == [3, 255]
    q = tmp_path / "b.ply"
    arr = np.array([(1.0, 2.0), (3.0, 4.0)], dtype=[("x", ">f4"), ("y", ">f8")])
    q.write_bytes(b"ply\nformat binary_big_endian 1.0\nelement vertex 2\nproperty float x\nproperty double y\n"
                  b"end_header\n" + arr.tobytes())
    w = read_elements(str(q))["vertex"]
    assert w["x"].tolist() == [1.0, 3.0] and w["y"].tolist() == [2.0, 4.0]
    write_vertices(str(tmp_path / "c.ply"), {"x": np.arange(3), "y": np.ones(3)})
    assert read_elements(str(tmp_path / "c.ply"))["vertex"]["x"].tolist() == [0.0, 1.0, 2.0]


def test_checkpoint_tuple_round_trip(tmp_path):
    g = _model(200, 3, seed=2)
    opt = OptimizationParams()
    g.training_setup(opt)
    for p in g.params():
        p.grad = torch.randn_like(p)
    g.optimizer.step()
    path = str(tmp_path / "chkpnt7000.pth")
    torch.save((g.capture(), 7000), path)
    model_params, it = torch.load(path, weights_only=True)
    h = GaussianModel(3, device="cpu")
    h.restore(model_params, opt)
    assert it == 7000 and h.active_sh_degree == g.active_sh_degree
    for a, b in zip(g.params(), h.params()):
        assert torch.equal(a.detach(), b.detach())
    sa = g.optimizer.state_dict()["state"]
    sb = h.optimizer.state_dict()["state"]
    for k in sa:
        assert torch.equal(sa[k]["exp_avg"], sb[k]["exp_avg"])
