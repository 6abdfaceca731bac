"""CPU checks of the simple-knn oracle (oracle/knn_oracle.c, the checker of rain_amd/csrc/knn.hip)
against its definition: the exact mean of the 3 smallest squared distances to other points
(simple_knn.cu:125-157), plus the reference's edge behaviour."""
import numpy as np
import pytest

from oracle import oracle as O

FMAX = np.float32(np.finfo(np.float32).max)


def brute(pts):
    d = pts[None, :, :] - pts[:, None, :]
    dd = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]  # fp32, unfused
    np.fill_diagonal(dd, FMAX)
    s = np.sort(dd, axis=1)
    s = np.concatenate([s, np.full((len(pts), 3), FMAX, np.float32)], axis=1)[:, :3]
    return ((s[:, 0] + s[:, 1]) + s[:, 2]) / np.float32(3)


@pytest.mark.parametrize("P,seed", [(4, 0), (5, 1), (100, 2), (1023, 3), (1025, 4), (3000, 5)])
def test_oracle_is_exact_3nn(P, seed):
    rng = np.random.default_rng(seed)
    pts = (rng.random((P, 3)) * 2.6 - 1.3).astype(np.float32)
    assert np.array_equal(O.dist_knn3(pts), brute(pts))


def test_oracle_clustered_duplicates_and_planar():
    rng = np.random.default_rng(7)
    a = (rng.normal(size=(500, 3)) * 0.01 + 3.0).astype(np.float32)    # a far cluster (origin pulls the bbox)
    b = np.repeat(a[:50], 2, axis=0)                                  # exact duplicates -> distance 0
    c = np.c_[rng.random((400, 2)), np.zeros(400)].astype(np.float32)  # z == 0 plane: 0/0 Morton axis
    pts = np.concatenate([a, b, c]).astype(np.float32)
    d = O.dist_knn3(pts)
    assert np.array_equal(d, brute(pts))
    assert (d[500:600] <= d[:100].max()).all()


def test_oracle_small_and_bbox():
    d1 = O.dist_knn3(np.array([[1, 2, 3]], np.float32))
    assert np.isinf(d1).all()
    d2 = O.dist_knn3(np.array([[1, 2, 3], [1, 2, 4]], np.float32))
    assert np.isinf(d2).all()
    d3 = O.dist_knn3(np.array([[1, 2, 3], [1, 2, 4], [1, 2, 6]], np.float32))
    assert np.all(d3 == FMAX / np.float32(3))
    pts = np.array([[1, 1, 1], [2, 3, 4], [5, 5, 5], [2, 2, 2]], np.float32)
    _, order, bbox = O.dist_knn3(pts, details=True)
    assert np.array_equal(bbox, [0, 0, 0, 5, 5, 5])  # CUB Reduce init {0,0,0}: the origin is inside
    assert sorted(order.tolist()) == [0, 1, 2, 3]
