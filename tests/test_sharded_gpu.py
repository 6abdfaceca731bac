"""The owner side of the Gaussian-sharded step (rain_amd/sharded.py ShardedStep.exchange_and_own:
record exchange in row chunks + rr_gauss_backward_views per chunk) is independent of the chunking,
bit for bit: every row's per-view sum, scale and Adam step are the same operations on the same
values whichever launch covers the row.  One process; the exchange is a stand-in in which every
rank sent this rank's records (deterministic, unlike a second blend backward whose float atomics
may add in another order), so the same logical records reach the owner in both layouts."""
import pytest
import torch

pytestmark = pytest.mark.gpu

REC = 10


class _EchoExchange:
    """all_to_all where every rank's chunk for this rank equals this rank's own chunk 0."""

    def __init__(self, world):
        self.world = world

    def all_to_all(self, recv, send, async_op=False):
        n = send.numel() // self.world
        s0 = send.view(self.world, n)[0]
        recv.view(self.world, n).copy_(s0.expand(self.world, n))
        return None


def _layout(R, world, Q, CR):
    """Logical records R [world*Q, 10] in rr_backward_records' chunked layout (include/rain_raster.h)."""
    out = torch.empty_like(R)
    Rv = R.view(world, Q, REC)
    r0 = 0
    while r0 < Q:
        n_c = min(CR, Q - r0)
        out[world * r0:world * (r0 + n_c)].view(world, n_c, REC).copy_(Rv[:, r0:r0 + n_c])
        r0 += n_c
    return out


def _state(g):
    ts = list(g.params())
    for p in g.params():
        st = g.optimizer.state[p]
        ts += [st["exp_avg"], st["exp_avg_sq"]]
    return ts + [g.xyz_gradient_accum, g.denom, g.max_radii2D]


def test_owner_chunking_is_bitwise_neutral():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rain_amd import cameras, synthetic
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.sharded import ShardedStep

    dev = torch.device("cuda:0")
    world = 3
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(5000, sh_degree=3, seed=3, bench=True))
    g.active_sh_degree = 3
    g.spatial_lr_scale = 4.4
    g.training_setup(OptimizationParams())
    cams = [c.to(dev) for c in cameras.fibonacci_cameras(world, 160, 120)]
    bg = torch.zeros(3, device=dev)
    keep = [(bg, c.world_view_transform.contiguous(), c.full_proj_transform.contiguous(),
             c.camera_center.contiguous()) for c in cams]
    P = g._xyz.shape[0]
    # Adam moments and statistics with content, so every term of the update is exercised
    ad0 = g.optimizer.fused_step(g)
    for p in g.params():
        st = g.optimizer.state[p]
        st["exp_avg"].normal_(0, 1e-3, generator=torch.Generator(device=dev).manual_seed(1))
        st["exp_avg_sq"].uniform_(0, 1e-6, generator=torch.Generator(device=dev).manual_seed(2))
    g.xyz_gradient_accum.uniform_(0, 1)
    g.denom.fill_(3.0)
    ad = g.optimizer.fused_step(g)  # the same rr_adam block for both runs
    del ad0
    sh = ShardedStep(_EchoExchange(world), 0, world)
    Q, P_pad, lo, nv = sh.layout(P)
    gen = torch.Generator().manual_seed(7)
    R = torch.randn(P_pad, REC, generator=gen) * 1e-3
    R[:, 9] = torch.randint(0, 4, (P_pad,), generator=gen).float()  # radius 0 (untouched) .. 3
    R = R.to(dev)
    stats = (g.xyz_gradient_accum, g.denom, g.max_radii2D)
    snap = [t.detach().clone() for t in _state(g)]
    results = []
    for cr in (None, 256, 768):
        for t, s0 in zip(_state(g), snap):
            t.data.copy_(s0)
        sh.rec_chunk_rows = cr
        CR = sh.chunk_rows(Q)
        assert (cr is None and CR >= Q) or CR == cr
        sh.exchange_and_own(g, cams, keep, _layout(R, world, Q, CR).reshape(-1), 0.3, ad, stats)
        torch.cuda.synchronize()
        results.append([t.detach().clone() for t in _state(g)])
    changed = sum(int(not torch.equal(a, b)) for a, b in zip(results[0], snap))
    assert changed >= 18, "the owner step left the state unchanged"
    for other in results[1:]:
        for i, (a, b) in enumerate(zip(results[0], other)):
            assert torch.equal(a, b), f"state tensor {i} differs between chunkings"


def test_multi_view_preprocess_equals_per_view():
    """rr_preprocess_rows_views (every view of the owner's rows in one launch) writes the same
    bytes as one rr_preprocess_rows call per view."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes
    import math

    from rain_amd import _native as N
    from rain_amd import cameras, synthetic
    from rain_amd.diff_gaussian_rasterization import _C
    from rain_amd.gaussian_model import GaussianModel
    from rain_amd.sharded import ShardedStep, _p

    dev = torch.device("cuda:0")
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(7000, sh_degree=3, seed=4, bench=True))
    g.active_sh_degree = 3
    world = 3
    cams = [c.to(dev) for c in cameras.fibonacci_cameras(world, 200, 150)]
    bg = torch.zeros(3, device=dev)
    L = N.raster()
    for rank in range(world):
        sh = ShardedStep(None, rank, world)
        send, chunk, fields, starts, keep = sh.preprocess_views(g, cams, bg, 0.3, _C.frame_flags())
        send.fill_(0xAB)  # culled rows leave their splat records unwritten: same fill on both sides
        send, chunk, fields, starts, keep = sh.preprocess_views(g, cams, bg, 0.3, _C.frame_flags())
        got = send.clone()
        Q, _P_pad, lo, nv = sh.layout(g._xyz.shape[0])
        gs, _M = sh._row_params(g, lo)
        ref = torch.full_like(send, 0xAB)
        stream = N.stream_of(g._xyz)
        for v, cam in enumerate(cams):
            fr = sh._frame(g, nv, cam, 0.3, _C.frame_flags() | N.RR_FLAG_RAW_PARAMS)
            rc = N.RRCamera(*[_p(t) for t in keep[v]])
            b = v * chunk
            N.check(L.rr_preprocess_rows(ctypes.byref(fr), ctypes.byref(rc), ctypes.byref(gs), Q,
                                         _p(ref, b + starts[3]), _p(ref, b + starts[0]), _p(ref, b + starts[1]),
                                         _p(ref, b + starts[2]), _p(ref, b + starts[4]), _p(ref, b + starts[5]),
                                         stream), "per-view preprocess")
        torch.cuda.synchronize()
        assert math.isfinite(float(got.float().sum()))
        assert torch.equal(got, ref), f"rank {rank}: multi-view preprocess differs"
