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


def test_multi_view_wire_preprocess_unpacks_to_the_per_view_geometry():
    """rr_preprocess_rows_views (every view of the owner's rows in one launch, 52-B wire rows) then
    rr_unpack_rows gives bitwise the geometry of one rr_preprocess_rows call per view: splat records
    of the visible rows (log2 o, 1/o rebuilt), pair counts, depth keys, radii, block sums."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes

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
    stream = N.stream_of(g._xyz)
    for rank in range(world):
        sh = ShardedStep(None, rank, world)
        send, chunk, fields, starts, keep = sh.preprocess_views(g, cams, bg, 0.3, _C.frame_flags())
        Q, _P_pad, lo, nv = sh.layout(g._xyz.shape[0])
        gs, _M = sh._row_params(g, lo)
        gbytes = int(L.rr_geometry_bytes(Q))
        lay = (ctypes.c_size_t * 5)()
        N.check(L.rr_geometry_layout(Q, lay), "layout")
        o_spl, o_til, o_key, o_bs, o_bw = list(lay)
        offs = (ctypes.c_size_t * 5)(*starts)
        for v, cam in enumerate(cams):
            got = torch.zeros(gbytes, dtype=torch.uint8, device=dev)
            got_r = torch.zeros(Q, dtype=torch.int32, device=dev)
            N.check(L.rr_unpack_rows(1, Q, _p(send, v * chunk), chunk, offs, _p(got), gbytes, _p(got_r), stream),
                    "unpack")
            ref = torch.zeros(gbytes, dtype=torch.uint8, device=dev)
            ref_r = torch.zeros(Q, dtype=torch.int32, device=dev)
            fr = sh._frame(g, nv, cam, 0.3, _C.frame_flags() | N.RR_FLAG_RAW_PARAMS)
            rc = N.RRCamera(*[_p(t) for t in keep[v]])
            N.check(L.rr_preprocess_rows(ctypes.byref(fr), ctypes.byref(rc), ctypes.byref(gs), Q, _p(ref_r),
                                         _p(ref, o_spl), _p(ref, o_til), _p(ref, o_key), _p(ref, o_bs),
                                         _p(ref, o_bw), stream), "per-view preprocess")
            torch.cuda.synchronize()
            assert torch.equal(got_r, ref_r), (rank, v)
            vis = ref_r > 0
            assert int(vis.sum()) > 100
            for off, width in ((o_til, 8), (o_key, 4)):
                assert torch.equal(got[off:off + Q * width], ref[off:off + Q * width]), (rank, v, off)
            nb = Q // 256
            assert torch.equal(got[o_bs:o_bs + 8 * nb], ref[o_bs:o_bs + 8 * nb])
            assert torch.equal(got[o_bw:o_bw + 4 * nb], ref[o_bw:o_bw + 4 * nb])
            gs_rows = got[o_spl:o_spl + 48 * Q].view(Q, 48)[vis]
            rs_rows = ref[o_spl:o_spl + 48 * Q].view(Q, 48)[vis]
            assert torch.equal(gs_rows, rs_rows), (rank, v, "splat records")
