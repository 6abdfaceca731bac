"""Gaussian-sharded, view-parallel training step for N ranks (include/rain_raster.h "row blocks").

The reference trains on one GPU, one view per iteration (train.py:87-147).  With N ranks one step
renders N views (rank v renders view v of the shared permutation, rain_amd.train.ViewSampler) and
applies ONE Adam step to the mean of their gradients — the SURVEY §8(e) contract.  The replicated
design (every rank holds every parameter, reduce-scatter the 236 MB of gradients, all-gather the
236 MB of parameters) moves ~2x(N-1)/N x 236 B per Gaussian over xGMI each step.  Here the bytes that
cross the links are per-(Gaussian, view) records instead:

  rank r owns the Gaussian rows [r*Q, (r+1)*Q) (Q: ceil(P/N) rounded up to 256):
  1. owner preprocess: for each of the step's N views (one launch, rr_preprocess_rows_views), its
     rows' 40-B wire records (the splat's 10 non-derived floats), pair counts, radii and
     per-256-row block sums, 52 B per row;
  2. all-to-all (RCCL over xGMI, every pair of GPUs on its own link): rank v receives view v's
     arrays of every block in one collective (one packed chunk per view), and one kernel
     (rr_unpack_rows) rebuilds its geometry buffer (48-B splat records with log2 o and 1/o, depth
     keys: bitwise the preprocess's);
  3. rank v renders view v from that geometry (rr_forward_from_geometry: depth sort, binning,
     blend), computes the L1+SSIM loss and its gradient, and runs the blend backward into one
     40-B record per Gaussian (rr_backward_records);
  4. all-to-all: the owner receives its rows' records of all N views (in row chunks when the row
     block is large enough that each chunk's owner launch still fills the GPU: chunk c's
     exchange then overlaps the owner kernel on chunk c-1);
  5. owner: the per-Gaussian backward of every view in view order, summed, x 1/N, Adam on its rows,
     densification statistics (rr_gauss_backward_views).
So ~(N-1)/N x (52 + 40) B per Gaussian per step cross xGMI (all-to-all: each GPU's share leaves on
its seven direct links at once), the per-Gaussian backward and Adam of a rank cover 1/N of the
rows, and no collective carries parameters or gradients.  The sum over views is formed per element
in view order, like one process accumulating the same N views: the step's arithmetic is that of
the single-GPU step on N views (tests/test_multirank_gpu.py).

Parameters, Adam moments and statistics are current on their owner's rows only;
`sync_replicas` all-gathers the row blocks where a full replica is read: densify / prune, opacity
reset, checkpoints, evaluation, the end of training.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.distributed as dist

from . import _native as N

REC_FLOATS = 10
WIRE_BYTES = 40  # rr_preprocess_rows_views' wire record (the splat's 10 non-derived floats)


def _p(t, byte_offset=0):
    return None if t is None or t.numel() == 0 else ctypes.c_void_p(t.data_ptr() + byte_offset)


def row_blocks(P: int, world: int):
    """(Q, P_pad): rows per rank (a multiple of 256) and the padded row count N*Q."""
    Q = max(256, int(math.ceil(P / float(world) / 256.0)) * 256)
    return Q, world * Q


class ShardedStep:
    """One rank's side of the Gaussian-sharded step (see the module docstring)."""

    # rows one owner-kernel launch needs to fill the GPU: 256 CUs x 6 resident workgroups x 128 rows
    FILL_ROWS = 256 * 6 * 128

    def __init__(self, exchange, rank: int, world: int, rec_chunk_rows: int | None = None):
        self.ex = exchange
        self.rank, self.world = rank, world
        self._bufs = {}
        self.rec_chunk_rows = rec_chunk_rows

    def chunk_rows(self, Q: int) -> int:
        """Rows per chunk of the record exchange (a multiple of 256).  Chunk c's all-to-all runs while
        the owners process chunk c-1, but every chunk is a launch of its own, so chunks are only
        cut where each still fills the GPU (Q >= 2 x FILL_ROWS, i.e. several million Gaussians at
        N = 8); rec_chunk_rows overrides (tests)."""
        if self.rec_chunk_rows:
            return max(256, int(self.rec_chunk_rows) // 256 * 256)
        if self.world == 1:  # nothing crosses a link: one launch
            return Q
        units = Q // 256
        C = max(1, min(4, Q // self.FILL_ROWS))
        return 256 * -(-units // C)

    def _buf(self, key, numel, dtype, dev):
        t = self._bufs.get(key)
        if t is None or t.numel() != numel or t.dtype != dtype or t.device != dev:
            t = self._bufs[key] = torch.empty((numel,), dtype=dtype, device=dev)
        return t

    def layout(self, P):
        Q, P_pad = row_blocks(P, self.world)
        lo = self.rank * Q
        return Q, P_pad, lo, max(0, min(Q, P - lo))

    # ---- parameters of the owned rows --------------------------------------------------------
    @staticmethod
    def _row_params(model, lo):
        M = 1 + model._features_rest.shape[1]
        xyz, f_dc, f_rest = model._xyz, model._features_dc, model._features_rest
        op, sc, rot = model._opacity, model._scaling, model._rotation
        return N.RRGaussians(_p(xyz, 12 * lo), _p(f_dc, 12 * lo), None, _p(op, 4 * lo), _p(sc, 12 * lo),
                             _p(rot, 16 * lo), None, _p(f_rest, 12 * (M - 1) * lo) if M > 1 else None), M

    def _frame(self, model, P, cam, low_pass, flags):
        D = model.active_sh_degree
        M = 1 + model._features_rest.shape[1]
        return N.RRFrame(int(P), D, M, int(cam.image_width), int(cam.image_height), math.tan(cam.FoVx * 0.5),
                         math.tan(cam.FoVy * 0.5), 1.0, float(low_pass), 0, 0, flags)

    def step(self, model, cams, bg, low_pass, flags, loss_fn, adam, stats):
        """One step of this rank: `cams` = the step's N cameras (rank order); `loss_fn(image, v)`
        -> dL/dimage for view v (this rank's); `adam` = rr_adam block (FusedAdam.fused_step) or None;
        `stats` = (grad_accum, denom, max_radii2D) or None.  Returns (image, loss tensor or None)."""
        L = N.raster()
        dev = model._xyz.device
        P = model._xyz.shape[0]
        Nw = self.world
        Q, P_pad, _lo, _nv = self.layout(P)
        stream = N.stream_of(model._xyz)
        u8 = torch.uint8

        # 1. owner preprocess of every view over the owned rows -> send buffer, one chunk per view
        send, chunk, fields, starts, keep = self.preprocess_views(model, cams, bg, low_pass, flags)

        # 2. one all-to-all: chunk i of recv = rank i's rows for this rank's view, then one kernel
        #    rebuilds the geometry arrays (rows in global order) from the wire records
        recv = self._buf("g_recv", Nw * chunk, u8, dev)
        self.ex.all_to_all(recv, send)
        geom = self._buf("geom", int(L.rr_geometry_bytes(P_pad)), u8, dev)
        radii = self._buf("radii", P_pad, torch.int32, dev)
        offs = (ctypes.c_size_t * 5)(starts[0], starts[1], starts[2], starts[3], starts[4])
        N.check(L.rr_unpack_rows(Nw, Q, _p(recv), chunk, offs, _p(geom), geom.numel(), _p(radii), stream),
                "unpack rows")

        # 3. render this rank's view from the geometry, loss, blend backward -> records
        cam = cams[self.rank]
        fr = self._frame(model, P_pad, cam, low_pass, flags)
        k = keep[self.rank]
        rc = N.RRCamera(*[_p(t) for t in k])
        H, W = int(cam.image_height), int(cam.image_width)
        img = torch.empty((int(L.rr_image_bytes(W, H)),), dtype=u8, device=dev)
        color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
        depth = torch.empty((1, H, W), dtype=torch.float32, device=dev)
        binning = self._bufs.get("binning")
        if binning is None or binning.device != dev:
            binning = torch.empty((0,), dtype=u8, device=dev)
        nr, npairs, need = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_size_t(0)
        # the blend backward's accumulators, zero-filled by this render's blend launch
        # (rr_set_forward_workspace): the backward then skips its 64-MB clear
        ws = self._buf("ws", int(L.rr_backward_workspace_bytes(P_pad)), u8, dev)
        N.check(L.rr_set_forward_workspace(_p(ws), ws.numel()), "register workspace")
        r = L.rr_forward_from_geometry(ctypes.byref(fr), ctypes.byref(rc), _p(radii), _p(geom), geom.numel(), _p(img),
                                       img.numel(), _p(binning), binning.numel(), ctypes.byref(nr),
                                       ctypes.byref(npairs), ctypes.byref(need), _p(color), _p(depth), stream)
        if r == N.RR_INCOMPLETE:
            binning = self._bufs["binning"] = torch.empty((int(need.value * 1.25) + 4096,), dtype=u8, device=dev)
            r = L.rr_forward_render_geometry(ctypes.byref(fr), ctypes.byref(rc), _p(radii), _p(geom), _p(img),
                                             _p(binning), binning.numel(), npairs.value, _p(color), _p(depth), stream)
        if r not in (0, N.RR_INCOMPLETE):
            L.rr_set_forward_workspace(None, 0)  # a failed render must not leave the registration behind
        N.check(r, "sharded forward")
        self.last = dict(num_rendered=nr.value, num_pairs=npairs.value, P_pad=P_pad, Q=Q)
        dimg, loss = loss_fn(color)
        dimg = dimg.contiguous()
        recs = self._buf("recs", P_pad * REC_FLOATS, torch.float32, dev)
        CR = self.chunk_rows(Q)
        frb = N.RRFrame.from_buffer_copy(fr)
        frb.flags |= N.RR_FLAG_WORKSPACE_REGISTERED
        N.check(L.rr_backward_records(ctypes.byref(frb), ctypes.byref(rc), _p(radii), _p(geom), _p(img), _p(binning),
                                      nr.value, _p(dimg), _p(ws), ws.numel(), Q, CR, _p(recs), stream),
                "sharded backward")

        self.exchange_and_own(model, cams, keep, recs, low_pass, adam, stats)
        return color, loss

    def preprocess_views(self, model, cams, bg, low_pass, flags):
        """Step 1: the owner's rows preprocessed for each of the step's views into the send buffer,
        one chunk per view (256-B aligned): [wire records Q x 40 B | pair counts Q x 8 | radii Q x 4 |
        block sums Q/256 x 8 | wide flags Q/256 x 4] — 52 B per row; the receiver rebuilds the 48-B
        splat records and the depth keys (rr_unpack_rows).  Returns (send, chunk bytes, fields,
        field starts, keep = per-view (bg, view, proj, campos) tensors)."""
        L = N.raster()
        dev = model._xyz.device
        P = model._xyz.shape[0]
        Nw = self.world
        Q, _P_pad, lo, nv = self.layout(P)
        stream = N.stream_of(model._xyz)
        gs, _M = self._row_params(model, lo)
        nb = Q // 256
        fields = ((WIRE_BYTES, Q), (8, Q), (4, Q), (8, nb), (4, nb))
        starts, c = [], 0
        for w, n in fields:
            starts.append(c)
            c += w * n
        chunk = (c + 255) // 256 * 256
        send = self._buf("g_send", Nw * chunk, torch.uint8, dev)
        keep = [(bg.contiguous(), cam.world_view_transform.contiguous(), cam.full_proj_transform.contiguous(),
                 cam.camera_center.contiguous()) for cam in cams]
        # every view in one launch (rr_preprocess_rows_views): view v's chunk at v * chunk
        views = (N.RRView * Nw)()
        for v, (cam, k) in enumerate(zip(cams, keep)):
            views[v] = N.RRView(_p(k[1]), _p(k[2]), _p(k[3]), math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5),
                                float(low_pass), int(cam.image_width), int(cam.image_height))
        fr = self._frame(model, nv, cams[0], low_pass, flags | N.RR_FLAG_RAW_PARAMS)
        # [radii, wire records, pair counts, (no depth keys), block sums, wide flags]
        offs = (ctypes.c_size_t * 6)(starts[2], starts[0], starts[1], 0, starts[3], starts[4])
        N.check(L.rr_preprocess_rows_views(ctypes.byref(fr), views, Nw, ctypes.byref(gs), Q, _p(send), chunk, offs,
                                           1, stream),
                "sharded preprocess")
        return send, chunk, fields, starts, keep

    def exchange_and_own(self, model, cams, keep, recs, low_pass, adam, stats):
        """Steps 4-5 of step(): the record exchange and the owners' per-Gaussian backward + Adam.
        `recs`: this rank's records in rr_backward_records' chunked layout for chunk_rows(Q);
        `keep[v]`: (bg, view, proj, campos) tensors of view v."""
        L = N.raster()
        dev = model._xyz.device
        P = model._xyz.shape[0]
        Nw = self.world
        Q, _P_pad, lo, nv = self.layout(P)
        stream = N.stream_of(model._xyz)
        CR = self.chunk_rows(Q)
        # 4. all-to-all of the records in row chunks (rr_backward_records lays chunk c out as
        #    [N][n_c][10] at row N*r0): chunk c of recv = view v's records of the owned rows
        #    [r0, r0 + n_c) for v = 0..N-1; all chunks are issued before the first owner launch
        recv = self._buf("recv", Nw * Q * REC_FLOATS, torch.float32, dev)
        chunks, r0 = [], 0
        while r0 < Q:
            n_c = min(CR, Q - r0)
            a, b = Nw * r0 * REC_FLOATS, Nw * (r0 + n_c) * REC_FLOATS
            chunks.append((r0, n_c, a, self.ex.all_to_all(recv[a:b], recs[a:b], async_op=True)))
            r0 += n_c

        # 5. owner, per chunk once its records are in: per-Gaussian backward of all views, summed in
        #    view order, x 1/N, Adam, statistics (rows are independent: any chunking gives the same
        #    bits)
        views = (N.RRView * Nw)()
        for v, c in enumerate(cams):
            kv = keep[v]
            views[v] = N.RRView(_p(kv[1]), _p(kv[2]), _p(kv[3]), math.tan(c.FoVx * 0.5), math.tan(c.FoVy * 0.5),
                                float(low_pass), int(c.image_width), int(c.image_height))
        acc, den, mr = stats if stats is not None else (None, None, None)
        for r0, n_c, a, work in chunks:
            if work is not None:
                work.wait()
            nv_c = max(0, min(n_c, nv - r0))
            if nv_c == 0:
                continue
            row = lo + r0
            gs_c, _M = self._row_params(model, row)
            frb = self._frame(model, nv_c, cams[0], low_pass, N.RR_FLAG_RAW_PARAMS)
            ad = _offset_adam(adam, model, row) if adam is not None else None
            out = N.RRGrads(None, None, None, None, None, None, None, None, None, _p(acc, 4 * row), _p(den, 4 * row),
                            _p(mr, 4 * row), ctypes.pointer(ad) if ad is not None else None)
            N.check(L.rr_gauss_backward_views(ctypes.byref(frb), views, Nw, ctypes.byref(gs_c), _p(recv, 4 * a), n_c,
                                              1.0 / Nw, ctypes.byref(out), stream), "sharded gaussian backward")

    # ---- replicas ------------------------------------------------------------------------------
    def sync_replicas(self, model):
        """All-gather every row block of the parameters, Adam moments and densification statistics,
        so that every rank holds the full, current state."""
        P = model._xyz.shape[0]
        Q, _P_pad, lo, _nv = self.layout(P)
        ts = list(model.params())
        for p in model.params():
            st = model.optimizer.state.get(p)
            if st and "exp_avg" in st:
                ts += [st["exp_avg"], st["exp_avg_sq"]]
        ts += [model.xyz_gradient_accum, model.denom, model.max_radii2D]
        for t in ts:
            self.ex.all_gather_rows(t.data if isinstance(t, torch.nn.Parameter) else t, Q, lo)


def _offset_adam(ad, model, lo):
    """rr_adam of FusedAdam.fused_step with every group's arrays moved to row `lo`."""
    out = N.RRAdam()
    out.beta1, out.beta2, out.eps = ad.beta1, ad.beta2, ad.eps
    widths = dict(xyz=3, f_dc=3, f_rest=3 * model._features_rest.shape[1], opacity=1, scaling=3, rotation=4)
    for name, w in widths.items():
        src = getattr(ad, name)
        dst = getattr(out, name)
        if src.param:
            d = 4 * w * lo
            dst.param, dst.exp_avg, dst.exp_avg_sq = src.param + d, src.exp_avg + d, src.exp_avg_sq + d
            dst.lr, dst.bias_correction1, dst.bias_correction2_sqrt = src.lr, src.bias_correction1, \
                src.bias_correction2_sqrt
    return out
