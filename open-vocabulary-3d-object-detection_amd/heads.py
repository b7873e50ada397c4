"""The five 3DETR prediction heads side by side (training, bf16 autocast, one process).

Reference: models/model_3detr.py:_build_heads / get_box_predictions — five GenericMLPs
(models/helpers.py:45-112), each Conv1d(256,256) -> BatchNorm1d -> ReLU -> Dropout(0.3)
-> Conv1d(256,256) -> BatchNorm1d -> ReLU -> Dropout(0.3) -> Conv1d(256, out), all on
the same (L*B*Q, 256) decoder-feature rows.  BatchNorm is per channel, so the five
heads are exactly one MLP over 5 x 256 channels with block-diagonal later layers:

  layer 1  ONE GEMM            x (R,256) @ W1cat^T (1280,256)          -> h1 (R,1280)
  BN+ReLU+Dropout              csrc/bnrows.hip over 1280 channels       -> z1
  layer 2  ONE batched GEMM    per head z1[i] @ W2_i^T (z1 head-major)  -> h2 (5,R,256)
  BN+ReLU+Dropout              (head-major addressing)                  -> z2 (R,1280)
  layer 3  ONE launch (csrc/headsout.hip): the five output layers on z2 + the text
           alignment of the visual embedding

Backward mirrors it; weight / bias gradients use the one-launch ov3d_wgrad kernel.
The heads' parameters and BN buffers are re-pointed at shared storages (the module
objects, their names and state-dict keys do not change), so the concatenated weights
exist without a per-step concatenation.  Dropout masks come from a counter-based hash
(bnrows.hip), regenerated in the backward.  Results equal the per-head evaluation up
to bf16 rounding (tests/test_heads_gpu.py).
"""
import ctypes
import os

import torch
import torch.nn as nn

from . import _native as nat
from . import attention as flash
from . import gemm
from .gemm import fused_weight_grad
from .sa_fused import _sync_group, bn_affine, bn_bwd_affine

# BatchNorm1d, or its SyncBatchNorm conversion (DDP, main.py:427-431): the statistics
# totals are then all-reduced over the BN's process group (exact SyncBN semantics)
_BN_TYPES = (nn.BatchNorm1d, nn.SyncBatchNorm)
# BatchNorm2d over channels-last rows == BatchNorm1d over the same rows (per-channel statistics
# over every position): the SharedMLP layers of the set-abstraction modules
_BN_ROW_TYPES = _BN_TYPES + (nn.BatchNorm2d,)

HEAD_ORDER = ("visual_embed_head", "center_head", "size_head", "angle_cls_head",
              "angle_residual_head")
NPARTS = 256


def _structure(mlp):
    """-> (conv1, bn1, drop1, conv2, bn2, drop2, conv3) of a reference head, or None."""
    m = list(mlp.layers)
    if len(m) != 9:
        return None
    c1, b1, r1, d1, c2, b2, r2, d2, c3 = m
    ok = (isinstance(c1, nn.Conv1d) and isinstance(c2, nn.Conv1d) and isinstance(c3, nn.Conv1d)
          and type(b1) in _BN_TYPES and type(b2) in _BN_TYPES
          and isinstance(r1, nn.ReLU) and isinstance(r2, nn.ReLU)
          and isinstance(d1, nn.Dropout) and isinstance(d2, nn.Dropout)
          and c1.bias is None and c2.bias is None and c3.bias is not None)
    return (c1, b1, d1, c2, b2, d2, c3) if ok else None


class HeadPack:
    """Shared storages for the five heads' hidden layers (built lazily on the device)."""

    def __init__(self, heads):
        self.parts = [_structure(heads[n]) for n in HEAD_ORDER]
        self.ok = all(p is not None for p in self.parts)
        if self.ok:
            c1 = self.parts[0][0]
            self.C = c1.in_channels
            self.H = c1.out_channels
            self.ok = all(p[0].in_channels == self.C and p[0].out_channels == self.H and
                          p[3].in_channels == self.H and p[3].out_channels == self.H and
                          p[6].in_channels == self.H for p in self.parts) and self.H % 64 == 0
        self.store = None
        self.sites = (flash.new_site(), flash.new_site())

    def _tensors(self):
        P = self.parts
        return {"w1": [p[0].weight for p in P], "w2": [p[3].weight for p in P],
                "g1": [p[1].weight for p in P], "b1": [p[1].bias for p in P],
                "g2": [p[4].weight for p in P], "b2": [p[4].bias for p in P],
                "rm1": [p[1].running_mean for p in P], "rv1": [p[1].running_var for p in P],
                "rm2": [p[4].running_mean for p in P], "rv2": [p[4].running_var for p in P]}

    def _shared(self):
        if self.store is None:
            return False
        for key, ts in self._tensors().items():
            base = self.store[key]
            step = ts[0].numel()
            for i, t in enumerate(ts):
                if t.data_ptr() != base.data_ptr() + i * step * base.element_size() or \
                        t.device != base.device:
                    return False
        return True

    def ensure(self):
        """(Re-)point parameters / buffers at the shared storages when needed (e.g. after
        .to(device) or load_state_dict with assign=True)."""
        if self._shared():
            self._ensure_bf16()
            return
        store = {}
        with torch.no_grad():
            for key, ts in self._tensors().items():
                base = torch.cat([t.detach().reshape(-1) for t in ts])
                store[key] = base
                step = ts[0].numel()
                for i, t in enumerate(ts):
                    view = base[i * step:(i + 1) * step].view(t.shape)
                    if isinstance(t, nn.Parameter):
                        t.data = view
                    else:
                        for p in self.parts:
                            for bn in (p[1], p[4]):
                                for name in ("running_mean", "running_var"):
                                    if bn._buffers[name] is t:
                                        bn._buffers[name] = view
        self.store = store
        self._ensure_bf16()

    def _ensure_bf16(self):
        """bf16 storages of the hidden layers' weights, registered as the parameters' shadow
        copies (gemm.register_shadow): the optimizer keeps them current, no per-step cast"""
        st = self.store
        for key in ("w1", "w2"):
            bk = key + "_bf"
            if bk not in st or st[bk].device != st[key].device:
                st[bk] = st[key].to(torch.bfloat16)
            ts = self._tensors()[key]
            step = ts[0].numel()
            for i, t in enumerate(ts):
                gemm.register_shadow(t, st[bk][i * step:(i + 1) * step].view(t.shape))

    def out_layout(self, w3):
        """ctypes arrays of the box heads' output widths, input and output columns"""
        n = tuple(int(w.shape[0]) for w in w3[1:])
        lay = getattr(self, "_lay", None)
        if lay is None or lay["key"] != n:
            ocol, o = [], 0
            for k in n:
                ocol.append(o)
                o += k
            lay = {"key": n, "Ns": o, "n": (ctypes.c_int * 4)(*n),
                   "kcol": (ctypes.c_int * 4)(*[self.H * (1 + i) for i in range(4)]),
                   "ocol": (ctypes.c_int * 4)(*ocol)}
            self._lay = lay
        return lay

    def bns(self):
        return [p[1] for p in self.parts], [p[4] for p in self.parts]


# shapes the output launch is compiled for (csrc/headsout.hip: KH, NV, MAXS, a box head's
# outputs <= 32); other head shapes (e.g. the reduced smoke model) take the per-head rows path
OUT_HIDDEN, OUT_VISUAL, OUT_BOX_HEADS, OUT_BOX_MAX = 256, 640, 4, 32


def supported(pack, rows):
    if not (pack.ok and rows.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    outs = [p[6].out_channels for p in pack.parts]
    if pack.H != OUT_HIDDEN or outs[0] != OUT_VISUAL or len(outs) != 1 + OUT_BOX_HEADS \
            or not all(0 < n <= OUT_BOX_MAX for n in outs[1:]):
        return False
    drops = set()
    groups = set()
    for p in pack.parts:
        for bn in (p[1], p[4]):
            if not bn.training or not bn.track_running_stats or bn.momentum is None:
                return False
            groups.add(id(_sync_group(bn)))
        drops.add((p[2].p if p[2].training else 0.0, p[5].p if p[5].training else 0.0))
    return len(drops) == 1 and len(groups) == 1


def _group_world(bn):
    g = _sync_group(bn)
    return g, (torch.distributed.get_world_size(g) if g is not None else 1)


def _stats_finalize(x, layout, R, C, gamma, beta, bns, rm, rv, nbt=None):
    """train-mode batch statistics of BN over R rows (x all ranks of a SyncBatchNorm group)
    -> (mean, invstd, scale, shift); running stats of the concatenated storages updated
    (momentum, unbiased var)."""
    dev = x.device
    parts = torch.empty((NPARTS, 2, C), dtype=torch.float64, device=dev)
    nat.call("ov3d_rows_bn_stats", x, int(x.dtype == torch.bfloat16), *layout, R, C, parts, NPARTS,
             like=x)
    bn0 = bns[0]
    group, world = _group_world(bn0)
    return bn_affine(parts, NPARTS, C, group, R * world, gamma, beta, bn0.eps, bn0.momentum, rm, rv,
                     nbt)


class _Heads(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pack, p1, p2, text, lq, *params):
        # params: the shared-storage views of w1 / w2 / g1 / b1 / g2 / b2 (5 each, the grads are
        # returned for them; the kernels use the storages directly), then the output layers'
        # weights (5) and biases (5) in HEAD_ORDER
        st = pack.store
        R = x.shape[0]
        H5 = 5 * pack.H
        H = pack.H
        bf = torch.bfloat16
        dev = x.device
        seed = flash._seed(dev)
        xb = x.to(bf).contiguous()
        # bf16 copies kept current by the optimizer (HeadPack.ensure registers them)
        w1 = st["w1_bf"].view(H5, pack.C)
        w2 = st["w2_bf"].view(5, H, H)
        bn1, bn2 = pack.bns()
        torch._foreach_add_([b.num_batches_tracked for b in bn1 + bn2], 1)
        h1 = (gemm.tile_gemm(xb, w1) if gemm._tile_gemm_ok(xb, w1, True)
              else xb @ w1.t())                                                  # (R, 5H)
        rowmajor = (H5, 0, H5)
        m1, i1, a1, s1 = _stats_finalize(h1, rowmajor, R, H5, st["g1"], st["b1"], bn1, st["rm1"],
                                         st["rv1"])
        # z1 written head-major (5, R, H): the second layer is a packed batched GEMM (batch
        # stride R*H; the row-major z1 viewed per head had batch stride H inside rows of 5H,
        # the layout the TunableOp solution faulted on)
        headmajor = (H, R * H, H)
        z1 = torch.empty((5, R, H), dtype=bf, device=dev)
        nat.call("ov3d_rows_bn_apply", h1, 1, *rowmajor, R, H5, a1, s1, float(p1), seed,
                 pack.sites[0], z1, *headmajor, like=x)
        h2 = (gemm.tile_bmm(z1, w2, True) if gemm.tile_bmm_ok(z1, w2, True)
              else torch.bmm(z1, w2.transpose(1, 2)))                           # (5, R, H)
        m2, i2, a2, s2 = _stats_finalize(h2, headmajor, R, H5, st["g2"], st["b2"], bn2, st["rm2"],
                                         st["rv2"])
        z2 = torch.empty((R, H5), dtype=bf, device=dev)
        nat.call("ov3d_rows_bn_apply", h2, 1, *headmajor, R, H5, a2, s2, float(p2), seed,
                 pack.sites[1], z2, *rowmajor, like=x)
        # output layers + the text alignment: one launch (csrc/headsout.hip)
        w3 = [gemm.cast_param(w.view(w.shape[0], -1), bf) for w in params[-10:-5]]
        b3 = list(params[-5:])
        lay = pack.out_layout(w3)
        Nv, Ns = w3[0].shape[0], lay["Ns"]
        out_v = torch.empty((R, Nv), dtype=torch.float32, device=dev)
        out_s = torch.empty((R, Ns), dtype=torch.float32, device=dev)
        T = text.shape[0] if text is not None else 0
        logits = torch.empty((R, T), dtype=torch.float32, device=dev) if text is not None else None
        ws = (ctypes.c_void_p * 4)(*[w.data_ptr() for w in w3[1:]])
        bs = (ctypes.c_void_p * 4)(*[b.data_ptr() for b in b3[1:]])
        work = torch.empty((max(nat.load().ov3d_heads_out_workspace(R, T), 1),), dtype=torch.float32,
                           device=dev)
        nat.call("ov3d_heads_out_fwd", z2, H5, R, w3[0], b3[0], Nv, text, T, int(lq), out_v, logits,
                 4, ctypes.addressof(ws), ctypes.addressof(bs), ctypes.addressof(lay["n"]),
                 ctypes.addressof(lay["kcol"]), ctypes.addressof(lay["ocol"]), out_s, Ns, work, like=x)
        ctx.save_for_backward(xb, h1, h2, z1, z2, w1, w2, *w3, m1, i1, a1, s1, m2, i2, a2, s2, text)
        # an output nobody consumed gets no zero-filled gradient (the visual embedding without
        # the 2D alignment loss: 21 MB of zeros per step)
        ctx.set_materialize_grads(False)
        ctx.seed = seed   # the forward's dropout snapshot (attention._seed)
        ctx.meta = (pack, float(p1), float(p2), R, x.dtype, int(lq), [w.shape for w in params[-10:-5]])
        if logits is None:
            return out_v, out_s
        return out_v, out_s, logits

    @staticmethod
    def backward(ctx, gv, gs, glog=None):
        (xb, h1, h2, z1, z2, w1, w2, w3v, w3a, w3b, w3c, w3d, m1, i1, a1, s1, m2, i2, a2, s2,
         text) = ctx.saved_tensors
        w3 = [w3v, w3a, w3b, w3c, w3d]
        pack, p1, p2, R, xdt, lq, w3_shapes = ctx.meta
        st = pack.store
        H = pack.H
        H5 = 5 * H
        bf = torch.bfloat16
        dev = xb.device
        seed = ctx.seed
        lay = pack.out_layout(w3)
        Nv, Ns = w3v.shape[0], lay["Ns"]
        T = text.shape[0] if text is not None else 0
        # g_v + g_logits . text and the box heads' output gradients in bf16, the box heads'
        # input gradient into dz2[:, H:]: one launch; the visual input gradient on the BLAS
        if gv is not None:
            gv = gv.contiguous()
        gs = gs.contiguous() if gs is not None else torch.zeros((R, Ns), dtype=torch.float32, device=dev)
        if glog is not None:
            glog = glog.contiguous()
        gvb = torch.empty((R, Nv), dtype=bf, device=dev)
        gsb = torch.empty((R, Ns), dtype=bf, device=dev)
        dz2 = torch.empty((R, H5), dtype=bf, device=dev)
        ws = (ctypes.c_void_p * 4)(*[w.data_ptr() for w in w3[1:]])
        nat.call("ov3d_heads_out_bwd", gv, glog if text is not None else None, text, R, Nv, T, lq,
                 gs, Ns, 4, ctypes.addressof(ws), ctypes.addressof(lay["n"]),
                 ctypes.addressof(lay["kcol"]), ctypes.addressof(lay["ocol"]), gvb, gsb, dz2, H5,
                 like=xb)
        if gemm._tile_gemm_ok(gvb, w3v, False) and gemm.tile_out_ok(dz2[:, :H]):
            gemm.tile_gemm(gvb, w3v, trans_b=False, out=dz2[:, :H])
        else:
            torch.mm(gvb, w3v, out=dz2[:, :H])
        # weight gradients: queued for the grouped launch at the end of the backward
        # (gemm.DEFER_WGRAD) as one problem per head parameter, else computed here
        P = pack.parts
        defer = gemm.DEFER_WGRAD and all(
            gemm.can_defer(xb, m.weight, m.bias) for p in P for m in (p[0], p[3], p[6]))
        d3 = [None] * 10
        gsl = [gvb]
        for i in range(4):
            o = lay["ocol"][i]
            gsl.append(gsb[:, o:o + lay["n"][i]])
        for i, p in enumerate(P):
            if defer:
                gemm.defer_weight_grad(gsl[i], z2[:, i * H:(i + 1) * H], p[6].weight, p[6].bias)
            else:
                dw, db = fused_weight_grad(gsl[i], z2[:, i * H:(i + 1) * H], bias=True)
                d3[i], d3[5 + i] = dw.view(w3_shapes[i]), db
        rowmajor = (H5, 0, H5)
        headmajor = (H, R * H, H)
        # BN2 (input h2 head-major, grad dz2 row-major) -> dh2 head-major
        dh2 = torch.empty((5, R, H), dtype=bf, device=dev)
        dg2, dbe2 = _bn_backward(dz2, rowmajor, h2, headmajor, R, H5, st["g2"], m2, i2, a2, s2, p2,
                                 seed, pack.sites[1], dh2, headmajor, bn=pack.bns()[1][0])
        if defer:
            for i in range(5):
                gemm.defer_weight_grad(dh2[i], z1[i], P[i][3].weight)
        else:
            dw2 = torch.empty((5, H, H), dtype=torch.float32, device=dev)
            for i in range(5):
                fused_weight_grad(dh2[i], z1[i], bias=False, out_w=dw2[i])
        dz1 = (gemm.tile_bmm(dh2, w2, False) if gemm.tile_bmm_ok(dh2, w2, False)
               else torch.bmm(dh2, w2))                                          # (5, R, H)
        dh1 = torch.empty((R, H5), dtype=bf, device=dev)
        dg1, dbe1 = _bn_backward(dz1, headmajor, h1, rowmajor, R, H5, st["g1"], m1, i1, a1, s1, p1,
                                 seed, pack.sites[0], dh1, rowmajor, bn=pack.bns()[0][0])
        if defer:
            for i in range(5):
                gemm.defer_weight_grad(dh1[:, i * H:(i + 1) * H], xb, P[i][0].weight)
        else:
            dw1, _ = fused_weight_grad(dh1, xb, bias=False)
        dx = (gemm.tile_gemm(dh1, w1, trans_b=False) if gemm._tile_gemm_ok(dh1, w1, False)
              else dh1 @ w1).to(xdt)
        grads = {"g1": dg1, "b1": dbe1, "g2": dg2, "b2": dbe2}
        if not defer:
            grads.update({"w1": dw1.view(-1), "w2": dw2.view(-1)})
        out = []
        for key in ("w1", "w2", "g1", "b1", "g2", "b2"):
            if key not in grads:
                out += [None] * 5
                continue
            g = grads[key]
            step = g.numel() // 5
            shape = pack._tensors()[key][0].shape
            out += [g[i * step:(i + 1) * step].view(shape) for i in range(5)]
        return (dx, None, None, None, None, None, *out, *d3)


def _bn_backward(dz, lz, x, lx, R, C, gamma, mean, invstd, scale, shift, p, seed, site, dx, ld,
                 bn=None):
    dev = x.device
    parts = torch.empty((NPARTS, 2, C), dtype=torch.float64, device=dev)
    nat.call("ov3d_rows_bn_bwd", 0, dz, *lz, x, 1, *lx, R, C, scale, shift, mean, invstd, None, None,
             None, float(p), seed, site, parts, NPARTS, None, 0, 0, 8, like=x)
    group, world = _group_world(bn) if bn is not None else (None, 1)
    cA, cB, cC, dg, db = bn_bwd_affine(parts, NPARTS, C, group, R * world, gamma, mean, invstd)
    nat.call("ov3d_rows_bn_bwd", 1, dz, *lz, x, 1, *lx, R, C, scale, shift, mean, invstd, cA, cB, cC,
             float(p), seed, site, None, 0, dx, *ld, like=x)
    return dg, db


def fused_heads(pack, rows, sem=None, lq=0):
    """rows (R, 256) -> {head name: (R, out) fp32} for the five MLP heads (training); with
    `sem` (the sem_cls_head Linear: frozen text embedding, no bias, T <= 32) also
    "sem_cls_logits" (R, T), in the reference's transposed layout (quirk Q8) when lq = Q > 0."""
    pack.ensure()
    P = pack.parts
    p1 = P[0][2].p if P[0][2].training else 0.0
    p2 = P[0][5].p if P[0][5].training else 0.0
    text = None
    if sem is not None and text_alignment_ok(sem, P[0][6].weight.shape[0]):
        text = sem.weight
    params = []
    for key, ts in pack._tensors().items():
        if key in ("rm1", "rv1", "rm2", "rv2"):
            continue
        params += ts
    gemm.ensure_fresh(params[:10])
    params += [p[6].weight for p in P] + [p[6].bias for p in P]
    res_t = _Heads.apply(rows, pack, p1, p2, text, lq if text is not None else 0, *params)
    out_v, out_s = res_t[0], res_t[1]
    res = {HEAD_ORDER[0]: out_v, "_raw": out_s}   # _raw: [center | size | angle cls | angle res]
    if text is not None:
        res["sem_cls_logits"] = res_t[2]
    o = 0
    for name, p in zip(HEAD_ORDER[1:], P[1:]):
        n = p[6].weight.shape[0]
        res[name] = out_s[:, o:o + n]
        o += n
    return res


def text_alignment_ok(sem, nv):
    """the alignment Linear folds into the output launch: frozen (T, nv) fp32 weight, no bias"""
    w = sem.weight
    return (isinstance(sem, nn.Linear) and sem.bias is None and not w.requires_grad and w.is_cuda
            and w.dtype == torch.float32 and w.is_contiguous() and w.shape[1] == nv
            and 0 < w.shape[0] <= nat.load().ov3d_heads_out_max_text())


# ------------------------------------------------------------------------- BN + ReLU rows
class _BnReluRows(torch.autograd.Function):
    """Training BatchNorm1d (batch statistics, running-stat update) + ReLU + Dropout over
    the rows of one GenericMLP block (models/helpers.py:45-112: the encoder -> decoder
    projection, model_3detr.py:106-120), on the bnrows kernels: 4 launches each way
    instead of PyTorch's channels-last batch_norm (70 us reductions at 16384 x 256)."""

    @staticmethod
    def forward(ctx, h, gamma, beta, bn, p, site):
        R, C = h.shape
        dev = h.device
        nbt = bn.num_batches_tracked if (bn.track_running_stats and
                                         bn.num_batches_tracked is not None) else None
        rowmajor = (C, 0, C)
        mean, invstd, scale, shift = _stats_finalize(h, rowmajor, R, C, gamma, beta, [bn],
                                                     bn.running_mean, bn.running_var, nbt)
        z = torch.empty((R, C), dtype=torch.bfloat16, device=dev)
        seed = flash._seed(dev)
        nat.call("ov3d_rows_bn_apply", h, int(h.dtype == torch.bfloat16), *rowmajor, R, C, scale,
                 shift, float(p), seed if p > 0 else None, site, z, *rowmajor, like=h)
        ctx.save_for_backward(h, gamma, mean, invstd, scale, shift)
        ctx.meta = (float(p), site)
        ctx.seed = seed if p > 0 else None
        ctx.bn = bn
        return z

    @staticmethod
    def backward(ctx, dz):
        h, gamma, mean, invstd, scale, shift = ctx.saved_tensors
        p, site = ctx.meta
        R, C = h.shape
        dev = h.device
        dz = dz.to(torch.bfloat16).contiguous()
        rowmajor = (C, 0, C)
        hf = int(h.dtype == torch.bfloat16)
        seed = ctx.seed
        parts = torch.empty((NPARTS, 2, C), dtype=torch.float64, device=dev)
        nat.call("ov3d_rows_bn_bwd", 0, dz, *rowmajor, h, hf, *rowmajor, R, C, scale, shift, mean,
                 invstd, None, None, None, float(p), seed, site, parts, NPARTS, None, 0, 0, 8,
                 like=h)
        group, world = _group_world(ctx.bn)
        cA, cB, cC, dg, db = bn_bwd_affine(parts, NPARTS, C, group, R * world, gamma, mean, invstd)
        dh = torch.empty((R, C), dtype=torch.bfloat16, device=dev)
        nat.call("ov3d_rows_bn_bwd", 1, dz, *rowmajor, h, hf, *rowmajor, R, C, scale, shift, mean,
                 invstd, cA, cB, cC, float(p), seed, site, None, 0, dh, *rowmajor, like=h)
        return dh.to(h.dtype), dg, db, None, None, None


def bn_relu_rows_ok(h, bn, relu, drop):
    """the fused rows path applies: training BN (or SyncBN) with running stats, then ReLU"""
    if not (h.is_cuda and h.dim() == 2 and h.shape[1] % 8 == 0 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    return (type(bn) in _BN_ROW_TYPES and bn.training and bn.track_running_stats
            and bn.momentum is not None and bn.affine and isinstance(relu, nn.ReLU)
            and (drop is None or isinstance(drop, nn.Dropout)))


def bn_relu_rows(h, bn, drop=None):
    """z = dropout(relu(bn(h))) in bf16 for training rows h (R, C)"""
    p = drop.p if (drop is not None and drop.training) else 0.0
    site = getattr(bn, "_rows_site", None)
    if site is None:
        site = flash.new_site()
        bn._rows_site = site
    if not h.is_contiguous():
        h = h.contiguous()
    with torch.autocast("cuda", enabled=False):
        return _BnReluRows.apply(h, bn.weight, bn.bias, bn, p, site)


# ----------------------------------------------------------- BN + ReLU + neighbour max-pool
# the last SharedMLP layer of an SA module on the rows path (the masked encoder's interim SA)
# straight into the max over its nsample rows: the activated rows z are never stored (forward:
# csrc/pool.hip ov3d_nbr_max_bnrelu_fwd; backward: ov3d_rows_bn_bwd_pooled rebuilds the dense
# pooled gradient row by row); OV3D_BN_POOL=0: bn_relu_rows + the plain pool
BN_POOL = os.environ.get("OV3D_BN_POOL", "1") != "0"


class _BnReluPoolRows(torch.autograd.Function):
    """max over S neighbour rows of relu(bn(h)) (training BN, batch statistics + running-stat
    update, no dropout): the _BnReluRows arithmetic followed by pointnet2_modules._NbrMax's,
    without the (R, C) activation in between; bit-equal to the two"""

    @staticmethod
    def forward(ctx, h, gamma, beta, bn, S):
        R, C = h.shape
        dev = h.device
        nbt = bn.num_batches_tracked if (bn.track_running_stats and
                                         bn.num_batches_tracked is not None) else None
        rowmajor = (C, 0, C)
        mean, invstd, scale, shift = _stats_finalize(h, rowmajor, R, C, gamma, beta, [bn],
                                                     bn.running_mean, bn.running_var, nbt)
        P = R // S
        out = torch.empty((P, C), dtype=torch.bfloat16, device=dev)
        arg = torch.empty((P, C), dtype=torch.uint8, device=dev)
        nat.call("ov3d_nbr_max_bnrelu_fwd", h, P, S, C, scale, shift, out, arg, like=h)
        ctx.save_for_backward(h, gamma, mean, invstd, scale, shift, arg)
        ctx.S = S
        ctx.bn = bn
        return out

    @staticmethod
    def backward(ctx, g):
        h, gamma, mean, invstd, scale, shift, arg = ctx.saved_tensors
        S = ctx.S
        R, C = h.shape
        dev = h.device
        g = g.to(torch.bfloat16).contiguous()
        parts = torch.empty((NPARTS, 2, C), dtype=torch.float64, device=dev)
        nat.call("ov3d_rows_bn_bwd_pooled", 0, g, arg, S, h, R, C, scale, shift, mean, invstd, None,
                 None, None, parts, NPARTS, None, like=h)
        group, world = _group_world(ctx.bn)
        cA, cB, cC, dg, db = bn_bwd_affine(parts, NPARTS, C, group, R * world, gamma, mean, invstd)
        dh = torch.empty((R, C), dtype=torch.bfloat16, device=dev)
        nat.call("ov3d_rows_bn_bwd_pooled", 1, g, arg, S, h, R, C, scale, shift, mean, invstd, cA, cB,
                 cC, None, 0, dh, like=h)
        return dh, dg, db, None, None


def bn_relu_pool_ok(h, bn, relu, S):
    """the fused BN + ReLU + max-pool rows path applies (bf16 contiguous rows, no dropout)"""
    return (BN_POOL and bn_relu_rows_ok(h, bn, relu, None) and h.dtype == torch.bfloat16
            and h.is_contiguous() and h.data_ptr() % 16 == 0 and 0 < S <= 256
            and h.shape[0] % S == 0 and h.shape[1] % 8 == 0)


def bn_relu_pool_rows(h, bn, S):
    """(R, C) training rows h -> (R / S, C) bf16: max over each S rows of relu(bn(h))"""
    with torch.autocast("cuda", enabled=False):
        return _BnReluPoolRows.apply(h, bn.weight, bn.bias, bn, S)


# ------------------------------------------------------------- BN + ReLU into the next GEMM
# a SharedMLP layer's BatchNorm + ReLU applied while the next layer's 256 x 256 product stages
# its rows (csrc/rows256.hip ov3d_rows256_bn, the masked encoder's interim SA: 2^18 rows): no
# separate apply pass and no activation rows -- the weight gradient applies the same BN + ReLU
# as it loads the pre-BN rows (ov3d_wgrad_bn).  OV3D_BN_GEMM=0: bn_relu_rows + the product
BN_GEMM = os.environ.get("OV3D_BN_GEMM", "1") != "0"


class _BnReluLinearRows(torch.autograd.Function):
    """y = relu(bn(h)) w^T (training BN, no dropout, no bias): the _BnReluRows and
    gemm._RowsLinear arithmetic in their order, bit-equal to the two; the weight gradient
    dy^T relu(bn(h)) is deferred the same way, its input rebuilt from h on load"""

    @staticmethod
    def forward(ctx, h, gamma, beta, bn, w):
        R, C = h.shape
        dev = h.device
        nbt = bn.num_batches_tracked if (bn.track_running_stats and
                                         bn.num_batches_tracked is not None) else None
        rowmajor = (C, 0, C)
        mean, invstd, scale, shift = _stats_finalize(h, rowmajor, R, C, gamma, beta, [bn],
                                                     bn.running_mean, bn.running_var, nbt)
        wc = gemm.cast_param(w, torch.bfloat16)
        y = torch.empty((R, wc.shape[0]), dtype=torch.bfloat16, device=dev)
        nat.call("ov3d_rows256_bn", h, h.stride(0), scale, shift, wc, wc.stride(0), y, y.stride(0),
                 None, 0, R, gemm._rows256_counters(dev), like=h)
        ctx.save_for_backward(h, gamma, mean, invstd, scale, shift, wc)
        ctx.bn = bn
        ctx.w = w
        return y

    @staticmethod
    def backward(ctx, dy):
        h, gamma, mean, invstd, scale, shift, wc = ctx.saved_tensors
        w = ctx.w
        R, C = h.shape
        dev = h.device
        dy = dy.to(torch.bfloat16).contiguous()
        dw = None
        with torch.autocast("cuda", enabled=False):
            dz = gemm._dgrad(dy, wc)                      # gemm._RowsLinear's input gradient
            # its weight gradient dy^T relu(bn(h)), the activation applied on load
            if gemm.can_defer(h, w):
                gemm.defer_weight_grad(dy, h, w, bn=(scale, shift))
            else:
                dw = gemm.fused_weight_grad(dy, h, bias=False, bn=(scale, shift))[0].to(w.dtype)
        rowmajor = (C, 0, C)
        parts = torch.empty((NPARTS, 2, C), dtype=torch.float64, device=dev)
        nat.call("ov3d_rows_bn_bwd", 0, dz, *rowmajor, h, 1, *rowmajor, R, C, scale, shift, mean,
                 invstd, None, None, None, 0.0, None, 0, parts, NPARTS, None, 0, 0, 8, like=h)
        group, world = _group_world(ctx.bn)
        cA, cB, cC, dg, db = bn_bwd_affine(parts, NPARTS, C, group, R * world, gamma, mean, invstd)
        dh = torch.empty((R, C), dtype=torch.bfloat16, device=dev)
        nat.call("ov3d_rows_bn_bwd", 1, dz, *rowmajor, h, 1, *rowmajor, R, C, scale, shift, mean,
                 invstd, cA, cB, cC, 0.0, None, 0, None, 0, dh, *rowmajor, like=h)
        return dh, dg, db, None, dw


def bn_relu_linear_ok(h, bn, relu, w, b):
    """the fused BN + ReLU -> 256 x 256 product applies (bf16 contiguous rows on rows256)"""
    return (BN_GEMM and gemm.ROWS256 and b is None and bn_relu_rows_ok(h, bn, relu, None)
            and h.dtype == torch.bfloat16 and h.is_contiguous() and h.data_ptr() % 16 == 0
            and h.shape[1] == 256 and h.shape[0] >= gemm.GEMM256_MIN_M
            and tuple(w.shape[:2]) == (256, 256) and w.numel() == 256 * 256 and w.is_contiguous()
            and bool(nat.load().ov3d_rows256_supported(h.shape[0], 256, 256)))


def bn_relu_linear_rows(h, bn, w):
    """(R, 256) training rows h -> relu(bn(h)) w^T (R, 256) bf16"""
    with torch.autocast("cuda", enabled=False):
        return _BnReluLinearRows.apply(h, bn.weight, bn.bias, bn, w)
