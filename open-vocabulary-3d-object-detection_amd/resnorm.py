"""Residual add + dropout + LayerNorm of the pre-norm transformer layers as one HIP
launch each way (csrc/resnorm.hip, ``ov3d_resnorm_fwd`` / ``ov3d_resnorm_bwd``).

Reference: models/transformer.py — every pre-norm sub-layer ends with
``x = x + dropout(branch)`` (forward_pre, 262-280 / 355-379), the next starts with
``norm(x)`` (+ ``pos`` / ``query_pos`` for the attention inputs), and the decoder applies
its final norm to every layer output (return_intermediate, 124-133).  A ``Pending``
residual (stream value, branch output not yet added, its dropout) is carried from one
sub-layer to the next and resolved inside the next norm's launch:

    s, xa, xap, xb = resnorm(Pending(src, y, p, site), norm_a, pos, norm_b)
    s   = src + dropout_p(y)           (fp32)
    xa  = bf16(norm_a(s)),  xap = bf16(norm_a(s) + pos),  xb = norm_b(s) (fp32)

Dropout keep masks are the counter hash of csrc/rowdrop.h (seed of attention.py, one
site per call site), regenerated in the backward.  Under bf16 autocast only: the fp32
path keeps the plain module code, which is what the parity tests compare against.
"""
import os
from collections import namedtuple

import torch
from torch import nn

from . import _native
from . import attention as flash
from . import gemm

Pending = namedtuple("Pending", "src y p site")
# a branch output not yet computed: y = x w^T + b (the sub-layer's output projection / FFN
# linear2); the decoder's lngemm launch (resnorm_gemm) computes it in place of a y operand, the
# plain resnorm() resolves it with a rows GEMM first
LinY = namedtuple("LinY", "x w b relu_p", defaults=(None,))
# relu_p (FFN linear2): x is dropout_p(relu(h)); the input gradient then takes the FFN's
# activation mask in its epilogue (dx = x > 0 ? dy w / (1 - p) : 0), as _FFN's backward does


class FanIn:
    """Gradient fan-in of one tensor over the resnorm calls that read it (the decoder's
    query_pos in 16 calls, its final norm's weight / bias in 8).  Autograd would return a
    gradient from every call and add them (15 + 14 small add launches per step); here the
    backward of the call that runs first writes the shared buffer, the others add to it
    inside their launch (``accumulate``), and the call that runs last returns the sum — the
    others return None.  The calls are chained through the residual stream, so their
    backward order is fixed and the sum is the one autograd forms, in the same order."""

    def __init__(self):
        self.n = 0       # calls registered in the forward
        self.seen = 0    # backward calls so far
        self.bufs = None

    def take(self):
        """-> (first, last) for the next backward call"""
        k = self.seen
        self.seen += 1
        last = self.seen == self.n
        if last:
            self.seen = 0
        return k == 0, last

enabled = True   # False: the plain module code under autocast as well (tests compare the two)
fan_in = True    # False: every call returns its own pos / norm_b gradient (autograd sums them)
fused_ffn = os.environ.get("OV3D_FUSED_FFN", "1") != "0"   # _FFN on short row blocks


def supported(x, *norms):
    C = x.shape[-1]
    if not (enabled and x.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    if not _native.load().ov3d_resnorm_supported(C):
        return False
    eps = None
    for n in norms:
        if n is None:
            continue
        if type(n) is not nn.LayerNorm or not n.elementwise_affine or n.bias is None or \
                tuple(n.normalized_shape) != (C,):
            return False
        if eps is not None and n.eps != eps:
            return False
        eps = n.eps
    return True


def _dt_flag(t):
    if t is None:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise TypeError(f"resnorm: unsupported dtype {t.dtype}")


def _rows(t, C):
    if t is None:
        return None
    if t.dtype not in (torch.float32, torch.bfloat16):
        t = t.float()
    return t.reshape(-1, C).contiguous()


class _ResNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, src, y, pos, ga, ba, gb, bb):
        p, site, want_a, want_ap, want_b, eps, shape, fans, xb_into = meta
        C = shape[-1]
        srcr, yr, posr = _rows(src, C), _rows(y, C), _rows(pos, C)
        R = 1
        for d in shape[:-1]:
            R *= d
        dev = next(t.device for t in (srcr, yr, ga, gb) if t is not None)
        s = torch.empty((R, C), dtype=torch.float32, device=dev)
        norm = want_a or want_ap or want_b
        mean = torch.empty(R, dtype=torch.float32, device=dev) if norm else None
        rstd = torch.empty(R, dtype=torch.float32, device=dev) if norm else None
        xa = torch.empty((R, C), dtype=torch.bfloat16, device=dev) if want_a else None
        xap = torch.empty((R, C), dtype=torch.bfloat16, device=dev) if want_ap else None
        xb_map = (0, 0, 0)
        if want_b and xb_into is not None:
            # (Q, B, C) rows written as bf16 into layer l of the (L, B, Q, C) heads input
            out, l = xb_into
            xb = out[l]
            xb_map = (shape[1], C, shape[0] * C)
        else:
            xb = torch.empty((R, C), dtype=torch.float32, device=dev) if want_b else None
        seed = flash._seed(dev) if p > 0 else None
        _native.call("ov3d_resnorm_fwd", R, C, srcr, _dt_flag(srcr), yr, _dt_flag(yr), float(p),
                     seed, site, ga, ba, posr, _dt_flag(posr), gb, bb, float(eps), s, mean, rstd,
                     xa, xap, xb, _dt_flag(xb), *xb_map, like=s)
        ctx.save_for_backward(s, mean, rstd, ga, gb)
        ctx.seed = seed   # the forward's dropout snapshot (attention._seed)
        ctx.params = (ga, ba, gb, bb)
        ctx.set_materialize_grads(False)   # unused outputs: no zero-filled gradients
        ctx.meta = (p, site, R, C, shape, src.dtype if src is not None else None,
                    y.dtype if y is not None else None, pos.dtype if pos is not None else None)
        ctx.fans = fans
        v = lambda t: t.view(shape) if t is not None else None   # noqa: E731
        if xb_map[0]:
            return v(s), v(xa), v(xap), xb.transpose(0, 1)
        return v(s), v(xa), v(xap), v(xb)

    @staticmethod
    def backward(ctx, ds, dxa, dxap, dxb):
        return (None,) + _bwd_core(ctx, ds, dxa, dxap, dxb, ctx.needs_input_grad)


def _bwd_core(ctx, ds, dxa, dxap, dxb, need, fused=None):
    """the resnorm backward launch; need = needs_input_grad over (meta, src, y, pos, ga, ba,
    gb, bb) -> (dsrc, dy, dpos, dga, dba, dgb, dbb) (views of the forward's shapes).
    fused = (w, relu_p, h, dx): the branch y = h w^T + b's input gradient dx = epi(dy w) is
    computed in the same launch (csrc/lngemm.hip) into dx; dy is then always produced."""
    p, site, R, C, shape, src_dt, y_dt, pos_dt = ctx.meta
    s, mean, rstd, ga, gb = ctx.saved_tensors[:5]
    dev = s.device

    def g(t, dt):
        return t.reshape(R, C).to(dt).contiguous() if t is not None else None

    # the decoder's layer outputs reach here as strided (L, B, C) views of the stacked
    # outputs' gradient: read in place (row r at (r // B) * s0 + (r % B) * s1)
    xb_map = (0, 0, 0)
    if dxb is not None and dxb.dtype in (torch.float32, torch.bfloat16) and dxb.dim() == 3 and \
            dxb.stride(2) == 1 and not dxb.is_contiguous() and len(shape) == 3 and \
            tuple(dxb.shape) == tuple(shape) and dxb.stride(0) >= C and dxb.stride(1) >= C:
        xb_map = (shape[1], dxb.stride(0), dxb.stride(1))
    ds, dxa, dxap = g(ds, torch.float32), g(dxa, torch.bfloat16), g(dxap, torch.bfloat16)
    if not xb_map[0]:
        dxb = g(dxb, torch.float32)
    if ga is None:
        dxa = dxap = None
    if gb is None:
        dxb = None
    dsrc = torch.empty((R, C), dtype=torch.float32, device=dev) if need[1] else None
    dy = torch.empty((R, C), dtype=y_dt, device=dev) if need[2] else None
    dpos = torch.empty((R, C), dtype=pos_dt, device=dev) if (need[3] and dxap is not None) else None
    has_a = dxa is not None or dxap is not None
    has_b = dxb is not None
    dga = torch.empty(C, dtype=torch.float32, device=dev) if (need[4] and has_a) else None
    dba = torch.empty(C, dtype=torch.float32, device=dev) if (need[5] and has_a) else None
    dgb = torch.empty(C, dtype=torch.float32, device=dev) if (need[6] and has_b) else None
    dbb = torch.empty(C, dtype=torch.float32, device=dev) if (need[7] and has_b) else None
    acc = 0
    pos_fan, nb_fan = ctx.fans
    # LayerNorm weight / bias gradients: deferred to one grouped launch at the end of the
    # backward (with the weight gradients, gemm.DEFER_WGRAD) from this call's partials
    params = ctx.params
    defer_norm = gemm.DEFER_WGRAD and not torch.is_grad_enabled() and (has_a or has_b) and all(
        t is None or gemm._leaf_param(t) is t for t in params)
    slots = []
    if defer_norm:
        for k, (nd, have) in enumerate(((need[4], has_a), (need[5], has_a),
                                        (need[6], has_b), (need[7], has_b))):
            if nd and have:
                slots.append((k, params[k]))
        dga = dba = dgb = dbb = None
        nb_fan = None
    ret_pos = ret_nb = True
    if pos_fan is not None and need[3]:
        first, ret_pos = pos_fan.take()
        if first:   # this call's gradient (or zeros) starts the sum
            pos_fan.bufs = dpos if dpos is not None else \
                torch.zeros((R, C), dtype=pos_dt, device=dev)
        elif dpos is not None:
            dpos, acc = pos_fan.bufs, acc | 1
        if ret_pos:
            dpos_ret, pos_fan.bufs = pos_fan.bufs, None
    if nb_fan is not None and (need[6] or need[7]):
        first, ret_nb = nb_fan.take()
        if first:
            z = lambda t, n: t if t is not None or not n else \
                torch.zeros(C, dtype=torch.float32, device=dev)   # noqa: E731
            nb_fan.bufs = (z(dgb, need[6]), z(dbb, need[7]))
        elif has_b:
            dgb, dbb = nb_fan.bufs
            acc |= 4
        if ret_nb:
            nb_ret, nb_fan.bufs = nb_fan.bufs, None
    lib = _native.load()
    nparts = lib.ov3d_lngemm_bwd_parts(R) if fused is not None else lib.ov3d_resnorm_bwd_parts(R, C)
    partials = torch.empty((nparts, 4, C), dtype=torch.float32, device=dev) \
        if (has_a or has_b) else None
    seed = ctx.seed if (p > 0 and dy is not None) else None
    if fused is not None:
        w, relu_p, h, dx = fused
        if dy is None:
            dy = torch.empty((R, C), dtype=torch.bfloat16, device=dev)
        seed = ctx.seed if p > 0 else None
        _native.call("ov3d_lngemm_bwd", R, s, mean, rstd, ds, dxa, dxap, dxb, _dt_flag(dxb),
                     *xb_map, ga, gb, float(p), seed, site, dsrc, dy, dpos, _dt_flag(dpos),
                     partials, acc, w, w.stride(0), w.shape[1], 2 if relu_p is not None else 0,
                     float(relu_p or 0.0), h, h.stride(0) if h is not None else 0, dx, dx.stride(0),
                     like=s)
        if not slots and (dga is not None or dba is not None or dgb is not None or dbb is not None):
            _colsums(partials, nparts, C, (dga, dba, dgb, dbb), acc)
    elif dsrc is not None or dy is not None or dpos is not None or has_a or has_b:
        _native.call("ov3d_resnorm_bwd", R, C, s, mean, rstd, ds, dxa, dxap, dxb, _dt_flag(dxb),
                     *xb_map, ga, gb,
                     float(p) if dy is not None else 0.0, seed, site, dsrc, dy, _dt_flag(dy),
                     dpos, _dt_flag(dpos), partials, nparts, dga, dba,
                     dgb, dbb, acc, like=s)
    if slots:
        gemm.defer_norm_grads(partials, nparts, C, slots)
    v = lambda t: t.view(shape) if t is not None else None   # noqa: E731
    if dsrc is not None and src_dt != torch.float32:
        dsrc = dsrc.to(src_dt)
    if pos_fan is not None and need[3]:
        dpos = dpos_ret if ret_pos else None
    if nb_fan is not None and (need[6] or need[7]):
        dgb, dbb = nb_ret if ret_nb else (None, None)
    if defer_norm:
        dga = dba = dgb = dbb = None
    return v(dsrc), v(dy), v(dpos), dga, dba, dgb, dbb


def _colsums(partials, nparts, C, outs, acc):
    """LayerNorm parameter gradients (dga, dba, dgb, dbb) from (nparts, 4, C) partials in
    one ov3d_colsum_group launch (the fixed summation order of resnorm_bwd's own column
    pass); acc bits 2 / 4: add into dga / dba, dgb / dbb (gradient fan-in)."""
    from .gemm import _ColSeg, _ColOut
    import ctypes
    tmp = torch.empty((4, C), dtype=torch.float32, device=partials.device)
    segs = (_ColSeg * 4)(*[_ColSeg(partials.data_ptr(), nparts, k) for k in range(4)])
    oa = (_ColOut * 4)(*[_ColOut(tmp[k].data_ptr(), k, 1) for k in range(4)])
    _native.call("ov3d_colsum_group", ctypes.addressof(segs), 4, ctypes.addressof(oa), 4, C,
                 like=partials)
    for k, o in enumerate(outs):
        if o is None:
            continue
        if acc & (2 if k < 2 else 4):
            o.add_(tmp[k])
        else:
            o.copy_(tmp[k])


class _RowsLinearMask(torch.autograd.Function):
    """y = h w^T + b for the FFN's linear2 whose input h = dropout_p(relu(.)) came from a
    relu-drop epilogue (LinY with relu_p): the input gradient takes the activation mask in
    its epilogue (dx = h > 0 ? dy w / (1 - p) : 0), the convention of _LnGemm."""

    @staticmethod
    def forward(ctx, h, w, b, relu_p):
        bf = torch.bfloat16
        hr = h.reshape(-1, h.shape[-1])
        wc, bc = gemm.cast_param(w, bf), gemm.cast_param(b, bf)
        with torch.autocast("cuda", enabled=False):
            y = gemm.act_gemm(hr, wc, _bias(bc), True)
        ctx.save_for_backward(hr, wc)
        ctx.params = (w, b)
        ctx.meta = (h.shape, float(relu_p))
        return y.view(*h.shape[:-1], wc.shape[0])

    @staticmethod
    def backward(ctx, dy):
        hr, wc = ctx.saved_tensors
        w, b = ctx.params
        hshape, relu_p = ctx.meta
        need = ctx.needs_input_grad
        dyr = dy.reshape(-1, wc.shape[0]).to(torch.bfloat16).contiguous()
        with torch.autocast("cuda", enabled=False):
            dx = gemm.act_gemm(dyr, wc, None, False, 2, relu_p, h=hr).view(hshape) \
                if need[0] else None
            dw, db = gemm.linear_weight_grads(dyr, hr, w, b, need[1], b is not None and need[2])
        return dx, dw, db, None


# LayerNorm boundary + the following row GEMM in one launch each way (csrc/lngemm.hip), the
# decoder's sub-layer boundaries; OV3D_LNGEMM=0: the resnorm + rows-GEMM launches
lngemm = os.environ.get("OV3D_LNGEMM", "1") != "0"


class _LnGemm(torch.autograd.Function):
    """resnorm(Pending(src, y, p, site)) feeding a linear layer directly:
        s = src + dropout_p(y);  xa = norm_a(s);  xap = xa + pos;  xb = norm_b(s)
        out_i = epi(xsel_i W[r0_i:r1_i]^T + b[r0_i:r1_i])       (xsel: xa or xap)
    y is a LinY (x w_y^T + b_y, computed here by a rows GEMM launch, its input gradient then
    fused into the resnorm backward launch) or a bf16 tensor or None.  The outputs are s, xb
    (None unless norm_b) and the out_i; xa / xap stay internal (saved for the backward).
    Forward: [y GEMM] + ONE lngemm launch; backward: the out_i input gradients (one rows-GEMM
    launch) + ONE lngemm launch (resnorm backward + dx of y's linear) — the two-launch
    resnorm / GEMM pairs of models/transformer.py:355-379's boundaries each become one."""

    @staticmethod
    def forward(ctx, meta, src, yx, yw, yb, pos, ga, ba, gb, bb, gw, gbias):
        p, site, eps, shape, fans, xb_into, relu_p, spec, epi = meta
        bf = torch.bfloat16
        C = shape[-1]
        R = 1
        for d in shape[:-1]:
            R *= d
        dev = ga.device
        lin = yw is not None
        ywc = gemm.cast_param(yw, bf) if lin else None
        if lin:
            yr = yx.reshape(-1, yx.shape[-1])
            with torch.autocast("cuda", enabled=False):
                y = gemm.act_gemm(yr, ywc, _bias(gemm.cast_param(yb, bf)), True)
        else:
            yr = None
            y = _rows(yx, C).to(bf).contiguous() if yx is not None else None
        srcr, posr = _rows(src, C), _rows(pos, C)
        s = torch.empty((R, C), dtype=torch.float32, device=dev)
        mean = torch.empty(R, dtype=torch.float32, device=dev)
        rstd = torch.empty(R, dtype=torch.float32, device=dev)
        use_a = any(sel == 0 for sel, _, _ in spec)
        use_ap = any(sel == 1 for sel, _, _ in spec)
        xa = torch.empty((R, C), dtype=bf, device=dev) if use_a else None
        xap = torch.empty((R, C), dtype=bf, device=dev) if use_ap else None
        want_b = gb is not None
        xb_map = (0, 0, 0)
        if want_b and xb_into is not None:
            out, l = xb_into
            xb = out[l]
            xb_map = (shape[1], C, shape[0] * C)
        else:
            xb = torch.empty((R, C), dtype=torch.float32, device=dev) if want_b else None
        gwc, gbc = gemm.cast_param(gw, bf), gemm.cast_param(gbias, bf)
        outs, probs = [], []
        from .gemm import _LnProblem
        import ctypes
        for sel, r0, r1 in spec:
            o = torch.empty((R, r1 - r0), dtype=bf, device=dev)
            w_i = gwc[r0:r1]
            b_i = gbc[r0:r1] if gbc is not None else None
            outs.append(o)
            probs.append(_LnProblem(w_i.data_ptr(), w_i.stride(0),
                                    b_i.data_ptr() if b_i is not None else None,
                                    o.data_ptr(), o.stride(0), r1 - r0, sel))
        arr = (_LnProblem * len(probs))(*probs)
        seed = flash._seed(dev) if (p > 0 or (epi is not None and epi[0] > 0)) else None
        ep, esite = (float(epi[0]), int(epi[1])) if epi is not None else (0.0, 0)
        _native.call("ov3d_lngemm_fwd", R, srcr, _dt_flag(srcr), y, float(p) if y is not None else 0.0,
                     seed if p > 0 else None, site, ga, ba, posr, _dt_flag(posr), gb, bb, float(eps),
                     s, mean, rstd, xa, xap, xb, _dt_flag(xb), *xb_map, len(probs),
                     ctypes.addressof(arr), 1 if epi is not None else 0, ep,
                     seed if ep > 0 else None, esite, like=s)
        ctx.save_for_backward(s, mean, rstd, ga, gb, xa, xap, yr, ywc, gwc)
        ctx.seed = seed
        ctx.params = (ga, ba, gb, bb)
        ctx.lin = (yw, yb, gw, gbias)
        ctx.set_materialize_grads(False)
        ctx.meta = (p if y is not None else 0.0, site, R, C, shape,
                    src.dtype if src is not None else None, bf if y is not None else None,
                    pos.dtype if pos is not None else None)
        ctx.spec = spec
        ctx.relu_p = relu_p
        ctx.ydt = (yx.shape, yx.dtype) if yx is not None else None
        ctx.fans = fans
        v = lambda t: t.view(shape) if t is not None else None   # noqa: E731
        xbo = xb.transpose(0, 1) if xb_map[0] else v(xb)
        return (v(s), xbo) + tuple(o.view(*shape[:-1], o.shape[1]) for o in outs)

    @staticmethod
    def backward(ctx, ds, dxb, *douts):
        s, mean, rstd, ga, gb, xa, xap, yr, ywc, gwc = ctx.saved_tensors
        yw, yb, gw, gbias = ctx.lin
        nig = ctx.needs_input_grad   # meta, src, yx, yw, yb, pos, ga, ba, gb, bb, gw, gbias
        p, site, R, C, shape = ctx.meta[:5]
        spec = ctx.spec
        bf = torch.bfloat16
        dev = s.device
        with torch.autocast("cuda", enabled=False):
            d = [dd.reshape(R, -1).to(bf).contiguous() if dd is not None else None for dd in douts]
            # the linear's input gradients: dxa (sel 0 problems), dxap (sel 1), one launch
            pairs = [(d[i], gwc[r0:r1], sel) for i, (sel, r0, r1) in enumerate(spec)
                     if d[i] is not None]
            dsel = {0: None, 1: None}
            if len(pairs) > 1 and gemm._group_ok([(a, w) for a, w, _ in pairs], False) and \
                    len({sel for _, _, sel in pairs}) == len(pairs):
                for (_, _, sel), o in zip(pairs, gemm.rows_gemm_group(
                        [(a, w, None) for a, w, _ in pairs], trans_b=False)):
                    dsel[sel] = o
            else:
                for a, w, sel in pairs:
                    o = gemm._dgrad(a, w)
                    dsel[sel] = o if dsel[sel] is None else dsel[sel] + o
            lin = ywc is not None
            need_y = lin and (nig[2] or nig[3] or nig[4])
            need = (False, nig[1], need_y or (not lin and nig[2]), nig[5], nig[6], nig[7], nig[8],
                    nig[9])
            dx = None
            fused = None
            if lin and nig[2]:
                dx = torch.empty((R, ywc.shape[1]), dtype=bf, device=dev)
                fused = (ywc, ctx.relu_p, yr if ctx.relu_p is not None else None, dx)
            if dsel[0] is None and dsel[1] is None and dxb is None:
                fused = None   # nothing reaches the norm: plain resnorm backward
            dsrc, dy, dpos, dga, dba, dgb, dbb = _bwd_core(ctx, ds, dsel[0], dsel[1], dxb, need,
                                                           fused=fused)
            dyw = dyb = None
            if lin:
                dyr = dy.reshape(R, C) if dy is not None else None
                if fused is None and nig[2] and dyr is not None:
                    if ctx.relu_p is not None:
                        dx = gemm.act_gemm(dyr, ywc, None, False, 2, ctx.relu_p, h=yr)
                    else:
                        dx = gemm._dgrad(dyr, ywc)
                if dyr is not None and (nig[3] or (yb is not None and nig[4])):
                    dyw, dyb = gemm.linear_weight_grads(dyr, yr, yw, yb, nig[3], nig[4])
                dyx = dx.view(ctx.ydt[0]).to(ctx.ydt[1]) if dx is not None else None
            else:
                dyx = dy
            # the linear's weight / bias gradients (row blocks of one weight, as _InProj)
            dgw = dgbias = None
            want_b = gbias is not None and nig[11]
            if nig[10] or want_b:
                items = [(d[i], xap if sel == 1 else xa, (r0, r1))
                         for i, (sel, r0, r1) in enumerate(spec) if d[i] is not None]
                if nig[10] and all(gemm.can_defer(x, gw, gbias if want_b else None)
                                   for _, x, _ in items):
                    for dd, x, rows in items:
                        gemm.defer_weight_grad(dd, x, gw, gbias if want_b else None, rows=rows)
                else:
                    dgw = torch.zeros(gw.shape, dtype=torch.float32, device=dev) if nig[10] else None
                    dgbias = torch.zeros(gbias.shape, dtype=torch.float32, device=dev) \
                        if want_b else None
                    for dd, x, (r0, r1) in items:
                        if dgw is not None and gemm._fused_ok(dd, x):
                            gemm.fused_weight_grad(dd, x, bias=dgbias is not None,
                                                   out_w=dgw[r0:r1],
                                                   out_b=dgbias[r0:r1] if dgbias is not None else None)
                            continue
                        if dgw is not None:
                            gemm.weight_grad(dd, x, out=dgw[r0:r1])
                        if dgbias is not None:
                            torch.sum(dd, dim=0, dtype=torch.float32, out=dgbias[r0:r1])
                    dgw = dgw.to(gw.dtype) if dgw is not None else None
                    dgbias = dgbias.to(gbias.dtype) if dgbias is not None else None
        return (None, dsrc, dyx, dyw, dyb, dpos, dga, dba, dgb, dbb, dgw, dgbias)


def resnorm_gemm(pend, norm_a, w, b, spec, pos=None, norm_b=None, pos_fan=None, norm_b_fan=None,
                 xb_into=None, epi=None):
    """-> (s, xb, [out_i]) of _LnGemm, or None when the fused launches do not apply (the
    caller then runs resnorm() and the linear layer).  spec: ((sel, r0, r1), ...) with sel
    0 = norm_a(s), 1 = norm_a(s) + pos as the input of out_i = xsel W[r0:r1]^T + b[r0:r1];
    epi = (p, site): out = dropout_p(relu(.)) (one problem)."""
    src, y, p, psite = pend
    if not (lngemm and enabled and src is not None and norm_a is not None and len(spec) <= 2):
        return None
    ref = src
    shape = tuple(ref.shape)
    C = shape[-1]
    R = ref.numel() // C
    lib = _native.load()
    if not (ref.is_cuda and w.is_cuda and w.dim() == 2 and w.shape[1] == C
            and all(lib.ov3d_lngemm_supported(R, C, r1 - r0) for _, r0, r1 in spec)):
        return None
    if any(sel == 1 for sel, _, _ in spec) and pos is None:
        return None
    if isinstance(y, LinY):
        x = y.x
        if not (x.dtype == torch.bfloat16 and tuple(y.w.shape) == (C, x.shape[-1])
                and lib.ov3d_lngemm_supported(R, C, x.shape[-1])
                and gemm.act_gemm_ok(x.reshape(-1, x.shape[-1]), gemm.cast_param(y.w, torch.bfloat16), True)):
            return None
        yx, yw, yb, relu_p = x, y.w, y.b, y.relu_p
    else:
        if y is not None and (tuple(y.shape) != shape or y.dtype != torch.bfloat16):
            return None
        yx, yw, yb, relu_p = y, None, None, None
    eps = norm_a.eps
    if norm_b is not None and norm_b.eps != eps:
        return None
    want_ap = any(sel == 1 for sel, _, _ in spec)
    if not (fan_in and want_ap and pos is not None and pos.requires_grad):
        pos_fan = None
    if norm_b is None or not fan_in:
        norm_b_fan = None
    for fan in (pos_fan, norm_b_fan):
        if fan is not None:
            fan.n += 1
    if norm_b is None or len(shape) != 3:
        xb_into = None
    meta = (float(p) if y is not None else 0.0, int(psite), eps, shape, (pos_fan, norm_b_fan),
            xb_into, relu_p, tuple(spec), epi)
    gb_ = norm_b.weight if norm_b is not None else None
    bb_ = norm_b.bias if norm_b is not None else None
    with torch.autocast("cuda", enabled=False):
        r = _LnGemm.apply(meta, src, yx, yw, yb, pos if want_ap else None, norm_a.weight,
                          norm_a.bias, gb_, bb_, w, b)
    return r[0], r[1], list(r[2:])


def resolve(y):
    """a LinY branch computed on its own (rows GEMM); other values unchanged"""
    if isinstance(y, LinY):
        if y.relu_p is not None:   # its gradient must carry the FFN mask (_RowsLinearMask)
            with torch.autocast("cuda", enabled=False):
                return _RowsLinearMask.apply(y.x, y.w, y.b, y.relu_p)
        return gemm.rows_linear(y.x, y.w, y.b)
    return y


def resnorm(pend, norm_a=None, pos=None, want_a=True, want_ap=False, norm_b=None, pos_fan=None,
            norm_b_fan=None, xb_into=None):
    """-> (s, xa, xap, xb) for Pending(src, y, p, site); unwanted outputs are None.
    pos_fan / norm_b_fan: FanIn shared by the calls that read the same pos / norm_b.
    xb_into = (out, l): xb of these (Q, B, C) rows is written in bf16 into out[l] of an
    (L, B, Q, C) buffer (the heads' row order) and returned as that (Q, B, C) view."""
    src, y, p, psite = pend
    if isinstance(y, LinY):
        y = resolve(y)
    ref = y if y is not None else src
    shape = tuple(ref.shape)
    if norm_a is None:
        want_a = want_ap = False
    if want_ap and pos is None:
        raise ValueError("resnorm: xap needs pos")
    eps = (norm_a.eps if norm_a is not None else (norm_b.eps if norm_b is not None else 1e-5))
    if not (fan_in and want_ap and pos is not None and pos.requires_grad):
        pos_fan = None
    if norm_b is None or not fan_in:
        norm_b_fan = None
    for fan in (pos_fan, norm_b_fan):
        if fan is not None:
            fan.n += 1
    if norm_b is None or len(shape) != 3:
        xb_into = None
    meta = (float(p) if y is not None else 0.0, int(psite), bool(want_a), bool(want_ap),
            norm_b is not None, eps, shape, (pos_fan, norm_b_fan), xb_into)
    ga = norm_a.weight if norm_a is not None else None
    ba = norm_a.bias if norm_a is not None else None
    gb = norm_b.weight if norm_b is not None else None
    bb = norm_b.bias if norm_b is not None else None
    with torch.autocast("cuda", enabled=False):
        return _ResNorm.apply(meta, src, y, pos if want_ap else None, ga, ba, gb, bb)


class Gather(torch.autograd.Function):
    """The decoder's layer outputs as ONE (L, Q, B, C) tensor without a copy: every layer's
    resnorm launch already wrote its rows into `out` (xb_into), so the forward returns
    out's (L, Q, B, C) view and the backward hands each layer its (Q, B, C) slice of the
    gradient as a strided view (read in place by the resnorm backward)."""

    @staticmethod
    def forward(ctx, out, *layers):
        ctx.n = len(layers)
        return out.permute(0, 2, 1, 3)

    @staticmethod
    def backward(ctx, g):
        return (None,) + tuple(g[l] for l in range(ctx.n))


def sites(module, n):
    """n dropout hash sites owned by `module` (allocated once)"""
    s = getattr(module, "_resnorm_sites", ())
    if len(s) < n:
        s = tuple(s) + tuple(flash.new_site() for _ in range(n - len(s)))
        module._resnorm_sites = s
    return s[:n]


class _ReluDropout(torch.autograd.Function):
    """h = dropout_p(relu(y)) on bf16 rows in one launch each way (csrc/resnorm.hip)."""

    @staticmethod
    def forward(ctx, y, p, site):
        C = y.shape[-1]
        yr = y.reshape(-1, C).contiguous()
        h = torch.empty_like(yr)
        seed = flash._seed(y.device) if p > 0 else None
        _native.call("ov3d_relu_dropout_fwd", yr, yr.shape[0], C, float(p), seed, site, h, like=yr)
        ctx.save_for_backward(h)
        ctx.p = float(p)
        ctx.yshape = y.shape
        return h.view(y.shape)

    @staticmethod
    def backward(ctx, dh):
        (h,) = ctx.saved_tensors
        dh = dh.to(h.dtype).reshape(h.shape).contiguous()
        dy = torch.empty_like(h)
        _native.call("ov3d_relu_dropout_bwd", h, dh, h.numel(), ctx.p, dy, like=h)
        return dy.view(ctx.yshape), None, None


class _FFN(torch.autograd.Function):
    """linear2(dropout(relu(linear1(x)))) on short bf16 row blocks (the decoder's FFN,
    models/transformer.py:375-377): the activation is the epilogue of linear1's rowsgemm
    launch forward, and of linear2's input-gradient launch backward (ov3d_rows_gemm_act),
    so the FFN is two launches each way (+ its weight gradients, deferred with the others)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, p, site):
        bf = torch.bfloat16
        C = x.shape[-1]
        xc = x.reshape(-1, C)
        w1c, b1c = gemm.cast_param(w1, bf), gemm.cast_param(b1, bf)
        w2c, b2c = gemm.cast_param(w2, bf), gemm.cast_param(b2, bf)
        M, F, N = xc.shape[0], w1c.shape[0], w2c.shape[0]
        seed = flash._seed(x.device) if p > 0 else None
        h = gemm.act_gemm(xc, w1c, _bias(b1c), True, 1, p, seed, site)
        y = gemm.act_gemm(h, w2c, _bias(b2c), True)
        ctx.save_for_backward(xc, h, w1c, w2c)
        ctx.params = (w1, b1, w2, b2)
        ctx.meta = (float(p), x.shape, x.dtype)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        xc, h, w1c, w2c = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        p, xshape, xdt = ctx.meta
        need = ctx.needs_input_grad
        M, F, N = h.shape[0], h.shape[1], w2c.shape[0]
        dy = dy.reshape(-1, N).to(torch.bfloat16).contiguous()
        dy1 = gemm.act_gemm(dy, w2c, None, False, 2, p, h=h)
        dw2, db2 = gemm.linear_weight_grads(dy, h, w2, b2, need[3], need[4])
        dw1, db1 = gemm.linear_weight_grads(dy1, xc, w1, b1, need[1], need[2])
        dx = gemm.act_gemm(dy1, w1c, None, False).to(xdt).view(xshape) if need[0] else None
        return dx, dw1, db1, dw2, db2, None, None


def _bias(b):
    return b.contiguous() if b is not None else None


def _ffn_ok(x, linear1, linear2, activation):
    if not isinstance(activation, nn.ReLU):
        return False
    return ffn_weights_ok(x, linear1.weight, linear2.weight)


def ffn_weights_ok(x, w1, w2):
    """the fused two-GEMM path for (R, C) bf16 rows and (F, C) / (N, F) weights"""
    if not (fused_ffn and x.is_cuda and x.dtype == torch.bfloat16
            and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16 and x.stride(-1) == 1
            and w1.dim() == 2 and w2.dim() == 2):
        return False
    xr = x.reshape(-1, x.shape[-1])
    bf = torch.bfloat16
    w1c, w2c = gemm.cast_param(w1, bf), gemm.cast_param(w2, bf)
    if not (gemm.act_gemm_ok(xr, w1c, True) and w2c.stride(1) == 1 and w2c.stride(0) % 8 == 0
            and w2c.data_ptr() % 16 == 0 and w2c.shape[1] == w1c.shape[0]):
        return False
    # the launches on the fresh (contiguous) h / dy / dy1 rows: linear2, its input gradient
    # (output F columns over N), linear1's input gradient (C columns over F); the short
    # row-block kernel or the long one, as gemm.act_gemm picks
    M, C, F, N = xr.shape[0], xr.shape[1], w1c.shape[0], w2c.shape[0]
    return gemm.shape_ok(M, N, F) and gemm.shape_ok(M, F, N) and gemm.shape_ok(M, C, F)


def ffn(x, linear1, linear2, activation, dropout, site):
    """linear2(dropout(activation(linear1(x)))) of a transformer layer (bf16 rows)"""
    if _ffn_ok(x, linear1, linear2, activation):
        p = dropout.p if dropout.training else 0.0
        with torch.autocast("cuda", enabled=False):
            return _FFN.apply(x, linear1.weight, linear1.bias, linear2.weight, linear2.bias, p, site)
    h = ffn_act(gemm.rows_linear(x, linear1.weight, linear1.bias), activation, dropout, site)
    return gemm.rows_linear(h, linear2.weight, linear2.bias)


def ffn_weights(x, w1, b1, w2, b2):
    """linear2(relu(linear1(x))) on bf16 rows (the query projection's conv pair, no dropout)"""
    with torch.autocast("cuda", enabled=False):
        return _FFN.apply(x, w1, b1, w2, b2, 0.0, 0)


def relu_rows(y):
    """relu of bf16 rows on the HIP row kernel (one launch each way)"""
    return _ReluDropout.apply(y, 0.0, 0)


def ffn_act(y, activation, dropout, site):
    """dropout(activation(y)) of a transformer FFN: one HIP launch for bf16 ReLU rows."""
    if (isinstance(activation, nn.ReLU) and y.is_cuda and y.dtype == torch.bfloat16
            and y.shape[-1] % 8 == 0):
        p = dropout.p if dropout.training else 0.0
        return _ReluDropout.apply(y, p, site)
    return dropout(activation(y))
