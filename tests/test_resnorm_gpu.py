"""Residual + dropout + LayerNorm launches (csrc/resnorm.hip, resnorm.py) against a plain
PyTorch fp32 restatement with the same keep mask (rebuilt from the documented row hash,
csrc/rowdrop.h): outputs and every gradient.  Then the bf16 encoder / decoder with the
fused launches against the same modules on the plain torch code (dropout 0)."""
import numpy as np
import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu
M32 = 0xFFFFFFFF


def _mix32(x):
    x = x & M32
    x = x ^ (x >> 16)
    x = (x * 0x7feb352d) & M32
    x = x ^ (x >> 15)
    x = (x * 0x846ca68b) & M32
    x = x ^ (x >> 16)
    return x


def _umul24(x, c):
    return ((x & 0xFFFFFF) * (c & 0xFFFFFF)) & M32


def _mix24(x):
    x = x & M32
    x = x ^ (x >> 16)
    x = _umul24(x, 0x7feb35) ^ (x >> 24)
    x = x ^ (x >> 15)
    x = _umul24(x, 0x846ca7) ^ (x >> 24)
    x = x ^ (x >> 16)
    return x


def row_keep(seed, site, R, C, p, device):
    """rowdrop.h keep(r, c) in int64 torch arithmetic"""
    s = int(seed)
    lo, hi = s & M32, (s >> 32) & M32
    sm = _mix32(torch.tensor(lo, dtype=torch.int64, device=device)
                ^ _mix32(torch.tensor((hi + site * 0x9E3779B9) & M32, dtype=torch.int64, device=device)))
    r = torch.arange(R, dtype=torch.int64, device=device)
    rb = _mix32(sm ^ ((r * 0xC2B2AE35) & M32))                                   # (R,)
    c = torch.arange(C, dtype=torch.int64, device=device)
    h = _mix24(rb[:, None] + (((c[None] >> 1) * 0x27D4EB2F) & M32))
    half = torch.where((c & 1).bool()[None], h >> 16, h & 0xFFFF)
    th = min(int(np.rint(np.float32(p) * np.float32(65536.0))), 65535) if p > 0 else 0
    return half >= th


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("R,C,p,src_bf16", [(1024, 256, 0.1, False), (16384, 256, 0.0, False),
                                            (3000, 128, 0.3, True), (64, 512, 0.1, False)])
def test_resnorm_matches_torch(cuda, R, C, p, src_bf16):
    from ov3d_amd import attention as flash
    from ov3d_amd import resnorm as rn
    torch.manual_seed(0)
    na = torch.nn.LayerNorm(C).to(cuda)
    nb = torch.nn.LayerNorm(C).to(cuda)
    with torch.no_grad():
        for n in (na, nb):
            n.weight.copy_(1 + 0.1 * torch.randn(C))
            n.bias.copy_(0.1 * torch.randn(C))
    src = torch.randn(R, 1, C, device=cuda)
    if src_bf16:
        src = src.bfloat16()
    src.requires_grad_()
    y = torch.randn(R, 1, C, device=cuda).bfloat16().requires_grad_()
    pos = torch.randn(R, 1, C, device=cuda).requires_grad_()
    site = flash.new_site()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        s, xa, xap, xb = rn.resnorm(rn.Pending(src, y, p, site), na, pos=pos, want_a=True,
                                    want_ap=True, norm_b=nb)
    g = [torch.randn_like(t) for t in (s, xa, xap, xb)]
    torch.autograd.backward((s, xa, xap, xb), g)
    fused = [t.grad.clone() for t in (src, y, pos)] + [na.weight.grad.clone(), na.bias.grad.clone(),
                                                       nb.weight.grad.clone(), nb.bias.grad.clone()]
    for t in (src, y, pos, na.weight, na.bias, nb.weight, nb.bias):
        t.grad = None
    # fp32 restatement with the same mask and torch's bf16 dropout rounding
    keep = row_keep(flash._seed(cuda).item(), site, R, C, p, cuda).view(R, 1, C)
    d = (y.float() * (1 / (1 - p))).bfloat16().float() if p > 0 else y.float()
    s_ref = src.float() + torch.where(keep, d, torch.zeros_like(d)) if p > 0 else src.float() + d
    ln_a = torch.nn.functional.layer_norm(s_ref, (C,), na.weight, na.bias, na.eps)
    xa_ref = ln_a.bfloat16()
    xap_ref = (ln_a + pos).bfloat16()
    xb_ref = torch.nn.functional.layer_norm(s_ref, (C,), nb.weight, nb.bias, nb.eps)
    assert _rel(s, s_ref) < 1e-6
    assert _rel(xa, xa_ref) < 8e-3 and _rel(xap, xap_ref) < 8e-3
    assert _rel(xb, xb_ref) < 1e-5
    torch.autograd.backward((s_ref, xa_ref, xap_ref, xb_ref), g)
    ref = [t.grad for t in (src, y, pos, na.weight, na.bias, nb.weight, nb.bias)]
    names = ("src", "y", "pos", "ga", "ba", "gb", "bb")
    for n, a, b in zip(names, fused, ref):
        tol = 1e-2 if n in ("src", "y") and (src_bf16 or n == "y") else 1e-4
        assert _rel(a, b) < tol, (n, _rel(a, b))


def _layers(cuda, enc_layers=2, dec_layers=3):
    from ov3d_amd.transformer import (TransformerDecoder, TransformerDecoderLayer,
                                      TransformerEncoder, TransformerEncoderLayer)
    torch.manual_seed(1)
    enc = TransformerEncoder(TransformerEncoderLayer(256, 4, 128, dropout=0.0), enc_layers)
    dec = TransformerDecoder(TransformerDecoderLayer(256, 4, 256, dropout=0.0), dec_layers,
                             return_intermediate=True)
    with torch.no_grad():
        for m in list(enc.modules()) + list(dec.modules()):
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.normal_(1, 0.1)
                m.bias.normal_(0, 0.1)
    return enc.to(cuda).train(), dec.to(cuda).train()


def test_encoder_decoder_fused_vs_plain_bf16(cuda):
    """the fused bf16 path is as close to the fp32 modules as the plain bf16 path is"""
    from ov3d_amd import resnorm as rn
    enc, dec = _layers(cuda)
    src = torch.randn(256, 2, 256, device=cuda)
    tgt = torch.zeros(64, 2, 256, device=cuda)
    qpos = torch.randn(64, 2, 256, device=cuda)
    mpos = torch.randn(256, 2, 256, device=cuda)
    g = torch.randn((3, 64, 2, 256), device=cuda, generator=torch.Generator(device=cuda).manual_seed(2))
    res = {}
    for mode in ("fp32", "plain", "fused"):
        rn.enabled = mode == "fused"
        try:
            for prm in list(enc.parameters()) + list(dec.parameters()):
                prm.grad = None
            s = src.clone().requires_grad_()
            q = qpos.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "fp32"):
                _, mem, _ = enc(s)
                out, _ = dec(tgt, mem, query_pos=q, pos=mpos)
            (out.float() * g).sum().backward()
            res[mode] = [out.float().detach(), s.grad.clone(), q.grad.clone()] + \
                [p.grad.clone() for p in list(enc.parameters()) + list(dec.parameters())]
        finally:
            rn.enabled = True
    for i, ref in enumerate(res["fp32"]):
        e_plain = _rel(res["plain"][i], ref)
        e_fused = _rel(res["fused"][i], ref)
        assert e_fused <= 1.5 * e_plain + 5e-3, (i, e_fused, e_plain)
        assert e_fused < 0.1, (i, e_fused)


@pytest.mark.parametrize("pos_bf16", [False, True])
def test_decoder_fan_in_and_strided_grads_bitwise(cuda, pos_bf16):
    """the shared query_pos / decoder-norm gradient buffers (resnorm.FanIn, accumulate
    launches) give autograd's per-call sums bit for bit, and the decoder outputs' gradient
    read in place as a strided (L, B, Q, C) view equals the contiguous one"""
    from ov3d_amd import attention as flash
    from ov3d_amd import resnorm as rn
    from ov3d_amd.transformer import TransformerDecoder, TransformerDecoderLayer
    torch.manual_seed(3)
    dec = TransformerDecoder(TransformerDecoderLayer(256, 4, 256, dropout=0.1), 4,
                             return_intermediate=True)
    with torch.no_grad():
        for m in dec.modules():
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.normal_(1, 0.1)
                m.bias.normal_(0, 0.1)
    dec = dec.to(cuda).train()
    flash.next_step(cuda)
    tgt = torch.zeros(64, 2, 256, device=cuda)
    mem = torch.randn(256, 2, 256, device=cuda)
    qpos = torch.randn(64, 2, 256, device=cuda).to(torch.bfloat16 if pos_bf16 else torch.float32)
    mpos = torch.randn(256, 2, 256, device=cuda)
    g = torch.randn((4, 2, 64, 256), device=cuda)
    res = {}
    for mode in ("autograd", "fan", "fan_strided"):
        rn.fan_in = mode != "autograd"
        try:
            dec.zero_grad(set_to_none=True)
            q = qpos.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out, _ = dec(tgt, mem, query_pos=q, pos=mpos)        # (L, Q, B, C)
            if mode == "fan_strided":   # as model_3detr: (L, B, Q, C) rows of the stack
                (out.permute(0, 2, 1, 3).reshape(-1, 256) * g.reshape(-1, 256)).sum().backward()
            else:
                (out * g.permute(0, 2, 1, 3).contiguous()).sum().backward()
            res[mode] = [out.detach().clone(), q.grad.clone()] + \
                [p.grad.clone() for p in dec.parameters()]
        finally:
            rn.fan_in = True
    for mode in ("fan", "fan_strided"):
        for i, (a, b) in enumerate(zip(res[mode], res["autograd"])):
            assert torch.equal(a, b), (mode, i, (a.float() - b.float()).abs().max().item())


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_relu_dropout_matches_torch(cuda, p):
    from ov3d_amd import attention as flash
    from ov3d_amd import resnorm as rn
    R, C = 4096, 128
    y = torch.randn(R, C, device=cuda).bfloat16().requires_grad_()
    site = flash.new_site()
    drop = torch.nn.Dropout(p).train()
    h = rn.ffn_act(y, torch.nn.ReLU(), drop, site)
    g = torch.randn(R, C, device=cuda).bfloat16()
    h.backward(g)
    keep = row_keep(flash._seed(cuda).item(), site, R, C, p, cuda)
    a = torch.relu(y.detach().float())
    ref = torch.where(keep, (a * (1 / (1 - p))).bfloat16().float(), torch.zeros_like(a)) if p > 0 \
        else a.bfloat16().float()
    assert torch.equal(h.float(), ref)
    gref = torch.where((ref > 0), g.float() * (1 / (1 - p)), torch.zeros_like(a)).bfloat16()
    assert torch.equal(y.grad, gref)


@pytest.mark.parametrize("qpos_kind", ["f32", "bf16", "none"])
def test_lngemm_decoder_equals_unfused_bitwise(cuda, qpos_kind):
    """every decoder norm fused with the linear layer after it (csrc/lngemm.hip,
    resnorm.resnorm_gemm: norm1 -> in-projection, norm2 -> query projection, norm3 -> linear1
    + ReLU + dropout, linear2 into the next launch) against the resnorm + rows-GEMM launches:
    outputs, query_pos and every parameter gradient bit for bit (same arithmetic, same
    order), dropout 0.1"""
    from ov3d_amd import attention as flash
    from ov3d_amd import resnorm as rn
    from ov3d_amd.transformer import TransformerDecoder, TransformerDecoderLayer
    torch.manual_seed(5)
    dec = TransformerDecoder(TransformerDecoderLayer(256, 4, 256, dropout=0.1), 3,
                             return_intermediate=True)
    with torch.no_grad():
        for m in dec.modules():
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.normal_(1, 0.1)
                m.bias.normal_(0, 0.1)
    dec = dec.to(cuda).train()
    flash.next_step(cuda)
    tgt = torch.zeros(128, 2, 256, device=cuda)
    mem = torch.randn(256, 2, 256, device=cuda)
    qpos = None if qpos_kind == "none" else torch.randn(128, 2, 256, device=cuda).to(
        torch.bfloat16 if qpos_kind == "bf16" else torch.float32)
    mpos = torch.randn(256, 2, 256, device=cuda)
    g = torch.randn((3, 2, 128, 256), device=cuda)
    res = {}
    for mode in ("fused", "unfused"):
        rn.lngemm = mode == "fused"
        try:
            dec.zero_grad(set_to_none=True)
            q = qpos.clone().requires_grad_() if qpos is not None else None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                assert dec.layers[0].ln_ok(tgt, q, None, None, (None,)) == (mode == "fused")
                out, _ = dec(tgt, mem, query_pos=q, pos=mpos)        # (L, Q, B, C)
            (out.permute(0, 2, 1, 3).reshape(-1, 256) * g.reshape(-1, 256)).sum().backward()
            res[mode] = [out.detach().clone()] + ([q.grad.clone()] if q is not None else []) + \
                [p.grad.clone() for p in dec.parameters()]
        finally:
            rn.lngemm = True
    names = ["out"] + (["qpos"] if qpos is not None else []) + [n for n, _ in dec.named_parameters()]
    bad = [(n, (a.float() - b.float()).abs().max().item())
           for n, a, b in zip(names, res["fused"], res["unfused"]) if not torch.equal(a, b)]
    assert not bad, bad


def _report(pairs):
    bad = []
    for n, a, b in pairs:
        if a is None and b is None:
            continue
        if not torch.equal(a, b):
            d = (a.float() - b.float()).abs()
            bad.append((n, int((d > 0).sum().item()), d.max().item(), b.float().abs().max().item()))
    return bad


@pytest.mark.parametrize("p,epi", [(0.0, 0), (0.1, 1)])
def test_lngemm_kernels_equal_two_launch_path(cuda, p, epi):
    """ov3d_lngemm_fwd / _bwd against ov3d_resnorm_fwd + ov3d_rows_gemm(_act) and
    ov3d_resnorm_bwd + ov3d_rows_gemm_act on the same operands: every output bit for bit"""
    import ctypes
    from ov3d_amd import _native, gemm
    from ov3d_amd import attention as flash
    torch.manual_seed(7)
    R, C = 1024, 256
    bf = torch.bfloat16
    dev = cuda
    flash.next_step(dev)
    seed = flash._seed(dev)
    src = torch.randn(R, C, device=dev)
    y = torch.randn(R, C, device=dev).to(bf)
    pos = torch.randn(R, C, device=dev)
    ga, ba, gb, bb = (1 + 0.1 * torch.randn(C, device=dev), 0.1 * torch.randn(C, device=dev),
                      1 + 0.1 * torch.randn(C, device=dev), 0.1 * torch.randn(C, device=dev))
    W0 = (0.05 * torch.randn(512, C, device=dev)).to(bf)
    b0 = (0.1 * torch.randn(512, device=dev)).to(bf)
    W1 = (0.05 * torch.randn(256, C, device=dev)).to(bf)
    b1 = (0.1 * torch.randn(256, device=dev)).to(bf)
    site, site2 = 11, 12
    outs = {}
    for mode in ("two", "one"):
        s = torch.empty(R, C, device=dev)
        mean = torch.empty(R, device=dev)
        rstd = torch.empty(R, device=dev)
        xa = torch.empty(R, C, device=dev, dtype=bf)
        xap = torch.empty(R, C, device=dev, dtype=bf)
        xb = torch.empty(R, C, device=dev)
        o0 = torch.empty(R, 512, device=dev, dtype=bf)
        o1 = torch.empty(R, 256, device=dev, dtype=bf)
        if mode == "two":
            _native.call("ov3d_resnorm_fwd", R, C, src, 0, y, 1, float(p), seed, site, ga, ba, pos,
                         0, gb, bb, 1e-5, s, mean, rstd, xa, xap, xb, 0, 0, 0, 0, like=s)
            _native.call("ov3d_rows_gemm_act", R, 512, C, xap, C, W0, C, 1, b0, 0, 0.0, None, 0,
                         None, 0, o0, 512, like=s)
            _native.call("ov3d_rows_gemm_act", R, 256, C, xa, C, W1, C, 1, b1, epi, float(p), seed,
                         site2, None, 0, o1, 256, like=s)
        else:
            probs = [gemm._LnProblem(W0.data_ptr(), C, b0.data_ptr(), o0.data_ptr(), 512, 512, 1),
                     gemm._LnProblem(W1.data_ptr(), C, b1.data_ptr(), o1.data_ptr(), 256, 256, 0)]
            if epi:   # the activation epilogue applies to every problem: one problem a launch
                arr = (gemm._LnProblem * 1)(probs[0])
                _native.call("ov3d_lngemm_fwd", R, src, 0, y, float(p), seed, site, ga, ba, pos, 0,
                             gb, bb, 1e-5, s, mean, rstd, xa, xap, xb, 0, 0, 0, 0, 1,
                             ctypes.addressof(arr), 0, 0.0, None, 0, like=s)
                arr2 = (gemm._LnProblem * 1)(probs[1])
                s2 = torch.empty_like(s)
                _native.call("ov3d_lngemm_fwd", R, src, 0, y, float(p), seed, site, ga, ba, pos, 0,
                             gb, bb, 1e-5, s2, torch.empty_like(mean), torch.empty_like(rstd),
                             None, None, None, 0, 0, 0, 0, 1, ctypes.addressof(arr2), 1, float(p),
                             seed, site2, like=s)
            else:
                arr = (gemm._LnProblem * 2)(*probs)
                _native.call("ov3d_lngemm_fwd", R, src, 0, y, float(p), seed, site, ga, ba, pos, 0,
                             gb, bb, 1e-5, s, mean, rstd, xa, xap, xb, 0, 0, 0, 0, 2,
                             ctypes.addressof(arr), 0, 0.0, None, 0, like=s)
        outs[mode] = dict(s=s, mean=mean, rstd=rstd, xa=xa, xap=xap, xb=xb, o0=o0, o1=o1)
    fwd_bad = _report([(k, outs["one"][k], outs["two"][k]) for k in outs["two"]])
    # backward: dy = dropout(resnorm_bwd(...)); dx = epi(dy W) with W (256, 256) = (out, in)
    s, mean, rstd = outs["two"]["s"], outs["two"]["mean"], outs["two"]["rstd"]
    ds = torch.randn(R, C, device=dev)
    dxa = torch.randn(R, C, device=dev).to(bf)
    dxap = torch.randn(R, C, device=dev).to(bf)
    Wy = (0.05 * torch.randn(C, 256, device=dev)).to(bf)
    H = torch.relu(torch.randn(R, 256, device=dev)).to(bf)
    res = {}
    for mode in ("two", "one"):
        dsrc = torch.empty(R, C, device=dev)
        dy = torch.empty(R, C, device=dev, dtype=bf)
        dpos = torch.empty(R, C, device=dev)
        dx = torch.empty(R, 256, device=dev, dtype=bf)
        if mode == "two":
            nparts = _native.load().ov3d_resnorm_bwd_parts(R, C)
            part = torch.empty(nparts, 4, C, device=dev)
            _native.call("ov3d_resnorm_bwd", R, C, s, mean, rstd, ds, dxa, dxap, None, 0, 0, 0, 0,
                         ga, None, float(p), seed, site, dsrc, dy, 1, dpos, 0, part, nparts,
                         None, None, None, None, 0, like=s)
            _native.call("ov3d_rows_gemm_act", R, 256, C, dy, C, Wy, 256, 0, None,
                         2 if epi else 0, float(p), None, 0, H if epi else None, 256 if epi else 0,
                         dx, 256, like=s)
        else:
            nparts = _native.load().ov3d_lngemm_bwd_parts(R)
            part = torch.empty(nparts, 4, C, device=dev)
            _native.call("ov3d_lngemm_bwd", R, s, mean, rstd, ds, dxa, dxap, None, 0, 0, 0, 0, ga,
                         None, float(p), seed, site, dsrc, dy, dpos, 0, part, 0, Wy, 256, 256,
                         2 if epi else 0, float(p), H if epi else None, 256 if epi else 0, dx, 256,
                         like=s)
        res[mode] = dict(dsrc=dsrc, dy=dy, dpos=dpos, dx=dx, part=part)
    bwd_bad = _report([(k, res["one"][k], res["two"][k]) for k in res["two"]])
    assert not fwd_bad and not bwd_bad, (fwd_bad, bwd_bad)
