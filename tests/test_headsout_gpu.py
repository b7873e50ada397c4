"""csrc/headsout.hip: the five heads' output layers + the query <-> text alignment in one
launch each way (ov3d_heads_out_fwd / _bwd) against fp32 PyTorch on the same bf16 operands:
out = z W^T + b per head, logits = out_visual text^T (model_3detr.py:152-154, 237-238; the
reference's transposed layout of quirk Q8 when lq = Q), and the backward's
bf16(g_v + g_logits text), bf16(g_s) and the box heads' input gradient."""
import ctypes

import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


def _case(cuda, R, T, nb, seed):
    g = torch.Generator(device=cuda).manual_seed(seed)
    H = 256
    z = torch.randn(R, 5 * H, device=cuda, generator=g).to(torch.bfloat16)
    wv = (torch.randn(640, H, device=cuda, generator=g) * 0.06).to(torch.bfloat16)
    bv = torch.randn(640, device=cuda, generator=g) * 0.1
    n = [3, 3, nb, nb]
    ws = [(torch.randn(k, H, device=cuda, generator=g) * 0.06).to(torch.bfloat16) for k in n]
    bs = [torch.randn(k, device=cuda, generator=g) * 0.1 for k in n]
    text = torch.randn(T, 640, device=cuda, generator=g) * 0.05
    return z, wv, bv, ws, bs, n, text


def _arrays(ws, bs, n):
    ocol, o = [], 0
    for k in n:
        ocol.append(o)
        o += k
    keep = dict(ws=(ctypes.c_void_p * 4)(*[w.data_ptr() for w in ws]),
                bs=(ctypes.c_void_p * 4)(*[b.data_ptr() for b in bs]),
                n=(ctypes.c_int * 4)(*n), kcol=(ctypes.c_int * 4)(*[256 * (1 + i) for i in range(4)]),
                ocol=(ctypes.c_int * 4)(*ocol))
    return keep, o, ocol


@pytest.mark.parametrize("R,T,nb,lq", [(8192, 21, 12, 0), (8192, 21, 12, 128), (16384, 19, 12, 256),
                                       (1000, 7, 1, 0), (40, 32, 32, 8)])
def test_heads_out_fwd_bwd_match_fp32(cuda, R, T, nb, lq):
    from ov3d_amd import _native as nat
    z, wv, bv, ws, bs, n, text = _case(cuda, R, T, nb, R + T)
    keep, Ns, ocol = _arrays(ws, bs, n)
    out_v = torch.empty(R, 640, device=cuda)
    out_s = torch.empty(R, Ns, device=cuda)
    logits = torch.empty(R, T, device=cuda)
    work = torch.empty(nat.load().ov3d_heads_out_workspace(R, T), device=cuda)
    nat.call("ov3d_heads_out_fwd", z, 1280, R, wv, bv, 640, text, T, lq, out_v, logits, 4,
             ctypes.addressof(keep["ws"]), ctypes.addressof(keep["bs"]), ctypes.addressof(keep["n"]),
             ctypes.addressof(keep["kcol"]), ctypes.addressof(keep["ocol"]), out_s, Ns, work, like=z)
    zf = z.float()
    ref_v = zf[:, :256] @ wv.float().t() + bv
    ref_s = torch.cat([zf[:, 256 * (1 + i):256 * (2 + i)] @ ws[i].float().t() + bs[i] for i in range(4)], 1)
    ref_l = ref_v @ text.t()
    if lq:
        ref_l = ref_l.reshape(R // lq, lq, T).transpose(1, 2).reshape(R, T)
    torch.testing.assert_close(out_v, ref_v, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out_s, ref_s, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(logits, ref_l, rtol=1e-4, atol=1e-4)
    # backward
    g = torch.Generator(device=cuda).manual_seed(5)
    gv = torch.randn(R, 640, device=cuda, generator=g)
    gl = torch.randn(R, T, device=cuda, generator=g)
    gs = torch.randn(R, Ns, device=cuda, generator=g)
    gvb = torch.empty(R, 640, dtype=torch.bfloat16, device=cuda)
    gsb = torch.empty(R, Ns, dtype=torch.bfloat16, device=cuda)
    dz = torch.full((R, 1280), 7.0, dtype=torch.bfloat16, device=cuda)
    nat.call("ov3d_heads_out_bwd", gv, gl, text, R, 640, T, lq, gs, Ns, 4, ctypes.addressof(keep["ws"]),
             ctypes.addressof(keep["n"]), ctypes.addressof(keep["kcol"]), ctypes.addressof(keep["ocol"]),
             gvb, gsb, dz, 1280, like=z)
    gl_rows = gl if not lq else gl.reshape(R // lq, T, lq).transpose(1, 2).reshape(R, T)
    ref_gv = gv + gl_rows @ text
    torch.testing.assert_close(gvb.float(), ref_gv, rtol=8e-3, atol=1e-3)
    assert torch.equal(gsb, gs.to(torch.bfloat16))
    gsr = gsb.float()
    for i in range(4):
        ref = gsr[:, ocol[i]:ocol[i] + n[i]] @ ws[i].float()
        torch.testing.assert_close(dz[:, 256 * (1 + i):256 * (2 + i)].float(), ref, rtol=8e-3, atol=1e-3)
    assert (dz[:, :256].float() == 7.0).all()      # the visual columns are the caller's


def test_heads_out_rejects_bad_shapes(cuda):
    from ov3d_amd import _native as nat
    z, wv, bv, ws, bs, n, text = _case(cuda, 64, 40, 12, 1)
    keep, Ns, _ = _arrays(ws, bs, n)
    out_v = torch.empty(64, 640, device=cuda)
    with pytest.raises(nat.NativeError):   # T = 40 > 32 text rows
        nat.call("ov3d_heads_out_fwd", z, 1280, 64, wv, bv, 640, text, 40, 0, out_v,
                 torch.empty(64, 40, device=cuda), 4, ctypes.addressof(keep["ws"]),
                 ctypes.addressof(keep["bs"]), ctypes.addressof(keep["n"]),
                 ctypes.addressof(keep["kcol"]), ctypes.addressof(keep["ocol"]),
                 torch.empty(64, Ns, device=cuda), Ns, torch.empty(64 * 40 * 5, device=cuda), like=z)
