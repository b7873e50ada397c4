"""Long row-block GEMMs (csrc/tilegemm.hip, gemm.tile_gemm: the encoder's linear layers,
M = batch * 2048) against the fp32 product of the same bf16 operands: the error is that of one
bf16 rounding of the output, as for the library GEMM it replaces; ragged row counts, strided
row views, both operand layouts, and the rows_linear dispatch."""
import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _tile_on(monkeypatch):
    """the kernel is opt-in in the step (gemm.TILE_GEMM); these tests exercise it directly"""
    from ov3d_amd import gemm
    monkeypatch.setattr(gemm, "TILE_GEMM", True)


def _check(out, ref, lib):
    err = (out.float() - ref).abs().max().item()
    lib_err = (lib.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1.5 * lib_err + 1e-3 * scale, (err, lib_err, scale)


@pytest.mark.parametrize("M,N,K,bias", [(16384, 768, 256, True), (16384, 256, 256, True),
                                        (16384, 128, 256, True), (16384, 256, 128, False),
                                        (4099, 384, 512, True), (2049, 128, 64, True)])
def test_tile_gemm_linear(cuda, M, N, K, bias):
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    wide = torch.randn(M, K + 64, device=cuda, generator=g).to(torch.bfloat16)
    a = wide[:, 32:32 + K]                       # strided row view (lda = K + 64)
    w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=cuda, generator=g).to(torch.bfloat16) if bias else None
    assert gemm._tile_gemm_ok(a, w, True)
    out = gemm.tile_gemm(a, w, b, trans_b=True)
    ref = a.float() @ w.float().t() + (b.float() if bias else 0)
    lib = torch.nn.functional.linear(a, w, b)
    assert out.shape == (M, N) and out.dtype == torch.bfloat16
    _check(out, ref, lib)


@pytest.mark.parametrize("M,N,K", [(16384, 256, 768), (16384, 256, 256), (16384, 128, 256),
                                   (16384, 256, 128), (3001, 512, 192)])
def test_tile_gemm_input_grad(cuda, M, N, K):
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(7 * M + N + K)
    dy = torch.randn(M, K, device=cuda, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, N, device=cuda, generator=g) / K ** 0.5).to(torch.bfloat16)
    assert gemm._tile_gemm_ok(dy, w, False)
    out = gemm.tile_gemm(dy, w, trans_b=False)
    _check(out, dy.float() @ w.float(), dy @ w)


def test_rows_linear_uses_tile_gemm_and_matches_library(cuda, monkeypatch):
    """gemm.rows_linear under bf16 autocast over encoder-sized row blocks (forward, input and
    weight gradients) with the tile kernel vs the library GEMMs"""
    from ov3d_amd import _native, gemm
    torch.manual_seed(0)
    lin = torch.nn.Linear(256, 768).to(cuda)
    x0 = torch.randn(2048, 8, 256, device=cuda)
    res = {}
    for on in (True, False):
        monkeypatch.setattr(gemm, "TILE_GEMM", on)
        lin.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        _native.timing_enable(["ov3d_tile_gemm"])
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = gemm.rows_linear(x, lin.weight, lin.bias)
        y.float().square().sum().backward()
        calls = len(_native.timing_collect()["ov3d_tile_gemm"])
        res[on] = (y.float(), x.grad, lin.weight.grad, lin.bias.grad, calls)
    assert res[True][4] == 2 and res[False][4] == 0     # forward + input gradient
    for a, b in zip(res[True][:4], res[False][:4]):
        assert ((a - b).norm() / b.norm()).item() < 1e-2


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_tile_gemm_ffn_epilogues_match_row_kernels(cuda, p):
    """the FFN epilogues (dropout(relu(.)) forward, the masked input gradient backward) equal the
    plain GEMM followed by the resnorm.hip row kernels bit for bit (same keep hash)"""
    from ov3d_amd import _native, gemm
    from ov3d_amd import attention as flash
    M, C, F = 16384, 256, 128
    g = torch.Generator(device=cuda).manual_seed(5)
    x = torch.randn(M, C, device=cuda, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(F, C, device=cuda, generator=g) / C ** 0.5).to(torch.bfloat16)
    b1 = torch.randn(F, device=cuda, generator=g).to(torch.bfloat16)
    seed = flash._seed(cuda) if p > 0 else None
    site = 1234
    assert gemm.act_gemm_ok(x, w1, True) and not gemm._rows_gemm_ok(x, w1, True)
    h = gemm.act_gemm(x, w1, b1, True, 1, p, seed, site)
    y = gemm.tile_gemm(x, w1, b1, trans_b=True)
    h_ref = torch.empty_like(y)
    _native.call("ov3d_relu_dropout_fwd", y, M, F, float(p), seed, site, h_ref, like=y)
    assert torch.equal(h, h_ref)
    if p > 0:
        frac = (h == 0).float().mean().item()
        assert 0.5 < frac < 0.65   # relu zeros about half, dropout 10 % of the rest
    # backward: dy (M, C) through linear2 (C, F) -> masked (M, F)
    w2 = (torch.randn(C, F, device=cuda, generator=g) / F ** 0.5).to(torch.bfloat16)
    dy = torch.randn(M, C, device=cuda, generator=g).to(torch.bfloat16)
    d1 = gemm.act_gemm(dy, w2, None, False, 2, p, h=h)
    raw = gemm.tile_gemm(dy, w2, trans_b=False)
    d1_ref = torch.empty_like(raw)
    _native.call("ov3d_relu_dropout_bwd", h, raw, h.numel(), float(p), d1_ref, like=h)
    assert torch.equal(d1, d1_ref)


def test_tile_gemm2_sums_two_products(cuda):
    """dK Wk + dV Wv in one launch (the decoder memory gradient) vs the fp32 sum"""
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(9)
    M, N, K = 16384, 256, 2048
    a1, a2 = (torch.randn(M, K, device=cuda, generator=g).to(torch.bfloat16) for _ in range(2))
    w1, w2 = ((torch.randn(K, N, device=cuda, generator=g) / K ** 0.5).to(torch.bfloat16)
              for _ in range(2))
    out = gemm.tile_gemm2(a1, w1, a2, w2)
    ref = a1.float() @ w1.float() + a2.float() @ w2.float()
    lib = (a1 @ w1).addmm_(a2, w2)
    _check(out, ref, lib)


@pytest.mark.parametrize("trans_b", [True, False])
def test_tile_bmm_heads_shapes(cuda, trans_b):
    """the heads' per-head second layer (5 x (8192 x 256) x (256 x 256)) and its input gradient
    as one batched launch vs the fp32 products"""
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(11)
    a = torch.randn(5, 8192, 256, device=cuda, generator=g).to(torch.bfloat16)
    w = (torch.randn(5, 256, 256, device=cuda, generator=g) / 16).to(torch.bfloat16)
    assert gemm.tile_bmm_ok(a, w, trans_b)
    out = gemm.tile_bmm(a, w, trans_b)
    wt = w.transpose(1, 2) if trans_b else w
    _check(out, torch.bmm(a.float(), wt.float()), torch.bmm(a, wt))


def test_tile_gemm_into_strided_output(cuda):
    """the visual head's input gradient written into the first 256 columns of 1280-wide rows"""
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(12)
    a = torch.randn(8192, 640, device=cuda, generator=g).to(torch.bfloat16)
    w = (torch.randn(640, 256, device=cuda, generator=g) / 25).to(torch.bfloat16)
    big = torch.full((8192, 1280), 7.0, device=cuda, dtype=torch.bfloat16)
    assert gemm._tile_gemm_ok(a, w, False) and gemm.tile_out_ok(big[:, :256])
    gemm.tile_gemm(a, w, trans_b=False, out=big[:, :256])
    _check(big[:, :256], a.float() @ w.float(), a @ w)
    assert bool((big[:, 256:] == 7.0).all())
