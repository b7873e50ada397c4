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
