"""Short row-block GEMMs (csrc/rowsgemm.hip, gemm.rows_gemm) against the fp32 product of the
same bf16 operands: the error is that of one bf16 rounding of the output, as for the library
GEMM it replaces; ragged row counts, strided row views, both operand layouts."""
import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


def _check(out, ref, lib):
    err = (out.float() - ref).abs().max().item()
    lib_err = (lib.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1.5 * lib_err + 1e-3 * scale, (err, lib_err, scale)


@pytest.mark.parametrize("M,N,K,bias", [(1024, 256, 256, True), (1000, 512, 256, True),
                                        (64, 32, 64, False), (2048, 768, 1024, True),
                                        (33, 96, 192, True)])
def test_rows_gemm_linear(cuda, M, N, K, bias):
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    wide = torch.randn(M, K + 64, device=cuda, generator=g).to(torch.bfloat16)
    a = wide[:, 32:32 + K]                       # strided row view (lda = K + 64)
    w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=cuda, generator=g).to(torch.bfloat16) if bias else None
    assert gemm._rows_gemm_ok(a, w, True)
    out = gemm.rows_gemm(a, w, b, trans_b=True)
    ref = a.float() @ w.float().t() + (b.float() if bias else 0)
    lib = torch.nn.functional.linear(a, w, b)
    assert out.shape == (M, N) and out.dtype == torch.bfloat16
    _check(out, ref, lib)


@pytest.mark.parametrize("M,N,K", [(1024, 256, 256), (1000, 256, 512), (96, 64, 128),
                                   (1024, 512, 1024), (17, 32, 64)])
def test_rows_gemm_input_grad(cuda, M, N, K):
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(7 * M + N + K)
    dy = torch.randn(M, K, device=cuda, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, N, device=cuda, generator=g) / K ** 0.5).to(torch.bfloat16)
    assert gemm._rows_gemm_ok(dy, w, False)
    out = gemm.rows_gemm(dy, w, trans_b=False)
    _check(out, dy.float() @ w.float(), dy @ w)


def test_rows_linear_uses_rows_gemm_and_matches_library(cuda):
    """gemm.rows_linear under bf16 autocast (forward, input and weight gradients) with the
    short-row kernels vs the library GEMMs"""
    from ov3d_amd import _native, gemm
    torch.manual_seed(0)
    lin = torch.nn.Linear(256, 512).to(cuda)
    x0 = torch.randn(8, 128, 256, device=cuda)
    res = {}
    for on in (True, False):
        gemm.ROWS_GEMM = on
        try:
            lin.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_()
            _native.timing_enable(["ov3d_rows_gemm"])
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = gemm.rows_linear(x, lin.weight, lin.bias)
            y.float().square().sum().backward()
            calls = len(_native.timing_collect()["ov3d_rows_gemm"])
            res[on] = (y.float(), x.grad, lin.weight.grad, lin.bias.grad, calls)
        finally:
            gemm.ROWS_GEMM = True
    assert res[True][4] == 2 and res[False][4] == 0     # forward + input gradient
    for a, b in zip(res[True][:4], res[False][:4]):
        assert ((a - b).norm() / b.norm()).item() < 1e-2


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fused_ffn_equals_unfused_bitwise(cuda, p, monkeypatch):
    """resnorm.ffn (ReLU + dropout in the epilogues of linear1 forward and of linear2's input
    gradient, ov3d_rows_gemm_act) gives the unfused linear -> ov3d_relu_dropout -> linear
    chain's output and every gradient bit for bit"""
    from ov3d_amd import attention as flash
    from ov3d_amd import resnorm as rn
    torch.manual_seed(2)
    l1 = torch.nn.Linear(256, 256).to(cuda)
    l2 = torch.nn.Linear(256, 256).to(cuda)
    drop = torch.nn.Dropout(p).train()
    act = torch.nn.ReLU()
    flash.next_step(cuda)
    x0 = torch.randn(1024, 256, device=cuda).to(torch.bfloat16)
    g = torch.randn(1024, 256, device=cuda)
    res = {}
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(rn, "_ffn_ok", lambda *a: False)
        for m in (l1, l2):
            m.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = rn.ffn(x, l1, l2, act, drop, site=77)
        (y.float() * g).sum().backward()
        res[fused] = [y, x.grad, l1.weight.grad, l1.bias.grad, l2.weight.grad, l2.bias.grad]
    for i, (a, b) in enumerate(zip(res[True], res[False])):
        assert torch.equal(a, b), (i, (a.float() - b.float()).abs().max().item())


@pytest.mark.parametrize("trans_b", [True, False])
def test_rows_gemm_group_equals_single_launches(cuda, trans_b):
    """ov3d_rows_gemm_group (problems of different N / K over the same rows: an attention's
    in-projection blocks) equals one ov3d_rows_gemm per problem, bit for bit"""
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(11)
    M = 1024
    shapes = [(512, 256), (256, 256), (256, 512)]   # (N, K)
    probs = []
    for N, K in shapes:
        a = torch.randn(M, K, device=cuda, generator=g).to(torch.bfloat16)
        w = (torch.randn(*((N, K) if trans_b else (K, N)), device=cuda, generator=g) / K ** 0.5
             ).to(torch.bfloat16)
        b = torch.randn(N, device=cuda, generator=g).to(torch.bfloat16) if trans_b else None
        probs.append((a, w, b))
    assert gemm._group_ok([(a, w) for a, w, _ in probs], trans_b)
    outs = gemm.rows_gemm_group(probs, trans_b=trans_b)
    for (a, w, b), o in zip(probs, outs):
        assert torch.equal(o, gemm.rows_gemm(a, w, b, trans_b=trans_b))
