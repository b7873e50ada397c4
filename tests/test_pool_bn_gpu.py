"""The masked encoder's interim SA tail (models/model_3detr.py:377-399: the last SharedMLP layer's
BatchNorm + ReLU, then F.max_pool2d over nsample, third_party pointnet2_modules
PointnetSAModuleVotes) fused into the pool: heads.bn_relu_pool_rows (csrc/pool.hip
ov3d_nbr_max_bnrelu_fwd, csrc/bnrows.hip ov3d_rows_bn_bwd_pooled) against heads.bn_relu_rows +
pointnet2_modules._NbrMax on the same rows: pooled values, arg rows' gradients, BN parameter
gradients and running statistics bit for bit, with ties (repeated rows) and dead channels."""
import copy

import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("P,S,C", [(8192, 32, 256), (300, 16, 128), (64, 5, 8)])
def test_bn_relu_pool_equals_two_passes(P, S, C):
    from ov3d_amd import heads
    from ov3d_amd.pointnet2_modules import _NbrMax
    torch.manual_seed(9)
    dev = torch.device("cuda", 0)
    h = torch.randn(P * S, C, device=dev)
    h[: S * 4] = h[:4].repeat_interleave(S, 0)        # all S rows equal: ties everywhere
    h = h.to(torch.bfloat16)
    bn1 = torch.nn.BatchNorm2d(C).to(dev).train()
    with torch.no_grad():
        bn1.weight.normal_(1, 0.2)
        bn1.weight[:2] = -0.5                           # negative scale: the min row wins
        bn1.bias.normal_(0, 0.2)
        bn1.bias[2:4] = -50.0                           # dead channels: every z is 0
    bn2 = copy.deepcopy(bn1)
    g = torch.randn(P, C, device=dev).to(torch.bfloat16)
    res = []
    for fused, bn in ((True, bn1), (False, bn2)):
        x = h.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert heads.bn_relu_pool_ok(x, bn, torch.nn.ReLU(), S)
            out = heads.bn_relu_pool_rows(x, bn, S) if fused else \
                _NbrMax.apply(heads.bn_relu_rows(x, bn), S)
        out.backward(g)
        res.append([out.detach(), x.grad, bn.weight.grad, bn.bias.grad, bn.running_mean.clone(),
                    bn.running_var.clone(), bn.num_batches_tracked.clone()])
    names = ["out", "dh", "dgamma", "dbeta", "running_mean", "running_var", "nbt"]
    bad = [(n, (a.float() - b.float()).abs().max().item()) for n, a, b in zip(names, *res)
           if not torch.equal(a, b)]
    assert not bad, bad


@pytest.mark.parametrize("defer", [False, True])
def test_bn_relu_into_rows256_equals_two_passes(monkeypatch, defer):
    """heads.bn_relu_linear_rows (csrc/rows256.hip ov3d_rows256_bn: the previous layer's BN +
    ReLU applied while the next 256 x 256 product stages its rows; its weight gradient
    ov3d_wgrad_bn applies the same BN + ReLU as it loads the pre-BN rows) against
    heads.bn_relu_rows + gemm.rows_linear: output, input / gamma / beta / weight gradients and
    running statistics bit for bit (2^17 + 64 rows: a ragged last tile), the weight gradient
    immediate or deferred to the end of the backward (gemm.DEFER_WGRAD)"""
    from ov3d_amd import gemm, heads
    monkeypatch.setattr(gemm, "DEFER_WGRAD", defer)
    torch.manual_seed(12)
    dev = torch.device("cuda", 0)
    R, C = (1 << 17) + 64, 256
    h = torch.randn(R, C, device=dev).to(torch.bfloat16)
    bn1 = torch.nn.BatchNorm2d(C).to(dev).train()
    with torch.no_grad():
        bn1.weight.normal_(1, 0.2)
        bn1.bias.normal_(0, 0.2)
        bn1.bias[:3] = -50.0                                 # dead channels
    bn2 = copy.deepcopy(bn1)
    conv1 = torch.nn.Conv2d(C, C, 1, bias=False).to(dev)
    conv2 = copy.deepcopy(conv1)
    g = torch.randn(R, C, device=dev).to(torch.bfloat16)
    res = []
    for fused, bn, conv in ((True, bn1, conv1), (False, bn2, conv2)):
        x = h.clone().requires_grad_()
        w2 = conv.weight.view(C, C)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if fused:
                assert heads.bn_relu_linear_ok(x, bn, torch.nn.ReLU(), conv.weight, None)
                y = heads.bn_relu_linear_rows(x, bn, w2)
            else:
                y = gemm.rows_linear(heads.bn_relu_rows(x, bn), w2)
        y.backward(g)
        res.append([y.detach(), x.grad, bn.weight.grad, bn.bias.grad, conv.weight.grad,
                    bn.running_mean.clone(), bn.running_var.clone()])
    names = ["y", "dh", "dgamma", "dbeta", "dW", "running_mean", "running_var"]
    bad = [(n, (a.float() - b.float()).abs().max().item()) for n, a, b in zip(names, *res)
           if not torch.equal(a, b)]
    assert not bad, bad
