"""FusedAdamW (csrc/adamw.hip) against torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW
(fp32) on the same gradients: parameters, moments, clipped gradients and the returned norm
after several steps, with and without clipping, plus the bf16 weight copies it rewrites
and a captured step graph equal to the eager steps."""
import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


def _params(cuda, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(768, 256), (768,), (256, 256), (3,), (21, 640), (5000,), (1,), (64, 3)]
    return [torch.nn.Parameter(torch.randn(*s, generator=g).to(cuda)) for s in shapes]


def _grads(params, k):
    g = torch.Generator().manual_seed(100 + k)
    return [torch.randn(p.shape, generator=g).to(p.device) * (0.5 + k) for p in params]


@pytest.mark.parametrize("clip", [0.1, None, 1e9])
def test_fused_adamw_matches_torch(cuda, clip):
    from ov3d_amd.optim import FusedAdamW
    pa, pb = _params(cuda), _params(cuda)
    oa = FusedAdamW(pa, lr=7e-4, weight_decay=0.1, max_grad_norm=clip)
    ob = torch.optim.AdamW(pb, lr=7e-4, weight_decay=0.1, foreach=False)
    for k in range(4):
        for ps in (pa, pb):
            for p, g in zip(ps, _grads(ps, k)):
                p.grad = g.clone()
        oa.step()
        norm = torch.nn.utils.clip_grad_norm_(pb, clip) if clip else None
        ob.step()
        if clip:
            assert abs(oa.last_grad_norm.item() - norm.item()) <= 1e-5 * norm.item()
        def close(x, y):
            # fp32 rounding of the same expressions: 1e-5 of the tensor's scale
            return torch.allclose(x, y, rtol=1e-5, atol=1e-6 * y.abs().max().item())

        for a, b in zip(pa, pb):
            assert close(a, b), (k, (a - b).abs().max().item())
            assert close(a.grad, b.grad)
            sa, sb = oa.state[a], ob.state[b]
            assert close(sa["exp_avg"], sb["exp_avg"]), (k, (sa["exp_avg"] - sb["exp_avg"]).abs().max())
            assert close(sa["exp_avg_sq"], sb["exp_avg_sq"])
            assert float(sa["step"]) == float(sb["step"]) == k + 1


def test_fused_adamw_rewrites_bf16_copies(cuda):
    from ov3d_amd import gemm
    from ov3d_amd.optim import FusedAdamW
    lin = torch.nn.Linear(256, 128).to(cuda)
    x = torch.randn(64, 256, device=cuda)
    opt = FusedAdamW(lin.parameters(), lr=1e-2, weight_decay=0.1, max_grad_norm=0.1)
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = gemm.rows_linear(x, lin.weight, lin.bias)
        y.float().square().mean().backward()
        opt.step()
        sh = gemm.shadow_of(lin.weight)
        assert sh is not None and torch.equal(sh, lin.weight.detach().bfloat16())


def test_fused_adamw_graph_replay_equals_eager(cuda):
    from ov3d_amd.optim import FusedAdamW
    pa, pb = _params(cuda, 1), _params(cuda, 1)
    oa = FusedAdamW(pa, lr=1e-3, weight_decay=0.05, max_grad_norm=0.5)
    ob = FusedAdamW(pb, lr=1e-3, weight_decay=0.05, max_grad_norm=0.5)
    src = [torch.zeros_like(p) for p in pa]

    def body(ps, opt):
        opt.zero_grad(set_to_none=True)
        loss = sum((p * s).sum() for p, s in zip(ps, src))
        loss.backward()
        opt.step()

    for s, g in zip(src, _grads(pa, 0)):
        s.copy_(g)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body(pa, oa)            # eager step builds the table
    torch.cuda.current_stream().wait_stream(side)
    body(pb, ob)
    graph = torch.cuda.CUDAGraph()
    oa.zero_grad(set_to_none=True)
    with torch.cuda.graph(graph):
        body(pa, oa)
    for k in range(1, 4):
        for s, g in zip(src, _grads(pa, k)):
            s.copy_(g)
        graph.replay()
        body(pb, ob)
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-8)


def test_multi_copy_ragged(cuda):
    """ov3d_multi_copy (graphs.StepGraph's batch copy): ragged sizes, odd byte counts, mixed
    dtypes, more than one launch's worth of tensors"""
    from ov3d_amd import _native
    g = torch.Generator().manual_seed(0)
    srcs, dsts = [], []
    for i in range(40):
        n = int(torch.randint(1, 70000, (1,), generator=g))
        dt = (torch.float32, torch.int64, torch.uint8, torch.bfloat16)[i % 4]
        s = (torch.rand(n, generator=g) * 100).to(dt).to(cuda)
        srcs.append(s)
        dsts.append(torch.empty_like(s))
    _native.multi_copy(dsts, srcs)
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s)


def test_fused_adamw_graph_follows_lr_schedule(cuda):
    """The reference changes lr every iteration (engine.py:79, warmup then cosine).  A
    captured FusedAdamW step reads each group's lr / weight decay from a device table that
    sync_hyper() rewrites before the replay: replays with a schedule over two parameter
    groups equal torch.optim.AdamW stepping eagerly with the same schedule."""
    from ov3d_amd.optim import FusedAdamW
    pa, pb = _params(cuda, 2), _params(cuda, 2)
    oa = FusedAdamW([{"params": pa[:4]}, {"params": pa[4:], "weight_decay": 0.0}],
                    lr=1e-3, weight_decay=0.1, max_grad_norm=None)
    ob = torch.optim.AdamW([{"params": pb[:4]}, {"params": pb[4:], "weight_decay": 0.0}],
                           lr=1e-3, weight_decay=0.1, foreach=False)
    src = [torch.zeros_like(p) for p in pa]

    def body(ps, opt):
        opt.zero_grad(set_to_none=True)
        sum((p * s).sum() for p, s in zip(ps, src)).backward()
        opt.step()

    def set_lr(opt, lr):
        for i, g in enumerate(opt.param_groups):
            g["lr"] = lr * (1.0 if i == 0 else 0.5)

    schedule = [1e-3, 3e-3, 7e-4, 2e-4, 5e-5]
    for s, g in zip(src, _grads(pa, 0)):
        s.copy_(g)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    set_lr(oa, schedule[0])
    with torch.cuda.stream(side):
        body(pa, oa)            # eager step builds the table
    torch.cuda.current_stream().wait_stream(side)
    set_lr(ob, schedule[0])
    body(pb, ob)
    graph = torch.cuda.CUDAGraph()
    oa.zero_grad(set_to_none=True)
    with torch.cuda.graph(graph):
        body(pa, oa)
    for k, lr in enumerate(schedule[1:], start=1):
        for s, g in zip(src, _grads(pa, k)):
            s.copy_(g)
        set_lr(oa, lr)
        oa.sync_hyper()
        graph.replay()
        set_lr(ob, lr)
        body(pb, ob)
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6 * b.abs().max().item()), \
            (a - b).abs().max().item()
    # the captured table must never be rebuilt: a new parameter set raises
    extra = torch.nn.Parameter(torch.ones(4, device=cuda))
    oa.add_param_group({"params": [extra]})
    extra.grad = torch.ones_like(extra)
    with pytest.raises(RuntimeError):
        oa.step()
