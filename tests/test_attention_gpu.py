"""Flash attention kernels (csrc/attn.hip) against a plain PyTorch fp32 reference of the
same op on the same bf16 inputs: softmax(q k^T / 8) [dropout] v per head, forward and
all three gradients.  Tolerances: bf16 rounding of P / dS inside the kernel (relative
Frobenius error <= 1e-2).  With dropout the reference rebuilds the kernel's keep mask
from the documented hash, so the comparison is exact in the mask."""
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


def _drop_mix(x):
    """attn.hip drop_mix: two 24-bit multiply rounds with 16-bit folds"""
    x = x & M32
    x = x ^ (x >> 16)
    x = _umul24(x, 0x7feb35) ^ (x >> 24)
    x = x ^ (x >> 16)
    x = _umul24(x, 0x846ca7)
    return x ^ (x >> 16)


def keep_mask(seed, site, B, H, Lq, Lk, p, device):
    """attn.hip drop_head_mix / drop_query_base / drop_mix of the pair, 16-bit half per key, in
    int64 torch arithmetic."""
    s = int(seed)
    lo, hi = s & M32, (s >> 32) & M32
    bh = torch.arange(B * H, dtype=torch.int64, device=device)
    inner = _mix32(torch.tensor(hi + site * 0x9E3779B9, dtype=torch.int64, device=device))
    hm = _mix32(lo ^ inner ^ ((bh * 0x85EBCA6B) & M32))                       # (BH,)
    q = torch.arange(Lq, dtype=torch.int64, device=device)
    qb = _mix32(hm[:, None] ^ ((q[None] * 0xC2B2AE35) & M32))                  # (BH, Lq)
    k = torch.arange(Lk, dtype=torch.int64, device=device)
    hsh = _drop_mix(qb[:, :, None] + (((k[None, None] >> 1) * 0x27D4EB2F) & M32))   # (BH, Lq, Lk)
    half = torch.where((k & 1).bool()[None, None], hsh >> 16, hsh & 0xFFFF)
    thresh = min(int(np.rint(np.float32(p) * np.float32(65536.0))), 65535) if p > 0 else 0
    return ((half ^ 0x8000) >= thresh).view(B, H, Lq, Lk)     # int16(half) >= thresh - 32768


def reference(q, k, v, H, p=0.0, mask=None):
    """q (Lq,B,E), k/v (Lk,B,E) fp32 -> (Lq,B,E)"""
    Lq, B, E = q.shape
    Lk = k.shape[0]
    d = E // H
    qh = q.reshape(Lq, B, H, d).permute(1, 2, 0, 3)
    kh = k.reshape(Lk, B, H, d).permute(1, 2, 0, 3)
    vh = v.reshape(Lk, B, H, d).permute(1, 2, 0, 3)
    pr = torch.softmax(qh @ kh.transpose(-1, -2) / d ** 0.5, dim=-1)
    if mask is not None:
        pr = pr * mask / (1 - p)
    return (pr @ vh).permute(2, 0, 1, 3).reshape(Lq, B, E)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("Lq,Lk,B,H,packed", [(2048, 2048, 2, 4, "qkv"), (128, 2048, 8, 4, "cross"),
                                              (128, 128, 8, 4, "qk"), (96, 200, 3, 2, "cross"),
                                              (64, 64, 1, 1, "qkv")])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_matches_reference(cuda, Lq, Lk, B, H, packed, p):
    from ov3d_amd import attention as A
    torch.manual_seed(Lq + Lk + B)
    E = H * 64
    if packed == "qkv" and Lq == Lk:
        base = (torch.randn(Lq, B, 3 * E, device=cuda) * 1.5).to(torch.bfloat16).requires_grad_()
        q, k, v = base.chunk(3, dim=-1)
        leaves = [base]
    elif packed == "qk" and Lq == Lk:
        qk = (torch.randn(Lq, B, 2 * E, device=cuda) * 1.5).to(torch.bfloat16).requires_grad_()
        v0 = torch.randn(Lk, B, E, device=cuda).to(torch.bfloat16).requires_grad_()
        q, k = qk.chunk(2, dim=-1)
        v = v0
        leaves = [qk, v0]
    else:
        q0 = (torch.randn(Lq, B, E, device=cuda) * 1.5).to(torch.bfloat16).requires_grad_()
        k0 = (torch.randn(Lk, B, E, device=cuda) * 1.5).to(torch.bfloat16).requires_grad_()
        v0 = torch.randn(Lk, B, E, device=cuda).to(torch.bfloat16).requires_grad_()
        q, k, v = q0, k0, v0
        leaves = [q0, k0, v0]
    site = 7
    seed = int(A._seed(q.device).item())
    out = A.attention(q, k, v, H, dropout_p=p, site=site)
    g = torch.randn_like(out.float())
    out.float().backward(g)
    got_grads = [t.grad.float().clone() for t in leaves]

    mask = keep_mask(seed, site, B, H, Lq, Lk, p, cuda) if p > 0 else None
    if mask is not None:
        keep = mask.float().mean().item()
        assert abs(keep - (1 - p)) < 5 * (p * (1 - p) / mask.numel()) ** 0.5 + 1e-3, keep
    leaves_r = [t.detach().float().requires_grad_() for t in leaves]
    if packed == "qkv" and Lq == Lk:
        qr, kr, vr = leaves_r[0].chunk(3, dim=-1)
    elif packed == "qk" and Lq == Lk:
        qr, kr = leaves_r[0].chunk(2, dim=-1)
        vr = leaves_r[1]
    else:
        qr, kr, vr = leaves_r
    ref = reference(qr, kr, vr, H, p, mask)
    ref.backward(g)
    assert _rel(out, ref) < 1e-2, _rel(out, ref)
    for gg, lr in zip(got_grads, leaves_r):
        assert _rel(gg, lr.grad) < 2e-2, _rel(gg, lr.grad)


def _drop_key(b, h):
    """attn.hip drop_key: key offset in its 64-key tile of bit b of a (query, h) word"""
    e, j = b >> 4, b & 15
    t, m = j >> 3, j & 7
    return 32 * t + 2 * (m & 1) + 8 * (m >> 1) + 4 * h + e


@pytest.mark.parametrize("Lq,Lk,B,H,nsplit", [(128, 200, 2, 2, 1), (256, 256, 1, 3, 1),
                                              (128, 2048, 2, 2, 8), (96, 64, 2, 1, 1),
                                              (1024, 1024, 1, 2, 1), (1024, 800, 1, 1, 1)])
def test_attention_drop_bits_layouts(cuda, Lq, Lk, B, H, nsplit):
    """The forward's stored drop bits, both layouts, decoded bit by bit against the hash."""
    from ov3d_amd import _native, attention as A
    lib = _native.load()
    torch.manual_seed(1)
    E = H * 64
    q = torch.randn(Lq, B, E, device=cuda).to(torch.bfloat16)
    k = torch.randn(Lk, B, E, device=cuda).to(torch.bfloat16)
    v = torch.randn(Lk, B, E, device=cuda).to(torch.bfloat16)
    p, site = 0.3, 11
    seed_t = A._seed(cuda)
    o = torch.empty(Lq, B, E, device=cuda, dtype=torch.bfloat16)
    lse = torch.empty(B * H, Lq, device=cuda)
    nw = lib.ov3d_attn_dropbits_words(B, H, Lq, Lk)
    nkt = (Lk + 63) // 64
    assert nw == 4 * nkt * B * H * Lq
    bits = torch.zeros(nw, dtype=torch.int32, device=cuda)
    ws = torch.empty(max(lib.ov3d_attn_fwd_workspace(B, H, Lq, Lk, nsplit), 1), device=cuda)
    rc = lib.ov3d_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), E, E, E, B, H, Lq, Lk, 0.125, p,
                           seed_t.data_ptr(), site, o.data_ptr(), E, lse.data_ptr(), bits.data_ptr(),
                           ws.data_ptr(), nsplit, _native._stream(q))
    assert rc == 0
    torch.cuda.synchronize()
    keep = keep_mask(int(seed_t.item()), site, B, H, Lq, Lk, p, cuda).view(B * H, Lq, Lk)
    w = bits.to(torch.int64) & M32
    half = 2 * nkt * B * H * Lq
    wq = w[:half].view(nkt, B * H, Lq, 2)
    wk = w[half:].view(Lq // 32, B * H, nkt * 64)
    bidx = torch.arange(32, device=cuda)
    # query-major: word (kt, bh, q, h) bit b -> key 64 kt + drop_key(b, h)
    drop_q = ((wq[..., None] >> bidx) & 1).bool()                        # (nkt, BH, Lq, 2, 32)
    keys = torch.tensor([[_drop_key(b, h) for b in range(32)] for h in range(2)], device=cuda)
    kabs = 64 * torch.arange(nkt, device=cuda)[:, None, None] + keys[None]   # (nkt, 2, 32)
    got = torch.zeros(B * H, Lq, nkt * 64, dtype=torch.bool, device=cuda)
    for kt in range(nkt):
        for h in range(2):
            got[:, :, kabs[kt, h]] = drop_q[kt, :, :, h, :]
    assert torch.equal(got[:, :, :Lk], ~keep)
    # key-major: word (qblk, bh, key) bit n -> query 32 qblk + n
    drop_k = ((wk[..., None] >> bidx) & 1).bool()                        # (Lq/32, BH, nkt*64, 32)
    got_k = drop_k.permute(1, 0, 3, 2).reshape(B * H, Lq, nkt * 64)
    assert torch.equal(got_k[:, :, :Lk], ~keep)


def test_attention_seed_advances_and_is_reproducible(cuda):
    from ov3d_amd import attention as A
    torch.manual_seed(0)
    x = torch.randn(128, 2, 3 * 128, device=cuda).to(torch.bfloat16)
    q, k, v = x.chunk(3, dim=-1)
    a1 = A.attention(q, k, v, 2, dropout_p=0.1, site=3)
    a2 = A.attention(q, k, v, 2, dropout_p=0.1, site=3)
    assert torch.equal(a1, a2)                    # same step, same site: same mask
    a3 = A.attention(q, k, v, 2, dropout_p=0.1, site=4)
    A.next_step(cuda)
    a4 = A.attention(q, k, v, 2, dropout_p=0.1, site=3)
    assert not torch.equal(a1, a3) and not torch.equal(a1, a4)


def test_dropout_hash_statistics(cuda):
    """The keep mask behaves like i.i.d. Bernoulli(1 - p): overall rate within 5 sigma and
    no correlation between neighbouring keys (same hash word), queries or heads."""
    p = 0.1
    m = keep_mask(123456789, 5, 2, 4, 512, 1024, p, cuda).float()     # 4.2M draws
    n = m.numel()
    assert abs(m.mean().item() - (1 - p)) < 5 * (p * (1 - p) / n) ** 0.5
    z = (m - m.mean()) / m.std()
    for a, b in [(z[..., 0::2], z[..., 1::2]), (z[..., :-1, :], z[..., 1:, :]),
                 (z[:, :-1], z[:, 1:]), (z[:-1], z[1:])]:
        corr = (a * b).mean().item()
        assert abs(corr) < 5e-3, corr


@pytest.mark.parametrize("E,H", [(128, 4), (256, 2)])
def test_module_head_dim_not_64_uses_sdpa(cuda, E, H):
    """head_dim != 64 (e.g. dec_dim 128 / 4 heads) is not a flash-kernel shape: the module
    must route it to scaled-dot-product attention, for self (q is k) and cross attention."""
    from ov3d_amd.transformer import MultiheadAttention
    torch.manual_seed(0)
    m = MultiheadAttention(E, H).to(cuda).eval()
    x = torch.randn(64, 2, E, device=cuda)
    mem = torch.randn(256, 2, E, device=cuda)
    x2 = x + 1
    for q, k, v in ((x, x, x), (x, x, x2), (x, mem, mem)):
        with torch.no_grad():
            ref = m(q, k, v).float()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(q, k, v).float()
        assert _rel(out, ref) < 2e-2


def test_deferred_cross_attention_kv_grads_equal_immediate(cuda):
    """The decoder's 8 cross attentions queue their dK / dV and _MemoryKV's backward runs
    them in one ov3d_attn_bwd_dkdv_batch launch: every parameter gradient of a bf16
    training step is bit-identical to the per-layer launches (same kernel body, disjoint
    column blocks)."""
    import ov3d_amd
    from bench import default_args
    from ov3d_amd import attention as A, synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    args = default_args(enc_dropout=0.0, dec_dropout=0.0, mlp_dropout=0.0)
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).train()
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(2, seed=3, num_points=20000, device=cuda)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    grads = {}
    calls = {}
    orig = A.flush_kv_grads
    for defer in (False, True):
        A.DEFER_KV = defer
        n = [0]

        def counting(buf, n=n):
            n[0] += len(A._KV_JOBS.get(id(buf), []))
            orig(buf)

        A.flush_kv_grads = counting
        try:
            model.zero_grad(set_to_none=True)
            torch.manual_seed(5)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(inputs)
            loss, _ = crit(out, dict(batch))
            loss.backward()
            torch.cuda.synchronize()
            grads[defer] = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
            calls[defer] = n[0]
        finally:
            A.DEFER_KV = True
            A.flush_kv_grads = orig
    assert calls[False] == 0 and calls[True] == 8, calls
    assert set(grads[True]) == set(grads[False])
    for k in grads[False]:
        assert torch.equal(grads[True][k], grads[False][k]), k


def _ref_masked(q, k, v, H, am, p=0.0, keep=None):
    """fp32 reference with a (B, Lq, Lk) bool mask (True = not attended, shared by the heads,
    models/transformer.py:183-190) and an optional keep mask"""
    Lq, B, E = q.shape
    Lk = k.shape[0]
    d = E // H
    qh = q.reshape(Lq, B, H, d).permute(1, 2, 0, 3)
    kh = k.reshape(Lk, B, H, d).permute(1, 2, 0, 3)
    vh = v.reshape(Lk, B, H, d).permute(1, 2, 0, 3)
    sc = (qh @ kh.transpose(-1, -2) / d ** 0.5).masked_fill(am[:, None], float("-inf"))
    pr = torch.softmax(sc, dim=-1)
    if keep is not None:
        pr = pr * keep / (1 - p)
    return (pr @ vh).permute(2, 0, 1, 3).reshape(Lq, B, E)


def _radius_mask(B, L, r2, cuda, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    xyz = (torch.rand(B, L, 3, generator=g) * torch.tensor([4.0, 4.0, 2.0])).to(cuda)
    dist = torch.cdist(xyz, xyz, p=2)
    return dist, r2


@pytest.mark.parametrize("Lq,Lk,B,H,kind", [(2048, 2048, 2, 4, "radius"), (1024, 1024, 2, 4, "radius"),
                                            (128, 2048, 2, 4, "random"), (96, 200, 3, 2, "random")])
@pytest.mark.parametrize("p", [0.0, 0.3])
def test_masked_attention_matches_reference(cuda, Lq, Lk, B, H, kind, p):
    """HIP masked attention (PackedMask) vs fp32 softmax with the boolean mask; radius masks
    packed from the distances (kind 1), random masks from a bool tensor (kind 0)."""
    from ov3d_amd import attention as A
    torch.manual_seed(Lq + Lk)
    E = H * 64
    if kind == "radius":
        dist, r2 = _radius_mask(B, Lq, 0.64, cuda)
        am = dist >= r2
        pm = A.pack_mask(dist, r2)
    else:
        am = torch.rand(B, Lq, Lk, device=cuda) < 0.7
        am[:, :, 0] = False   # every query attends to something
        pm = A.pack_mask(am)
    assert 0.05 < am.float().mean().item() < 0.995
    q0 = (torch.randn(Lq, B, E, device=cuda) * 1.5).to(torch.bfloat16).requires_grad_()
    k0 = (torch.randn(Lk, B, E, device=cuda) * 1.5).to(torch.bfloat16).requires_grad_()
    v0 = torch.randn(Lk, B, E, device=cuda).to(torch.bfloat16).requires_grad_()
    site = 11
    seed = int(A._seed(q0.device).item())
    out = A.attention(q0, k0, v0, H, dropout_p=p, site=site, mask=pm)
    g = torch.randn_like(out.float())
    out.float().backward(g)
    keep = keep_mask(seed, site, B, H, Lq, Lk, p, cuda) if p > 0 else None
    lr = [t.detach().float().requires_grad_() for t in (q0, k0, v0)]
    ref = _ref_masked(*lr, H, am, p, keep)
    ref.backward(g)
    assert _rel(out, ref) < 1e-2, _rel(out, ref)
    for t, r in zip((q0, k0, v0), lr):
        assert _rel(t.grad, r.grad) < 2e-2, _rel(t.grad, r.grad)


def test_mask_pack_layouts(cuda):
    """ov3d_attn_mask_pack: both word layouts decode to the mask bit for bit, and the
    distance form (kind 1) equals the bool form of dist >= thr (kind 0)"""
    from ov3d_amd import attention as A
    B, Lq, Lk = 2, 96, 200
    am = torch.rand(B, Lq, Lk, device=cuda) < 0.4
    w = A.pack_mask(am).words.cpu().numpy().view(np.uint32)
    nkt = (Lk + 63) // 64
    W = nkt * B * Lq * 2
    wq = w[:W].reshape(nkt, B, Lq, 2)
    wk = w[W:].reshape(Lq // 32, B, nkt * 64)
    m = am.cpu().numpy()
    dec_q = np.zeros((B, Lq, nkt * 64), bool)
    for n in range(32):
        for h in range(2):
            kk = np.arange(nkt) * 64 + _drop_key(n, h)
            dec_q[:, :, kk] = ((wq[:, :, :, h] >> n) & 1).transpose(1, 2, 0).astype(bool)
    assert np.array_equal(dec_q[:, :, :Lk], m) and not dec_q[:, :, Lk:].any()
    dec_k = np.zeros((B, Lq, nkt * 64), bool)
    for n in range(32):
        dec_k[:, n::32, :] = ((wk >> n) & 1).transpose(1, 0, 2).astype(bool)
    assert np.array_equal(dec_k[:, :, :Lk], m) and not dec_k[:, :, Lk:].any()
    dist = torch.rand(B, Lq, Lk, device=cuda) * 2
    thr = 0.64
    a = A.pack_mask(dist, thr).words
    b = A.pack_mask(dist >= thr).words
    assert torch.equal(a, b)


@pytest.mark.parametrize("B,L", [(8, 2048), (3, 1000)])
def test_squared_distance_mask_equals_cdist_mask(cuda, B, L):
    """The masked encoder's packing from cdist's matmul-form squared distances (clamp + sqrt
    fused, transformer.euclid_sq) gives the bits of packing torch.cdist's output, under the
    step's bf16 autocast as well; the squared form is cdist's own matrix before its sqrt"""
    from ov3d_amd import attention as A
    from ov3d_amd import transformer as T
    g = torch.Generator(device=cuda).manual_seed(3)
    xyz = torch.rand(B, L, 3, device=cuda, generator=g) * torch.tensor([6.0, 6.0, 3.0], device=cuda)
    xyz[:, 7] = xyz[:, 3]          # coincident points: clamp at 0
    with torch.autocast("cuda", dtype=torch.bfloat16):
        sq = T.euclid_sq(xyz)
        dist = torch.cdist(xyz.float(), xyz.float(), p=2)
    assert sq.dtype == torch.float32
    assert torch.equal(sq.clamp_min(0).sqrt(), dist)
    Lq = L // 32 * 32
    for r2 in (0.16, 0.64, 1.44):
        a = A.pack_mask(sq[:, :Lq].contiguous(), r2, squared=True).words
        b = A.pack_mask(dist[:, :Lq].contiguous(), r2).words
        assert torch.equal(a, b), r2


@pytest.mark.parametrize("B,L,scale", [(8, 2048, (6.0, 6.0, 3.0)), (3, 1024, (6.0, 6.0, 3.0)),
                                       (2, 2048, (0.5, 0.5, 0.5))])
def test_point_mask_equals_cdist_mask(cuda, B, L, scale):
    """The masked encoder's mask packed straight from the points (kind 3: the squared distance
    as the fma chain of cdist's K = 5 matmul form, attention.pack_mask_points) gives the bits of
    packing torch.cdist's output (coincident points included): no distance matrix, no GEMM"""
    from ov3d_amd import attention as A
    g = torch.Generator(device=cuda).manual_seed(4)
    xyz = torch.rand(B, L, 3, device=cuda, generator=g) * torch.tensor(scale, device=cuda)
    xyz[:, 7] = xyz[:, 3]
    dist = torch.cdist(xyz.float(), xyz.float(), p=2)
    for r2 in (0.16, 0.64, 1.44, 0.05):
        a = A.pack_mask_points(xyz, r2).words
        b = A.pack_mask(dist, r2).words
        assert torch.equal(a, b), r2


@pytest.mark.parametrize("with_interim", [False, True])
def test_masked_encoder_packed_equals_bool_mask_path(cuda, monkeypatch, with_interim):
    """MaskedTransformerEncoder (bf16 fused layers): PackedMask through the HIP kernels vs
    the (B*H, L, L) bool mask through PyTorch's fused SDPA, dropout off: same encoder
    output and gradients within bf16 tolerance"""
    import copy
    from ov3d_amd import transformer as T
    from ov3d_amd.pointnet2_modules import PointnetSAModuleVotes
    torch.manual_seed(5)
    layer = T.TransformerEncoderLayer(256, 4, 128, dropout=0.0)
    # the interim SA's max-pool picks its rows from bf16 values, so tiny differences re-route
    # its gradient: compared here with and without it (outputs / indices only with it)
    interim = PointnetSAModuleVotes(radius=0.4, nsample=32, npoint=512, mlp=[256, 256, 256, 256],
                                    normalize_xyz=True) if with_interim else None
    enc = T.MaskedTransformerEncoder(layer, 3, [0.16, 0.64, 1.44], interim).to(cuda).train()
    B, L = 2, 1024
    xyz = torch.rand(B, L, 3, device=cuda) * torch.tensor([4.0, 4.0, 2.0], device=cuda)
    src0 = torch.randn(L, B, 256, device=cuda)
    res = {}
    for packed in (True, False):
        twin = copy.deepcopy(enc)
        if not packed:
            monkeypatch.setattr(T.MaskedTransformerEncoder, "_packed_ok", staticmethod(lambda *a: False))
        calls = []
        real, real_pts = T.flash.pack_mask, T.flash.pack_mask_points
        monkeypatch.setattr(T.flash, "pack_mask", lambda *a, **k: calls.append(1) or real(*a, **k))
        monkeypatch.setattr(T.flash, "pack_mask_points",
                            lambda *a, **k: calls.append(1) or real_pts(*a, **k))
        src = src0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, out, inds = twin(src, xyz=xyz)
        monkeypatch.undo()
        assert len(calls) == (3 if packed else 0)
        gw = torch.randn(out.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(1))
        (out.float() * gw).sum().backward()
        res[packed] = (out.detach().float(), src.grad.clone(), inds,
                       {n: p.grad.clone() for n, p in twin.named_parameters() if p.grad is not None})
    if with_interim:
        assert torch.equal(res[True][2], res[False][2])
    assert _rel(res[True][0], res[False][0]) < 2e-2
    if with_interim:
        return
    assert _rel(res[True][1], res[False][1]) < 3e-2
    for n, g in res[False][3].items():
        assert _rel(res[True][3][n], g) < 5e-2, n


@pytest.mark.parametrize("L,B,p", [(128, 8, 0.1), (96, 3, 0.0), (64, 2, 0.3)])
@pytest.mark.parametrize("split", ["0", "1"])
def test_short_attention_one_launch_backward_equals_two(cuda, monkeypatch, L, B, p, split):
    """attn_bwd_small_kernel (dQ then dK / dV in one workgroup per (b, h)) gives exactly the
    gradients of the dQ + dK/dV launches; attn_bwd_small2_kernel (the two passes side by side in
    two workgroups, D = rowsum(dO . O) recomputed by the dK / dV pass) gives the same dQ bit for
    bit and dK / dV up to that sum's order (fp32 rounding, then bf16)"""
    from ov3d_amd import _native, attention as A
    lib = _native.load()
    monkeypatch.setenv("OV3D_ATTN_SMALL_SPLIT", split)
    torch.manual_seed(L + B)
    H = 4
    E = H * 64
    base = (torch.randn(L, B, 3 * E, device=cuda) * 1.5).to(torch.bfloat16)
    seed = A._seed(cuda).clone()
    grads = []
    prev = lib.ov3d_attn_small_bwd(-1)
    try:
        for fused in (1, 0):
            lib.ov3d_attn_small_bwd(fused)
            A._SNAPS[cuda] = seed.clone()
            x = base.clone().requires_grad_()
            q, k, v = x.chunk(3, dim=-1)
            out = A.attention(q, k, v, H, dropout_p=p, site=3)
            out.float().backward(torch.ones_like(out, dtype=torch.float32))
            grads.append(x.grad.clone())
    finally:
        lib.ov3d_attn_small_bwd(prev)
    if split == "0":
        assert torch.equal(grads[0], grads[1])
    else:
        assert torch.equal(grads[0][..., :E], grads[1][..., :E])
        torch.testing.assert_close(grads[0][..., E:].float(), grads[1][..., E:].float(),
                                   rtol=8e-3, atol=1e-4)


@pytest.mark.parametrize("Lq,Lk,B,H,masked", [(1024, 1024, 2, 4, False), (2048, 2048, 1, 2, False),
                                              (1024, 1000, 2, 2, True)])
def test_forward_with_drop_bits_ahead_equals_hashing_forward(cuda, monkeypatch, Lq, Lk, B, H, masked):
    """Long attentions take their drop bits from attn_dropgen_kernel and the forward reads
    them (BITS); the outputs, lse and both stored bit layouts equal the hashing forward's
    bit for bit (OV3D_ATTN_DROPGEN_MIN: -1 = never ahead, 0 = always)."""
    from ov3d_amd import _native, attention as A
    lib = _native.load()
    torch.manual_seed(Lq + H)
    E = H * 64
    q = torch.randn(Lq, B, E, device=cuda).to(torch.bfloat16)
    k = torch.randn(Lk, B, E, device=cuda).to(torch.bfloat16)
    v = torch.randn(Lk, B, E, device=cuda).to(torch.bfloat16)
    mask = None
    if masked:
        mask = A.pack_mask(torch.rand(B, Lq, Lk, device=cuda) * 2.0, 1.0)
    seed = torch.tensor([12345], dtype=torch.int64, device=cuda)
    res = []
    for mode in ("-1", "0"):
        monkeypatch.setenv("OV3D_ATTN_DROPGEN_MIN", mode)
        o = torch.empty(Lq, B, E, dtype=torch.bfloat16, device=cuda)
        lse = torch.empty(B * H, Lq, device=cuda)
        bits = torch.zeros(lib.ov3d_attn_dropbits_words(B, H, Lq, Lk), dtype=torch.int32, device=cuda)
        _native.call("ov3d_attn_fwd_masked", q, k, v, E, E, E, B, H, Lq, Lk, 0.125, 0.1, seed, 3, o,
                     E, lse, bits, None, 1, mask.words if mask is not None else None, like=q)
        torch.cuda.synchronize()
        res.append((o, lse, bits))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_launch_stamps_time_the_encoder_launches(cuda):
    """ov3d_stamps_arm: encoder-size launches (Lq * Lk >= min_work) stamp every wave's entry and
    exit (bench.py's in-step roofline timing); shorter launches take no slot; the kernel outputs
    are unchanged by the stamps; the stamped duration agrees with HIP events on the same launch."""
    from ov3d_amd import _native, attention as A
    L, B, H = 1024, 2, 4
    E = H * A.HEAD_DIM
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn((L, B, 3 * E), device=cuda, dtype=torch.bfloat16, generator=g).requires_grad_(True)
    gout = torch.randn((L, B, E), device=cuda, dtype=torch.bfloat16, generator=g)
    spec = ((0, 0), (0, E), (0, 2 * E))
    ref = A.attention_packed([x], spec, L, L, H, 0.0)
    ref.backward(gout)
    gref = x.grad.clone()
    x.grad = None
    buf = torch.zeros((1 << 18,), dtype=torch.int64, device=cuda)
    _native.stamps_arm(buf, min_work=L * L)
    try:
        small = torch.randn((128, B, 3 * E), device=cuda, dtype=torch.bfloat16, generator=g)
        A.attention_packed([small], spec, 128, 128, H, 0.0)         # below min_work: no slot
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = A.attention_packed([x], spec, L, L, H, 0.0)
        e1.record()
        out.backward(gout)
        torch.cuda.synchronize()
    finally:
        _native.stamps_arm(None)
    assert torch.equal(out, ref) and torch.equal(x.grad, gref)
    rec = _native.stamps_read(buf)
    kinds = [k for k, _, _ in rec]
    assert kinds == ["fwd", "dq", "dkdv"], rec
    assert all(w == L * L and 0 < ms < 50 for _, ms, w in rec), rec
    assert rec[0][1] <= e0.elapsed_time(e1) * 1.05 + 0.01, (rec, e0.elapsed_time(e1))


def test_pregen_drop_bits_forward_equals_hashing_forward(cuda):
    """drop bits generated ahead (ov3d_attn_dropgen on a side stream, attention.pregen_dropout)
    give the forward and backward of the hashing forward bit for bit"""
    from ov3d_amd import attention as flash
    torch.manual_seed(3)
    B, H, L = 2, 4, 256
    q, k, v = (torch.randn(L, B, H * 64, device=cuda, dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3))
    site = flash.new_site()
    outs = []
    for pregen in (False, True):
        for t in (q, k, v):
            t.grad = None
        if pregen:
            flash.pregen_dropout(cuda, [(site, B, H, L, L, 0.1)])
        o = flash.attention(q, k, v, H, dropout_p=0.1, site=site)
        o.float().square().sum().backward()
        outs.append((o.detach().clone(), q.grad.clone(), k.grad.clone(), v.grad.clone()))
    assert not flash._PREGEN   # consumed
    for a, b in zip(*outs):
        assert torch.equal(a, b)
