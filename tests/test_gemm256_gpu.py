"""The 256 x 256 tile GEMM and the implicit-GEMM 3x3 convolution (csrc/gemm256.hip,
gemm.gemm256 / gemm.conv3x3_gemm256): the RegionCLIP res5 convolutions over all ROIs
(clip.inference, criterion.py:397) and the decoder's memory K / V projections
(models/transformer.py:369-372).  Against the fp32 product / F.conv2d of the same bf16
operands: the error is that of one bf16 rounding of the output (plus fp32 summation order), as
for the library GEMM + im2col it replaces.  Ragged M and N (tiles past the matrix), strided
rows, bias bf16 / fp32, residual, ReLU; convolutions whose tiles straddle images, zero padding
at every border, K-steps crossing the (ky, kx) taps."""
import pytest
import torch
import torch.nn.functional as F

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


def _check(out, ref, lib=None):
    """|out - ref| within one bf16 rounding of ref (2^-8 relative) plus 1e-3 of the scale, and
    no worse than 1.5x the library's own error when given"""
    d = (out.float() - ref).abs()
    scale = ref.abs().max().item()
    bound = ref.abs() * 2.0 ** -8 + 1e-3 * scale
    bad = (d > bound).sum().item()
    assert bad == 0, (bad, d.max().item(), scale)
    if lib is not None:
        lib_err = (lib.float() - ref).abs().max().item()
        assert d.max().item() <= 1.5 * lib_err + 1e-3 * scale, (d.max().item(), lib_err)


@pytest.mark.parametrize("M,N,K,bias,res,relu", [
    (1000, 640, 1280, "bf16", False, True),      # res5 conv1 (ragged rows)
    (4096, 2560, 640, "bf16", True, True),       # res5 conv3 + identity close
    (333, 2560, 1280, "bf16", False, False),     # downsample conv
    (16384, 2048, 256, "f32", False, False),     # decoder memory K / V (8 layers stacked)
    (300, 40, 64, None, True, False),            # one K-step, N tail inside one tile
    (513, 264, 128, "f32", False, True),         # two K-steps, N tail past a tile
    (257, 512, 192, "bf16", True, True),         # three K-steps
    (1300, 320, 80, "bf16", True, True),         # K tail: layer1 conv3 (80 channels)
    (700, 640, 160, "bf16", False, True),        # K tail after two full steps (layer2, 160)
    (300, 96, 8, None, False, False),            # a single 8-wide chunk
])
def test_gemm256_matches_fp32(cuda, M, N, K, bias, res, relu):
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(M + 3 * N + 7 * K)
    wide = torch.randn(M, K + 64, device=cuda, generator=g).to(torch.bfloat16)
    a = wide[:, 64:64 + K]                               # strided rows (lda = K + 64)
    w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = None
    if bias:
        b = torch.randn(N, device=cuda, generator=g)
        b = b.to(torch.bfloat16) if bias == "bf16" else b
    r = torch.randn(M, N, device=cuda, generator=g).to(torch.bfloat16) if res else None
    assert gemm.gemm256_ok(a, w, residual=r)
    out = gemm.gemm256(a, w, bias=b, residual=r, relu=relu)
    ref = a.float() @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    if r is not None:
        ref = ref + r.float()
    if relu:
        ref = ref.clamp_min(0)
    assert out.shape == (M, N) and out.dtype == torch.bfloat16
    lib = torch.nn.functional.linear(a, w, b.to(torch.bfloat16) if b is not None else None)
    if r is not None:
        lib = lib + r
    if relu:
        lib = lib.clamp_min(0)
    _check(out, ref, lib)


def test_gemm256_exact_integers(cuda):
    """small-integer operands: every product and sum is exact in fp32 and the outputs are exact
    in bf16 -- the result must be bit-equal (catches fragment / swizzle / epilogue index errors
    that a tolerance could hide); asymmetric operands (A = I would hide a transpose)"""
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(5)
    M, N, K = 700, 520, 320
    a = torch.randint(-1, 2, (M, K), device=cuda, generator=g).to(torch.bfloat16)
    w = torch.randint(-1, 2, (N, K), device=cuda, generator=g).to(torch.bfloat16)
    w[:, 0] = torch.arange(N, device=cuda) % 7 - 3   # column-dependent: a swapped C write shows
    a[:, 1] = torch.arange(M, device=cuda) % 5 - 2
    b = torch.randint(-4, 5, (N,), device=cuda, generator=g).float()
    out = gemm.gemm256(a, w, bias=b)
    ref = a.float() @ w.float().t() + b
    assert ref.abs().max().item() < 256                  # exact in bf16
    assert torch.equal(out.float(), ref)


@pytest.mark.parametrize("n,H,W,C,cout,res", [
    (5, 18, 18, 640, 640, False),    # res5 block 1 conv2 (ROI 18 x 18), tiles straddle ROIs
    (13, 9, 9, 640, 640, True),      # res5 blocks 2-6 conv2 (9 x 9: 81 rows per ROI)
    (2, 34, 46, 320, 320, False),    # layer3 conv2 on an image-sized map
    (3, 5, 7, 64, 72, False),        # small: one K-step per tap, Cout tail
])
def test_conv3x3_gemm256_matches_conv2d(cuda, n, H, W, C, cout, res):
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(n * H * W + C)
    x = torch.randn(n, H, W, C, device=cuda, generator=g).to(torch.bfloat16)
    wt = (torch.randn(cout, 3, 3, C, device=cuda, generator=g) / (9 * C) ** 0.5).to(torch.bfloat16)
    b = torch.randn(cout, device=cuda, generator=g).to(torch.bfloat16)
    r = torch.randn(n * H * W, cout, device=cuda, generator=g).to(torch.bfloat16) if res else None
    wm = wt.reshape(cout, 9 * C)
    assert gemm.conv3x3_ok(x, wm)
    out = gemm.conv3x3_gemm256(x, wm, bias=b, residual=r, relu=True)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), wt.permute(0, 3, 1, 2).float(), b.float(), padding=1)
    ref = ref.permute(0, 2, 3, 1)
    if r is not None:
        ref = ref + r.float().view(n, H, W, cout)
    ref = ref.clamp_min(0)
    assert out.shape == (n, H, W, cout)
    _check(out, ref)


def test_conv3x3_gemm256_border_taps_exact(cuda):
    """integer input and weights with one nonzero tap per output channel group: each output is
    one shifted input pixel, so the zero padding at every border and the (ky, kx) order are
    checked exactly"""
    from ov3d_amd import gemm
    n, H, W, C = 3, 9, 9, 64
    g = torch.Generator(device=cuda).manual_seed(9)
    x = torch.randint(-8, 9, (n, H, W, C), device=cuda, generator=g).to(torch.bfloat16)
    cout = 9 * 8
    wt = torch.zeros(cout, 3, 3, C, device=cuda)
    for t in range(9):
        for j in range(8):
            wt[8 * t + j, t // 3, t % 3, (5 * j + t) % C] = 1.0
    wt = wt.to(torch.bfloat16)
    out = gemm.conv3x3_gemm256(x, wt.reshape(cout, 9 * C))
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), wt.permute(0, 3, 1, 2).float(), padding=1)
    assert torch.equal(out.float(), ref.permute(0, 2, 3, 1))


def test_gemm256_pair_equals_two_products(cuda):
    """the decoder's K and V projections of the memory (8 layers stacked: 16384 x 2048 x 256) in
    one launch equal the two single launches bit for bit, and the fp32 products within one
    rounding (models/transformer.py:369-372)"""
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(11)
    M, N, K = 16384, 2048, 256
    a1, a2 = (torch.randn(M, K, device=cuda, generator=g).to(torch.bfloat16) for _ in range(2))
    w1, w2 = ((torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).to(torch.bfloat16) for _ in range(2))
    b1, b2 = (torch.randn(N, device=cuda, generator=g).to(torch.bfloat16) for _ in range(2))
    o1, o2 = gemm.gemm256_pair(a1, w1, b1, a2, w2, b2)
    assert torch.equal(o1, gemm.gemm256(a1, w1, bias=b1))
    assert torch.equal(o2, gemm.gemm256(a2, w2, bias=b2))
    _check(o1, a1.float() @ w1.float().t() + b1.float())
    _check(o2, a2.float() @ w2.float().t() + b2.float())


@pytest.mark.parametrize("R,C,H,d", [(4096, 2560, 40, 64), (300, 384, 6, 64)])
def test_gemm256_batched_attnpool_products(cuda, R, C, H, d):
    """the attention pool's per-head products in one launch each (regionclip._pool_fused):
    a_h = q_h Wk_h (K = d, strided A columns, (H, R, C) output) and o_h = y_h Wv_h^T + bv_h
    (N = d, f32 bias, column-block output): equal to the per-problem single launches bit for
    bit and within one rounding of the fp32 bmm"""
    from ov3d_amd import gemm
    g = torch.Generator(device=cuda).manual_seed(R + H)
    q = torch.randn(R, C, device=cuda, generator=g).to(torch.bfloat16)
    wkt = (torch.randn(H, C, d, device=cuda, generator=g) / d ** 0.5).to(torch.bfloat16)
    a = torch.empty((H, R, C), dtype=torch.bfloat16, device=cuda)
    gemm.gemm256_batched(q, C, d, wkt, d, C * d, a, C, R * C, R, C, d, H)
    ref = torch.bmm(q.float().view(R, H, d).transpose(0, 1), wkt.float().transpose(1, 2))
    _check(a, ref)
    for h in (0, H - 1):
        assert torch.equal(a[h], gemm.gemm256(q[:, h * d:(h + 1) * d].contiguous(), wkt[h].contiguous()))
    y = torch.randn(H, R, C, device=cuda, generator=g).to(torch.bfloat16)
    wv = (torch.randn(H * d, C, device=cuda, generator=g) / C ** 0.5).to(torch.bfloat16)
    bv = torch.randn(H * d, device=cuda, generator=g)
    o = torch.full((R, H * d), 7.0, dtype=torch.bfloat16, device=cuda)
    gemm.gemm256_batched(y, C, R * C, wv, C, d * C, o, H * d, d, R, d, C, H, bias=bv, sbias=d)
    ref = torch.bmm(y.float(), wv.float().view(H, d, C).transpose(1, 2)) + bv.view(H, 1, d)
    _check(o.view(R, H, d).transpose(0, 1), ref)


@pytest.mark.parametrize("M,ldx", [(262144, 256), (131072 + 37, 264), (200, 256), (5, 320)])
def test_rows256_equals_gemm256_bitwise(M, ldx):
    """csrc/rows256.hip (the masked encoder's interim SA products: W resident per CU, X streamed
    through LDS) against gemm256 on the same bf16 operands, no bias: every output bit, with a
    ragged last tile and strided rows; and the fp32 product within one bf16 rounding"""
    from ov3d_amd import _native, gemm
    torch.manual_seed(3)
    dev = torch.device("cuda", 0)
    xb = torch.randn(M, ldx, device=dev).to(torch.bfloat16)
    x = xb[:, :256]
    w = (0.06 * torch.randn(256, 256, device=dev)).to(torch.bfloat16)
    y = torch.full((M, 256), float("nan"), device=dev, dtype=torch.bfloat16)
    _native.call("ov3d_rows256", x, x.stride(0), 256, 256, w, w.stride(0), y, y.stride(0), M,
                 gemm._rows256_counters(dev), like=x)
    ref = gemm.gemm256(x, w)
    assert torch.equal(y, ref)
    _check(y[:4096], x[:4096].float() @ w.float().t())


def test_rows256_routes_interim_sa_products():
    """_linear / _dgrad send the 2^18-row 256 x 256 products to rows256 (and equal gemm256's)"""
    from ov3d_amd import _native, gemm
    torch.manual_seed(4)
    dev = torch.device("cuda", 0)
    x = torch.randn(1 << 17, 256, device=dev).to(torch.bfloat16)
    w = (0.06 * torch.randn(256, 256, device=dev)).to(torch.bfloat16)
    assert gemm.rows256_ok(x, w) and not gemm.rows256_ok(x[:1000], w)
    seen = []
    orig = _native.call

    def spy(name, *a, **k):
        seen.append(name)
        return orig(name, *a, **k)

    _native.call = spy
    try:
        y = gemm._linear(x, w, None)
        dx = gemm._dgrad(x, w)
    finally:
        _native.call = orig
    assert seen.count("ov3d_rows256") == 2, seen
    assert torch.equal(y, gemm.gemm256(x, w))
    assert torch.equal(dx, gemm.gemm256(x, w.t().contiguous()))


@pytest.mark.parametrize("M", [262144, 131072 + 37, 77])
def test_rows256_k264_equals_gemm256_bitwise(M):
    """the interim SA's first layer: 259 inputs zero-padded to 264 columns (rows and weight), on
    rows256's K-tail mode against gemm256's K-tail step, every output bit (rows with all-zero
    inputs included: the zero steps are the same instructions)"""
    from ov3d_amd import _native, gemm
    torch.manual_seed(5)
    dev = torch.device("cuda", 0)
    x = torch.randn(M, 264, device=dev).to(torch.bfloat16)
    x[:, 259:] = 0
    x[:3] = 0
    w = torch.nn.functional.pad((0.06 * torch.randn(256, 259, device=dev)).to(torch.bfloat16), (0, 5))
    y = torch.full((M, 256), float("nan"), device=dev, dtype=torch.bfloat16)
    _native.call("ov3d_rows256", x, x.stride(0), 264, 256, w, w.stride(0), y, y.stride(0), M,
                 gemm._rows256_counters(dev), like=x)
    assert torch.equal(y, gemm.gemm256(x, w))
    if M >= gemm.GEMM256_MIN_M:
        assert gemm.rows256_ok(x, w) and torch.equal(gemm._linear(x, w, None), y)


@pytest.mark.parametrize("M", [262144, 131072 + 37, 150])
def test_rows256_n264_equals_gemm256_bitwise(M):
    """the first interim SA layer's input gradient dy (M, 256) . W (256, 264): 264 output columns
    (the 8 past 256 from an extra 16-column block per wave) against gemm256, every bit; routed
    from gemm._dgrad"""
    from ov3d_amd import _native, gemm
    torch.manual_seed(6)
    dev = torch.device("cuda", 0)
    dy = torch.randn(M, 256, device=dev).to(torch.bfloat16)
    w = torch.nn.functional.pad((0.06 * torch.randn(256, 259, device=dev)).to(torch.bfloat16), (0, 5))
    wt = w.t().contiguous()                        # (264, 256) rows
    y = torch.full((M, 264), float("nan"), device=dev, dtype=torch.bfloat16)
    _native.call("ov3d_rows256", dy, dy.stride(0), 256, 264, wt, wt.stride(0), y, y.stride(0), M,
                 gemm._rows256_counters(dev), like=dy)
    assert torch.equal(y, gemm.gemm256(dy, wt))
    if M >= gemm.GEMM256_MIN_M:
        assert gemm.rows256_ok(dy, wt) and torch.equal(gemm._dgrad(dy, w), y)
