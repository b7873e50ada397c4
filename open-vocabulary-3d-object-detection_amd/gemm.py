"""Row-major linear layer with a split-K weight gradient.

Every dense layer of the hot path is a GEMM over R rows (points, memory tokens or
query slots) with small channel counts: y = x W^T with x (R, Cin), W (Cout, Cin),
R = 2^20 for the SA MLP, 2^14 for the encoder, Cout*Cin <= 768*256.  Its weight
gradient dW = dy^T x has a tiny output tile and an R-long reduction; handed to the
BLAS as one GEMM it runs on 7-21 workgroups of the 256 CUs (1.4-2.1 ms per SA layer,
measured: profiles/r01_kernel_stats_v2.csv).  Here the reduction is split into
row chunks computed as one batched GEMM (>= ~256 workgroups) and summed in fp32.
"""
import ctypes
import os
import weakref

import torch
from torch.autograd import Function

_TARGET_TILES = 512     # aim for this many (chunk x 64x64 tile) work items
_MIN_ROWS = 256         # never split below this many rows per chunk


def _chunks(R, cout, cin):
    tiles = max(1, ((cout + 63) // 64) * ((cin + 63) // 64))
    nc = 1
    while (nc * 2 * tiles <= _TARGET_TILES and R % (nc * 2) == 0 and R // (nc * 2) >= _MIN_ROWS):
        nc *= 2
    return nc


_F32_OUT = None   # does this build's bmm take out_dtype=float32 for bf16 inputs (hipBLASLt)?

# Short row blocks (the decoder: nqueries * batch = 1024 rows) run on csrc/rowsgemm.hip: one
# memory round trip per launch instead of a library GEMM's K pipeline.  Longer row blocks
# stay on hipBLASLt, whose large tiles reuse operands across rows.
ROWS_GEMM = True
ROWS_GEMM_MAX_M = int(os.environ.get("OV3D_ROWS_GEMM_MAX_M", "2048"))


def _rows_gemm_ok(a, w, trans_b):
    if not (ROWS_GEMM and a.is_cuda and a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and a.dim() == 2 and w.dim() == 2 and a.stride(1) == 1 and w.stride(1) == 1):
        return False
    M, K = a.shape
    N = w.shape[0] if trans_b else w.shape[1]
    if M > ROWS_GEMM_MAX_M or (w.shape[1] if trans_b else w.shape[0]) != K:
        return False
    if a.data_ptr() % 16 or w.data_ptr() % 16 or a.stride(0) % 8 or w.stride(0) % 8:
        return False
    from . import _native
    return bool(_native.load().ov3d_rows_gemm_supported(M, N, K))


def rows_gemm(a, w, bias=None, trans_b=True):
    """a (M, K) bf16 rows; w bf16 (N, K) when trans_b (y = a w^T + bias, nn.Linear) else
    (K, N) (y = a w) -> (M, N) bf16 (csrc/rowsgemm.hip; check _rows_gemm_ok first)"""
    from . import _native
    M, K = a.shape
    N = w.shape[0] if trans_b else w.shape[1]
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if bias is not None and (bias.dtype != torch.bfloat16 or not bias.is_contiguous()):
        bias = bias.to(torch.bfloat16).contiguous()
    _native.call("ov3d_rows_gemm", M, N, K, a, a.stride(0), w, w.stride(0), int(trans_b), bias,
                 out, N, like=a)
    return out


class _RgProblem(ctypes.Structure):
    """mirror of ov3d_rows_gemm_problem (include/ov3d.h)"""
    _fields_ = [("A", ctypes.c_void_p), ("lda", ctypes.c_longlong), ("W", ctypes.c_void_p),
                ("ldw", ctypes.c_longlong), ("bias", ctypes.c_void_p), ("C", ctypes.c_void_p),
                ("ldc", ctypes.c_longlong), ("N", ctypes.c_int), ("K", ctypes.c_int)]


class _LnProblem(ctypes.Structure):
    """mirror of ov3d_lngemm_problem (include/ov3d.h)"""
    _fields_ = [("W", ctypes.c_void_p), ("ldw", ctypes.c_longlong), ("bias", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("ldo", ctypes.c_longlong), ("N", ctypes.c_int),
                ("sel", ctypes.c_int)]


def rows_gemm_group(problems, trans_b=True):
    """[(a, w, bias)] over the same rows -> [outputs], one launch (every pair must pass
    _rows_gemm_ok; at most 4)"""
    from . import _native
    M = problems[0][0].shape[0]
    outs, keep, probs = [], [], []
    for a, w, b in problems:
        N = w.shape[0] if trans_b else w.shape[1]
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
        if b is not None and (b.dtype != torch.bfloat16 or not b.is_contiguous()):
            b = b.to(torch.bfloat16).contiguous()
        keep.append(b)
        outs.append(out)
        probs.append(_RgProblem(a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0),
                                b.data_ptr() if b is not None else None, out.data_ptr(), N, N,
                                a.shape[1]))
    arr = (_RgProblem * len(probs))(*probs)
    _native.call("ov3d_rows_gemm_group", M, len(probs), ctypes.addressof(arr), int(trans_b),
                 like=problems[0][0])
    return outs


ROWS_GEMM_GROUP = os.environ.get("OV3D_ROWS_GEMM_GROUP", "1") != "0"


def _group_ok(pairs, trans_b):
    return (ROWS_GEMM_GROUP and 1 < len(pairs) <= 4 and len({a.shape[0] for a, _ in pairs}) == 1
            and all(_rows_gemm_ok(a, w, trans_b) for a, w in pairs))


# Long row blocks (the encoder: batch * 2048 rows, the heads: batch * 1024) run on
# csrc/tilegemm.hip: persistent 64- / 128-row tiles, both operands double-buffered in LDS, the
# FFN activation as an epilogue (DESIGN.md "Long row-block GEMMs").  OV3D_TILE_GEMM=0: hipBLASLt.
TILE_GEMM = os.environ.get("OV3D_TILE_GEMM", "1") == "1"


def _tile_gemm_ok(a, w, trans_b):
    if not (TILE_GEMM and a.is_cuda and a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and a.dim() == 2 and w.dim() == 2 and a.stride(1) == 1 and w.stride(1) == 1):
        return False
    M, K = a.shape
    N = w.shape[0] if trans_b else w.shape[1]
    if M <= ROWS_GEMM_MAX_M or (w.shape[1] if trans_b else w.shape[0]) != K:
        return False
    if a.data_ptr() % 16 or w.data_ptr() % 16 or a.stride(0) % 8 or w.stride(0) % 8:
        return False
    from . import _native
    return bool(_native.load().ov3d_tile_gemm_supported(M, N, K))


def tile_gemm(a, w, bias=None, trans_b=True, out=None):
    """as rows_gemm, on the long row-block kernel (check _tile_gemm_ok first); `out` an (M, N)
    bf16 row view (stride(1) == 1, 16-byte aligned, row stride % 8 == 0) or None"""
    from . import _native
    M, K = a.shape
    N = w.shape[0] if trans_b else w.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if bias is not None and (bias.dtype != torch.bfloat16 or not bias.is_contiguous()
                             or bias.data_ptr() % 8):   # 8-byte bias pieces
        bias = bias.to(torch.bfloat16).contiguous().clone()
    wide = bias is not None and N > 2048   # the kernel stages the bias row in LDS (N <= 2048)
    _native.call("ov3d_tile_gemm", M, N, K, a, a.stride(0), w, w.stride(0), int(trans_b),
                 None if wide else bias, out, out.stride(0), like=a)
    if wide:
        out.add_(bias)
    return out


def tile_out_ok(out):
    return (out.dtype == torch.bfloat16 and out.dim() == 2 and out.stride(1) == 1
            and out.stride(0) % 8 == 0 and out.data_ptr() % 16 == 0)


def tile_bmm_ok(a, w, trans_b):
    """a (B, M, K) x w (B, N, K) (trans_b) / (B, K, N) on the long row-block kernel"""
    if not (TILE_GEMM and a.is_cuda and a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and a.dim() == 3 and w.dim() == 3 and a.shape[0] == w.shape[0]
            and a.stride(2) == 1 and w.stride(2) == 1):
        return False
    B, M, K = a.shape
    N = w.shape[1] if trans_b else w.shape[2]
    if M <= ROWS_GEMM_MAX_M or (w.shape[2] if trans_b else w.shape[1]) != K:
        return False
    if (a.data_ptr() % 16 or w.data_ptr() % 16 or any(x % 8 for x in a.stride()[:2] + w.stride()[:2])):
        return False
    from . import _native
    return bool(_native.load().ov3d_tile_gemm_supported(M, N, K))


def tile_bmm(a, w, trans_b):
    """torch.bmm(a, w.transpose(1, 2) if trans_b else w) -> (B, M, N) bf16, one launch"""
    from . import _native
    B, M, K = a.shape
    N = w.shape[1] if trans_b else w.shape[2]
    out = torch.empty((B, M, N), dtype=torch.bfloat16, device=a.device)
    _native.call("ov3d_tile_gemm_batched", B, M, N, K, a, a.stride(1), a.stride(0), w, w.stride(1),
                 w.stride(0), int(trans_b), out, N, M * N, like=a)
    return out


def _aligned_bias(b):
    if b is not None and (b.dtype != torch.bfloat16 or not b.is_contiguous() or b.data_ptr() % 8):
        b = b.to(torch.bfloat16).contiguous().clone()
    return b


def shape_ok(M, N, K):
    """a (M, K) x (K, N) product on fresh contiguous bf16 rows runs on rows_gemm or tile_gemm"""
    from . import _native
    lib = _native.load()
    if ROWS_GEMM and M <= ROWS_GEMM_MAX_M:
        return bool(lib.ov3d_rows_gemm_supported(M, N, K))
    return TILE_GEMM and M > ROWS_GEMM_MAX_M and bool(lib.ov3d_tile_gemm_supported(M, N, K))


def act_gemm_ok(a, w, trans_b):
    """rows_gemm / tile_gemm can run a (M, K) x w product with an activation epilogue"""
    return _rows_gemm_ok(a, w, trans_b) or _tile_gemm_ok(a, w, trans_b)


def act_gemm(a, w, bias=None, trans_b=True, epilogue=0, p=0.0, seed=None, site=0, h=None):
    """(M, N) bf16 = a (M, K) x w (w (N, K) when trans_b, else (K, N)) + bias, with the FFN
    epilogue (0 none, 1 dropout_p(relu(.)), 2 h > 0 ? . / (1 - p) : 0) on the short row-block
    kernel (M <= ROWS_GEMM_MAX_M) or the long one; check act_gemm_ok first"""
    from . import _native
    M, K = a.shape
    N = w.shape[0] if trans_b else w.shape[1]
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    name = "ov3d_rows_gemm_act" if _rows_gemm_ok(a, w, trans_b) else "ov3d_tile_gemm_act"
    _native.call(name, M, N, K, a, a.stride(0), w, w.stride(0), int(trans_b), _aligned_bias(bias),
                 int(epilogue), float(p), seed, int(site), h, h.stride(0) if h is not None else 0,
                 out, N, like=a)
    return out


def tile_gemm2(a1, w1, a2, w2):
    """a1 w1 + a2 w2 (input-gradient layout: w (K, N)) in one launch of the long row-block
    kernel (check _tile_gemm_ok on both pairs first)"""
    from . import _native
    M, N = a1.shape[0], w1.shape[1]
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a1.device)
    _native.call("ov3d_tile_gemm2", M, N, a1.shape[1], a1, a1.stride(0), w1, w1.stride(0),
                 a2.shape[1], a2, a2.stride(0), w2, w2.stride(0), 0, out, N, like=a1)
    return out


# Large products (the RegionCLIP res5 convolutions over all ROIs, the decoder's memory K / V
# projections): 256 x 256 tiles on csrc/gemm256.hip, bias / residual / ReLU in the epilogue,
# and the 3x3 convolution as an implicit GEMM (no column matrix).  OV3D_GEMM256=0: hipBLASLt.
GEMM256 = os.environ.get("OV3D_GEMM256", "1") == "1"


def _rows_ok(t):
    return (t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.data_ptr() % 16 == 0 and t.is_cuda)


def gemm256_ok(a, w, residual=None, out=None):
    """a (M, K) x w (N, K)^T can run on gemm256 (bf16 rows, K % 8, N % 8, 16-byte rows)"""
    if not (GEMM256 and _rows_ok(a) and _rows_ok(w)):
        return False
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] < K or K % 8 or N % 8 or 256 * max(a.stride(0), w.stride(0)) * 2 + 2 * K >= 2 ** 31:
        return False
    if residual is not None and not (_rows_ok(residual) and tuple(residual.shape) == (M, N)):
        return False
    return out is None or (_rows_ok(out) and tuple(out.shape) == (M, N))


def _bias_arg(bias):
    if bias is None:
        return None, 0
    if bias.dtype == torch.float32:
        b = bias if bias.is_contiguous() and bias.data_ptr() % 16 == 0 else bias.contiguous().clone()
        return b, 1
    b = bias.to(torch.bfloat16)
    if not b.is_contiguous() or b.data_ptr() % 16:
        b = b.contiguous().clone()
    return b, 0


def gemm256(a, w, bias=None, residual=None, relu=False, out=None):
    """act(a w^T + bias + residual) -> (M, N) bf16 on the 256 x 256 tile kernel (check
    gemm256_ok first); bias bf16 or fp32 (N,), residual (M, N) bf16 rows"""
    from . import _native
    M, K = a.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    b, bf32 = _bias_arg(bias)
    _native.call("ov3d_gemm256", a, a.stride(0), w, w.stride(0), b, bf32, residual,
                 residual.stride(0) if residual is not None else 0, out, out.stride(0), M, N, K,
                 int(bool(relu)), like=a)
    return out


def gemm256_pair(a1, w1, b1, a2, w2, b2):
    """(a1 w1^T + b1, a2 w2^T + b2) in ONE launch of the tile kernel (same shapes; check
    gemm256_ok on both pairs and that a1 / a2, w1 / w2 share their row strides first)"""
    from . import _native
    M, K = a1.shape
    N = w1.shape[0]
    o1 = torch.empty((M, N), dtype=torch.bfloat16, device=a1.device)
    o2 = torch.empty_like(o1)
    (bb1, bf32), (bb2, _) = _bias_arg(b1), _bias_arg(b2.to(b1.dtype) if b1 is not None else None)
    _native.call("ov3d_gemm256_pair", a1, a2, a1.stride(0), w1, w2, w1.stride(0), bb1, bb2, bf32,
                 o1, o2, N, M, N, K, like=a1)
    return o1, o2


def gemm256_batched(A, lda, sA, B, ldb, sB, C, ldc, sC, M, N, K, nbatch, bias=None, sbias=0,
                    relu=False, like=None):
    """nbatch products in one launch of the tile kernel: problem p reads A + p sA, B + p sB (bf16
    rows, K contiguous), bias + p sbias (bf16 or f32, or None) and writes C + p sC (bf16); all
    offsets and leading dimensions in elements of the given base tensors (no shape checks here:
    the C entry validates strides and alignment)"""
    from . import _native
    bf32 = 0
    if bias is not None:
        bf32 = int(bias.dtype == torch.float32)
    _native.call("ov3d_gemm256_batched", A, lda, sA, B, ldb, sB, bias, sbias, bf32, C, ldc, sC, M, N,
                 K, nbatch, int(bool(relu)), like=like if like is not None else A)


def conv3x3_ok(x, w):
    """x (n, H, W, C) NHWC bf16, w (Cout, >= 9C) bf16 rows: the implicit-GEMM 3x3 convolution"""
    if not (GEMM256 and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.is_contiguous()
            and x.data_ptr() % 16 == 0 and _rows_ok(w)):
        return False
    n, H, W, C = x.shape
    return (C % 64 == 0 and w.shape[1] >= 9 * C and w.shape[0] % 8 == 0 and n * H * W < 2 ** 31
            and (256 + 2 * W + 2 + H * W) * C * 2 < 2 ** 31)


def conv3x3_gemm256(x, w, bias=None, residual=None, relu=False):
    """3x3 convolution (pad 1, stride 1) of NHWC x with the (Cout, 3, 3, C) channels-last weight
    viewed as (Cout, 9C) rows, + bias (+ residual rows) (+ ReLU) -> (n, H, W, Cout) bf16, as an
    implicit GEMM (check conv3x3_ok first)"""
    from . import _native
    n, H, W, C = x.shape
    cout = w.shape[0]
    out = torch.empty((n, H, W, cout), dtype=torch.bfloat16, device=x.device)
    b, bf32 = _bias_arg(bias)
    _native.call("ov3d_conv3x3_gemm256", x, n, H, W, C, w, w.stride(0), b, bf32, residual,
                 residual.stride(0) if residual is not None else 0, out, cout, cout,
                 int(bool(relu)), like=x)
    return out


# products over this many rows and more (the masked encoder's interim SA: 2^18 rows) run on the
# 256 x 256 tile kernel (gemm256, ~1 PF/s there) rather than the long row-block kernel (~0.5)
GEMM256_MIN_M = int(os.environ.get("OV3D_GEMM256_MIN_M", str(1 << 17)))


# (M, 256 or 264) x (256, K)^T products over this many rows and more, without bias (the masked
# encoder's interim SA layers and their 256-wide input gradients), on the streaming kernel
# (csrc/rows256.hip: W resident per CU, equal to gemm256's outputs bit for bit); "0": gemm256
ROWS256 = os.environ.get("OV3D_ROWS256", "1") != "0"


def rows256_ok(a, w, bias=None):
    """a (M, K) x w (N, K)^T runs on rows256: (K, N) = (256, 256), (264, 256) (the zero-padded
    first layer) or (256, 264) (its input gradient)"""
    from . import _native
    K = a.shape[1] if a.dim() == 2 else 0
    N = w.shape[0] if w.dim() == 2 else 0
    return (ROWS256 and bias is None and a.shape[0] >= GEMM256_MIN_M and _rows_ok(a) and _rows_ok(w)
            and (K, N) in ((256, 256), (264, 256), (256, 264)) and w.shape[1] == K
            and bool(_native.load().ov3d_rows256_supported(a.shape[0], N, K)))


def rows256(a, w):
    """a (M, K) w (N, K)^T -> (M, N) bf16 (check rows256_ok first)"""
    from . import _native
    N = w.shape[0]
    out = torch.empty((a.shape[0], N), dtype=torch.bfloat16, device=a.device)
    _native.call("ov3d_rows256", a, a.stride(0), a.shape[1], N, w, w.stride(0), out, out.stride(0),
                 a.shape[0], _rows256_counters(a.device), like=a)
    return out


_R256_COUNTERS = {}


def _rows256_counters(device):
    c = _R256_COUNTERS.get(device)
    if c is None:   # tile claims of csrc/rows256.hip: zero, and left zero by every launch
        c = torch.zeros(2, dtype=torch.int32, device=device)
        _R256_COUNTERS[device] = c
    return c


def _linear(x, w, b):
    """F.linear on bf16 rows (bias in the epilogue): short row blocks on rowsgemm, long ones
    on tilegemm, the longest on rows256 (256 x 256 weights) or gemm256"""
    if _rows_gemm_ok(x, w, True):
        return rows_gemm(x, w, b, trans_b=True)
    if x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and rows256_ok(x, w, b):
        return rows256(x, w)
    if x.shape[0] >= GEMM256_MIN_M and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 \
            and gemm256_ok(x, w):
        return gemm256(x, w, bias=b)
    if _tile_gemm_ok(x, w, True):
        return tile_gemm(x, w, b, trans_b=True)
    if x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and gemm256_ok(x, w):
        # K % 64 != 0 (the masked encoder's interim SA: 256 features + xyz padded to 264)
        return gemm256(x, w, bias=b)
    return torch.nn.functional.linear(x, w, b)


def linear_weight_grads(dy, xc, w, b, need_w, need_b):
    """(dW, db) of y = xc w^T + b for the gradient dy (bf16 rows like xc), or (None, None)
    when they were queued for the grouped launch at the end of the backward (DEFER_WGRAD)"""
    want_b = b is not None and need_b
    if need_w and can_defer(xc, w, b if want_b else None):
        defer_weight_grad(dy, xc, w, b if want_b else None)
        return None, None
    if need_w and _fused_ok(dy, xc):
        dw, db = fused_weight_grad(dy, xc, bias=want_b)
        return dw.to(w.dtype), (db.to(b.dtype) if want_b else None)
    dw = weight_grad(dy, xc).to(w.dtype) if need_w else None
    db = torch.sum(dy, dim=0, dtype=torch.float32).to(b.dtype) if want_b else None
    return dw, db


def _dgrad(dy, w):
    """dy (M, N) @ w (N, K) for the input gradient of a linear layer"""
    if _rows_gemm_ok(dy, w, False):
        return rows_gemm(dy, w, trans_b=False)
    if dy.shape[0] >= GEMM256_MIN_M and dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
        wt = w.t().contiguous()   # (K, N) rows: dx = dy wt^T on the 256 x 256 tile kernel
        if rows256_ok(dy, wt):
            return rows256(dy, wt)
        if gemm256_ok(dy, wt):
            return gemm256(dy, wt)
    if _tile_gemm_ok(dy, w, False):
        return tile_gemm(dy, w, trans_b=False)
    if dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and dy.shape[0] > ROWS_GEMM_MAX_M:
        wt = w.t().contiguous()   # (K, N) rows: dx = dy wt^T on the tile kernel
        if gemm256_ok(dy, wt):
            return gemm256(dy, wt)
    return dy @ w


def _bmm_f32(a, b):
    """bf16 x bf16 -> fp32 batched GEMM without rounding the per-chunk partials to bf16."""
    global _F32_OUT
    if a.dtype in (torch.bfloat16, torch.float16) and a.is_cuda and _F32_OUT is not False:
        try:
            out = torch.bmm(a, b, out_dtype=torch.float32)
            _F32_OUT = True
            return out
        except (RuntimeError, TypeError):
            _F32_OUT = False
    return torch.bmm(a, b)


_WG_COUNTERS = {}


def _wg_counters(device):
    c = _WG_COUNTERS.get(device)
    if c is None:   # arrival counters of csrc/wgrad.hip: zero, and left zero by every launch
        c = torch.zeros(4096, dtype=torch.int32, device=device)
        _WG_COUNTERS[device] = c
    return c


def _wg_splits(R, N, K):
    from . import _native
    tiles = _native.load().ov3d_wgrad_tiles(N, K)
    # short R: parallelism; long R: fewer partials to sum (tools/wgrad_split_probe.py sweep)
    rows = 128 if R <= 2048 else (256 if R <= 4096 else 512)
    return max(1, min((R + rows - 1) // rows, 512 // tiles))


def _wg_group_splits(R):
    """row splits of one problem in the grouped launch (256 x 256 tiles, csrc/wgrad.hip):
    1024-row chunks (32 stages of 32 rows) keep the split partials to 256 KB per tile and
    chunk, and give a few workgroups per CU over the step's ~100 problems"""
    return max(1, (R + 1023) // 1024)


def _fused_ok(dy, x):
    """the one-launch HIP weight/bias gradient applies to bf16 rows on the ROCm device"""
    return (dy.is_cuda and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
            and dy.dim() == 2 and x.dim() == 2 and dy.stride(1) == 1 and x.stride(1) == 1)


def fused_weight_grad(dy, x, bias=True, out_w=None, out_b=None, bn=None):
    """dW = dy^T x (fp32, (N, K)) and db = column sums of dy (fp32, (N,)) in ONE HIP launch
    (csrc/wgrad.hip, ov3d_wgrad); dy (R, N), x (R, K) bf16 rows (row strides taken from the
    tensors).  out_w / out_b: optional fp32 destinations (row slices of a larger gradient).
    bn=(scale, shift): x is relu(x * scale + shift) in bf16, applied on load (ov3d_wgrad_bn)."""
    from . import _native
    R, N = dy.shape
    K = x.shape[1]
    if dy.stride(1) != 1 or x.stride(1) != 1:
        raise ValueError("fused_weight_grad: rows must be contiguous")
    dev = dy.device
    dw = out_w if out_w is not None else torch.empty((N, K), dtype=torch.float32, device=dev)
    db = None
    if bias:
        db = out_b if out_b is not None else torch.empty((N,), dtype=torch.float32, device=dev)
    nsplit = _wg_splits(R, N, K)
    lib = _native.load()
    if lib.ov3d_wgrad_tiles(N, K) > 4096:
        raise ValueError("fused_weight_grad: too many output tiles")
    ws_n = lib.ov3d_wgrad_workspace(R, N, K, nsplit)
    ws = torch.empty((max(ws_n, 1),), dtype=torch.float32, device=dev)
    if bn is not None:
        _native.call("ov3d_wgrad_bn", dy, dy.stride(0), x, x.stride(0), R, N, K, bn[0], bn[1], dw,
                     dw.stride(0), db, ws, _wg_counters(dev), nsplit, like=dy)
    else:
        _native.call("ov3d_wgrad", dy, dy.stride(0), x, x.stride(0), R, N, K, dw, dw.stride(0), db,
                     ws, _wg_counters(dev), nsplit, like=dy)
    return dw, db


# ---------------------------------------------------------------- deferred weight grads
# dW / db of a linear layer are not needed by anything else in the backward pass, so they
# can run after it: every deferred (dy, x) pair of one backward pass goes into ONE grouped
# launch (csrc/wgrad.hip ov3d_wgrad_group) queued to run when the autograd engine finishes
# (queue_callback), instead of ~100 latency-bound launches interleaved with the dgrad
# chain.  The layers' backward returns None for the weight / bias and the flush assigns
# (or adds into) ``param.grad`` itself, so hooks on those parameters do not fire:
# enabled only by the single-process training step (bench.py / graphs.StepGraph), never
# under DDP (its reducer needs the per-parameter gradient hooks).
DEFER_WGRAD = False
WGRAD_SINGLE_MIN_R = int(os.environ.get("OV3D_WGRAD_SINGLE_MIN_R", str(1 << 17)))
_PENDING = []
_PENDING_COLS = []   # deferred LayerNorm weight / bias gradients (resnorm.py)
_QUEUED = [False]


def _ensure_flush():
    if not _QUEUED[0]:
        torch.autograd.Variable._execution_engine.queue_callback(flush_weight_grads)
        _QUEUED[0] = True


class _ColSeg(ctypes.Structure):
    """mirror of ov3d_colsum_seg"""
    _fields_ = [("partials", ctypes.c_void_p), ("nparts", ctypes.c_int), ("k", ctypes.c_int)]


class _ColOut(ctypes.Structure):
    """mirror of ov3d_colsum_out"""
    _fields_ = [("dst", ctypes.c_void_p), ("first_seg", ctypes.c_int), ("nseg", ctypes.c_int)]


def defer_norm_grads(partials, nparts, C, slots):
    """queue LayerNorm parameter gradients: slots [(k, param)], column block k of the
    (nparts, 4, C) resnorm backward partials is param's gradient (summed with the blocks of
    the other calls that use the same param, in backward order)."""
    _ensure_flush()
    _PENDING_COLS.append((partials, nparts, C, [(k, p) for k, p in slots]))


def _flush_norm_grads():
    from . import _native
    cols = list(_PENDING_COLS)
    _PENDING_COLS.clear()
    if not cols:
        return
    by_c = {}
    for partials, nparts, C, slots in cols:
        outs = by_c.setdefault(C, {})
        for k, p in slots:
            outs.setdefault(id(p), [p, []])[1].append((partials, nparts, k))
    for C, outs in by_c.items():
        entries = list(outs.values())
        dev = entries[0][0].device
        flat = torch.empty(len(entries) * C, dtype=torch.float32, device=dev)
        segs, outa = [], []
        for i, (p, sl) in enumerate(entries):
            outa.append(_ColOut(flat[i * C:].data_ptr(), len(segs), len(sl)))
            segs += [_ColSeg(t.data_ptr(), n, k) for t, n, k in sl]
        sa = (_ColSeg * len(segs))(*segs)
        oa = (_ColOut * len(outa))(*outa)
        _native.call("ov3d_colsum_group", ctypes.addressof(sa), len(segs), ctypes.addressof(oa),
                     len(outa), C, like=flat)
        with torch.no_grad():
            for i, (p, _) in enumerate(entries):
                g = flat[i * C:(i + 1) * C].view(p.shape)
                if p.grad is None:
                    p.grad = g
                else:
                    p.grad.add_(g)


class _WgProblem(ctypes.Structure):
    """mirror of ov3d_wgrad_problem (include/ov3d.h)"""
    _fields_ = [("dy", ctypes.c_void_p), ("ldy", ctypes.c_longlong), ("x", ctypes.c_void_p),
                ("ldx", ctypes.c_longlong), ("R", ctypes.c_int), ("N", ctypes.c_int),
                ("K", ctypes.c_int), ("nsplit", ctypes.c_int), ("dW", ctypes.c_void_p),
                ("ldw", ctypes.c_longlong), ("db", ctypes.c_void_p)]


def _leaf_param(w):
    """the fp32 leaf parameter w is (or fully aliases as a contiguous view), else None"""
    if w is None:
        return None
    base = w if w._base is None else w._base
    if not (base.is_leaf and base.requires_grad and base.dtype == torch.float32 and base.is_cuda):
        return None
    if w is not base and not (w.is_contiguous() and w.numel() == base.numel()
                              and w.data_ptr() == base.data_ptr()):
        return None
    return base


def can_defer(x, w, b=None):
    """x: the saved bf16 input rows (dy is cast to x's dtype and made row-contiguous)"""
    return (DEFER_WGRAD and not torch.is_grad_enabled() and x.is_cuda
            and x.dtype == torch.bfloat16 and x.dim() == 2 and x.stride(1) == 1
            and _leaf_param(w) is not None and (b is None or _leaf_param(b) is not None))


def defer_weight_grad(dy, x, w, b=None, rows=None, bn=None):
    """queue dW = dy^T x (+ db = sum dy) for parameter w (and bias b); rows=(r0, r1): the
    block of w's rows this pair produces (nn.MultiheadAttention in_proj); bn=(scale, shift):
    the input is relu(x * scale + shift) (its own ov3d_wgrad_bn launch)."""
    _ensure_flush()
    _PENDING.append((dy, x, _leaf_param(w), w.shape, _leaf_param(b) if b is not None else None,
                     rows, bn))


def flush_weight_grads():
    """run every queued weight gradient in one grouped launch and store them as .grad"""
    from . import _native
    _QUEUED[0] = False
    _flush_norm_grads()
    items = list(_PENDING)
    _PENDING.clear()
    if not items:
        return
    bufs = {}      # id(param) -> [param, fp32 buffer, covered rows]
    probs = []

    def buf(param):
        e = bufs.get(id(param))
        if e is None:
            e = [param, None, 0]
            bufs[id(param)] = e
        return e

    for dy, x, wp, wshape, bp, rows, _ in items:
        r0, r1 = rows if rows is not None else (0, wshape[0])
        buf(wp)[2] += r1 - r0
        if bp is not None:
            buf(bp)[2] += r1 - r0
    for e in bufs.values():
        full = e[2] == e[0].shape[0]
        e[1] = (torch.empty if full else torch.zeros)(e[0].shape, dtype=torch.float32,
                                                       device=e[0].device)
    for dy, x, wp, wshape, bp, rows, bn in items:
        R, N = dy.shape
        K = x.shape[1]
        r0, r1 = rows if rows is not None else (0, wshape[0])
        dw = bufs[id(wp)][1].view(wshape)[r0:r1].reshape(r1 - r0, K)
        db = bufs[id(bp)][1][r0:r1] if bp is not None else None
        if R >= WGRAD_SINGLE_MIN_R or bn is not None:
            # long problems (the masked encoder's interim SA, R = 2^18) run on their own
            # launch: the grouped stream-K split gives them hundreds of partial slots
            # (tools/wgrad_big.py: 104 vs 140 us at R = 2^18, N = K = 256)
            fused_weight_grad(dy, x, bias=db is not None, out_w=dw, out_b=db, bn=bn)
            continue
        probs.append(_WgProblem(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), R, N, K,
                                _wg_group_splits(R), dw.data_ptr(), dw.stride(0),
                                db.data_ptr() if db is not None else None))
    if not probs:
        _assign_grads(bufs)
        return
    arr = (_WgProblem * len(probs))(*probs)
    lib = _native.load()
    ws_n = lib.ov3d_wgrad_group_workspace(ctypes.addressof(arr), len(probs))
    dev = items[0][0].device
    ws = torch.empty((max(ws_n, 1),), dtype=torch.float32, device=dev)
    _native.call("ov3d_wgrad_group", ctypes.addressof(arr), len(probs), ws, like=ws)
    _assign_grads(bufs)


def _assign_grads(bufs):
    with torch.no_grad():
        for param, g, _ in bufs.values():
            if param.grad is None:
                param.grad = g
            else:
                param.grad.add_(g)


def weight_grad(dy, x, out=None):
    """dy (R, Cout), x (R, Cin) -> dy^T x (Cout, Cin) in fp32, split-K over R
    (written into `out`, a contiguous fp32 (Cout, Cin) tensor, when given)."""
    R, cout = dy.shape
    cin = x.shape[1]
    nc = _chunks(R, cout, cin)
    if nc == 1:
        g = _bmm_f32(dy.t()[None], x[None])[0].float()
        return g if out is None else out.copy_(g)
    part = _bmm_f32(dy.view(nc, R // nc, cout).transpose(1, 2), x.view(nc, R // nc, cin))
    return torch.sum(part, dim=0, dtype=torch.float32, out=out)


# bf16 copies of the fp32 parameters used under autocast.  Casting per call costs a kernel
# per weight and bias per step (~300 launches); instead every stale copy is refreshed with
# ONE multi-tensor copy the first time a parameter changed by the optimizer (its version
# counter moved) is used.  Disabled while a hipGraph is captured (graphs.py), where a host
# side version check would not be replayed.
SHADOW_CACHE = True
_SHADOWS = {}   # id(base parameter) -> [weakref(base), bf16 copy, version copied]


def refresh_shadows(force=False):
    """Re-copy every stale (or, with force, every) registered parameter in one multi-tensor
    copy.  A captured step graph calls this with force=True at its start."""
    dead = [k for k, e in _SHADOWS.items() if e[0]() is None]
    for k in dead:
        del _SHADOWS[k]
    stale = [e for e in _SHADOWS.values() if force or e[2] != e[0]()._version]
    if stale:
        with torch.no_grad():
            torch._foreach_copy_([e[1] for e in stale], [e[0]() for e in stale])
        for e in stale:
            e[2] = e[0]()._version


def shadow_of(p):
    """the registered bf16 copy of parameter p (or None)"""
    e = _SHADOWS.get(id(p))
    return e[1] if e is not None and e[0]() is p else None


def mark_shadow_fresh(p):
    """p's bf16 copy was rewritten together with p (optim.FusedAdamW)"""
    e = _SHADOWS.get(id(p))
    if e is not None and e[0]() is p:
        e[2] = p._version


def register_shadow(p, view):
    """make `view` (bf16, p's shape, e.g. a slice of a shared storage) p's refreshed bf16
    copy: FusedAdamW rewrites it with p, refresh_shadows() re-copies it when stale"""
    e = _SHADOWS.get(id(p))
    if e is not None and e[0]() is p and e[1].data_ptr() == view.data_ptr():
        return
    _SHADOWS[id(p)] = [weakref.ref(p), view, -1]


def ensure_fresh(params):
    """re-copy the stale registered shadows if one of `params` changed (not during capture)"""
    if torch.cuda.is_current_stream_capturing():
        return
    for p in params:
        e = _SHADOWS.get(id(p))
        if e is not None and e[0]() is p and e[2] != p._version:
            refresh_shadows()
            return


def cast_param(w, dt):
    """w (a parameter or a view of one) as `dt`, from the shared refreshed copies."""
    if w is None or w.dtype == dt:
        return w
    base = w if w._base is None else w._base
    if not (SHADOW_CACHE and w.is_cuda and base.is_leaf and base.requires_grad
            and base.dtype == torch.float32 and dt == torch.bfloat16):
        return w.to(dt)
    e = _SHADOWS.get(id(base))
    if e is None or e[0]() is not base:
        e = [weakref.ref(base), torch.empty_like(base, dtype=dt), -1]
        _SHADOWS[id(base)] = e
    if e[2] != base._version and not torch.cuda.is_current_stream_capturing():
        refresh_shadows()
    sh = e[1]
    if w is base:
        return sh
    return sh.as_strided(w.size(), w.stride(), w.storage_offset() - base.storage_offset())


class _RowsLinear(Function):
    @staticmethod
    def forward(ctx, x, w, b):
        dt = torch.get_autocast_dtype("cuda") if (x.is_cuda and torch.is_autocast_enabled("cuda")) \
            else x.dtype
        xc, wc = x.to(dt), cast_param(w, dt)
        with torch.autocast("cuda", enabled=False):
            y = _linear(xc, wc, cast_param(b, dt))   # bias in the GEMM epilogue
        ctx.save_for_backward(xc, wc)
        ctx.meta = (x.dtype, w.dtype, b is not None)
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        xdt, wdt, has_b = ctx.meta
        dy = dy.to(xc.dtype).contiguous()
        with torch.autocast("cuda", enabled=False):
            dx = _dgrad(dy, wc).to(xdt) if ctx.needs_input_grad[0] else None
            want_b = has_b and ctx.needs_input_grad[2]
            w, b = ctx.params
            if ctx.needs_input_grad[1] and can_defer(xc, w, b if want_b else None):
                defer_weight_grad(dy, xc, w, b if want_b else None)
                return dx, None, None
            if ctx.needs_input_grad[1] and _fused_ok(dy, xc):
                dw, db = fused_weight_grad(dy, xc, bias=want_b)
                dw = dw.to(wdt)
                db = db.to(wdt) if want_b else None
            else:
                dw = weight_grad(dy, xc).to(wdt) if ctx.needs_input_grad[1] else None
                db = torch.sum(dy, dim=0, dtype=torch.float32).to(wdt) if want_b else None
        return dx, dw, db


class _RowsLinearPadK(Function):
    """y = x[:, :K] W^T (+ b) for bf16 rows x (R, Kp) whose columns K .. Kp-1 are zero (Kp a
    multiple of 8, K = W's input width): the GEMM runs on the zero-padded weight (aligned K, the
    interim SA's 259 -> 264), dW = dy^T x[:, :K] comes from the strided rows directly (deferred
    like the other weight gradients), dx is (R, Kp) with zero pad columns."""

    @staticmethod
    def forward(ctx, x, w, b):
        bf = torch.bfloat16
        K, Kp = w.shape[1], x.shape[1]
        wc = cast_param(w, bf)
        wp = torch.nn.functional.pad(wc, (0, Kp - K))
        with torch.autocast("cuda", enabled=False):
            y = _linear(x, wp, cast_param(b, bf))
        ctx.save_for_backward(x, wp)
        ctx.meta = (w.dtype, b is not None, K)
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wp = ctx.saved_tensors
        wdt, has_b, K = ctx.meta
        w, b = ctx.params
        dy = dy.to(torch.bfloat16).contiguous()
        with torch.autocast("cuda", enabled=False):
            dx = _dgrad(dy, wp) if ctx.needs_input_grad[0] else None
            xk = x[:, :K]
            dw, db = linear_weight_grads(dy, xk, w, b, ctx.needs_input_grad[1],
                                         has_b and ctx.needs_input_grad[2])
        return dx, dw, db


def rows_linear_padk(x, w, b=None):
    """rows_linear for bf16 rows with zero-padded columns beyond W's input width"""
    return _RowsLinearPadK.apply(x, w, b)


def rows_linear(x, w, b=None):
    """y = x W^T (+ b) for x (..., Cin); split-K dW on the ROCm device, plain F.linear on CPU."""
    if not x.is_cuda:
        return torch.nn.functional.linear(x, w, b)
    shape = x.shape
    y = _RowsLinear.apply(x.reshape(-1, shape[-1]), w, b)
    return y.view(*shape[:-1], w.shape[0])


class _InProj(Function):
    """Row blocks of one (3E, E) projection applied to different inputs:
    y_g = x_g W[r0:r1]^T + b[r0:r1] (nn.MultiheadAttention's in_proj for self / cross
    attention).  The backward writes each block's weight / bias gradient straight into
    ONE (3E, E) / (3E,) gradient, instead of autograd's slice-backward (zero-fill the
    full-size gradient, copy the block in, accumulate the three) per block."""

    @staticmethod
    def forward(ctx, w, b, spec, *xs):
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else xs[0].dtype
        wc, bc = cast_param(w, dt), cast_param(b, dt)
        outs, saved = [], []
        with torch.autocast("cuda", enabled=False):
            xcs = [x.reshape(-1, x.shape[-1]).to(dt) for x in xs]
            if _group_ok([(xc, wc[r0:r1]) for xc, (r0, r1) in zip(xcs, spec)], True):
                ys = rows_gemm_group([(xc, wc[r0:r1], bc[r0:r1] if bc is not None else None)
                                      for xc, (r0, r1) in zip(xcs, spec)], trans_b=True)
            else:
                ys = [_linear(xc, wc[r0:r1], bc[r0:r1] if bc is not None else None)
                      for xc, (r0, r1) in zip(xcs, spec)]
            for x, xc, y, (r0, r1) in zip(xs, xcs, ys, spec):
                outs.append(y.view(*x.shape[:-1], r1 - r0))
                saved.append(xc)
        ctx.save_for_backward(wc, *saved)
        ctx.meta = (spec, w.dtype, b is not None, tuple(x.dtype for x in xs),
                    tuple(x.shape for x in xs))
        ctx.params = (w, b)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *dys):
        wc, *xcs = ctx.saved_tensors
        spec, wdt, has_b, xdts, xshapes = ctx.meta
        wp, bp = ctx.params
        want_b = has_b and ctx.needs_input_grad[1]
        defer = ctx.needs_input_grad[0] and all(can_defer(xc, wp, bp if want_b else None)
                                                for xc in xcs)
        full = sum(r1 - r0 for r0, r1 in spec) == wc.shape[0]   # else zero the other rows
        alloc = torch.empty if full else torch.zeros
        dw = alloc(wc.shape, dtype=torch.float32, device=wc.device) \
            if ctx.needs_input_grad[0] and not defer else None
        db = alloc(wc.shape[0], dtype=torch.float32, device=wc.device) \
            if want_b and not defer else None
        dxs = []
        with torch.autocast("cuda", enabled=False):
            dys = [(torch.zeros(xc.shape[0], r1 - r0, dtype=xc.dtype, device=xc.device)
                    if dy is None else dy.reshape(-1, r1 - r0).to(xc.dtype).contiguous())
                   for dy, xc, (r0, r1) in zip(dys, xcs, spec)]
            want = [i for i in range(len(dys)) if ctx.needs_input_grad[3 + i]]
            pairs = [(dys[i], wc[spec[i][0]:spec[i][1]]) for i in want]
            dx_all = [None] * len(dys)
            if _group_ok(pairs, False):   # the input gradients in one launch
                for i, d in zip(want, rows_gemm_group([(a, w, None) for a, w in pairs],
                                                      trans_b=False)):
                    dx_all[i] = d
            for i, (dy, xc, (r0, r1)) in enumerate(zip(dys, xcs, spec)):
                if ctx.needs_input_grad[3 + i]:
                    d = dx_all[i] if dx_all[i] is not None else _dgrad(dy, wc[r0:r1])
                    dxs.append(d.to(xdts[i]).view(xshapes[i]))
                else:
                    dxs.append(None)
                if defer:
                    defer_weight_grad(dy, xc, wp, bp if want_b else None, rows=(r0, r1))
                    continue
                if dw is not None and _fused_ok(dy, xc):
                    fused_weight_grad(dy, xc, bias=db is not None, out_w=dw[r0:r1],
                                      out_b=db[r0:r1] if db is not None else None)
                    continue
                if dw is not None:
                    weight_grad(dy, xc, out=dw[r0:r1])
                if db is not None:
                    torch.sum(dy, dim=0, dtype=torch.float32, out=db[r0:r1])
        return (dw.to(wdt) if dw is not None else None,
                db.to(wdt) if db is not None else None, None, *dxs)


def in_projection(w, b, groups):
    """groups: sequence of (x, r0, r1) -> tuple of x W[r0:r1]^T + b[r0:r1]."""
    xs = [g[0] for g in groups]
    if not xs[0].is_cuda:
        return tuple(torch.nn.functional.linear(x, w[r0:r1], b[r0:r1] if b is not None else None)
                     for x, r0, r1 in groups)
    spec = tuple((r0, r1) for _, r0, r1 in groups)
    return _InProj.apply(w, b, spec, *xs)
