"""Flash attention on the HIP kernels of csrc/attn.hip (``ov3d_attn_fwd/bwd``).

Used by transformer.MultiheadAttention for the reference's nn.MultiheadAttention
core (models/transformer.py:223,271,307-308,365-372): head_dim 64, no mask, bf16
operands (autocast), fp32 softmax statistics, dropout on the attention
probabilities as nn.MultiheadAttention(dropout=...) applies it in training.

Q, K and V are passed as column ranges of their projection outputs, which keep the
reference's seq-first row layout (L, B, n*E): the kernels read (l, b, head, d) at
row l*B + b, column off + head*64 + d, so the heads are never permuted or copied;
the gradients are written into one buffer per source tensor the same way.

Dropout randomness: keep(q, k) is a counter-based hash of (step seed, call site,
b*H + h, q, k).  The forward hashes once and stores the drop bits (two 1-bit-per-pair
layouts, query-major for the dQ kernel and key-major for the dK/dV kernel: 16 + 16 MB per
encoder layer), saved on the ctx like the logsumexp; the backward reads them.  The step
seed is a device int64 advanced once per training forward (``next_step``, captured by a
hipGraph like any other kernel) and snapshotted for that forward.  The call site is fixed
per module.

Masked encoder (reference models/transformer.py:152-190): the boolean mask
``cdist(xyz, xyz) >= radius`` (True = not attended), the same for every head, reaches the
kernels as a ``PackedMask`` of 1-bit words (``pack_mask``: one launch from the distances,
no (B*H, L, L) tensor); masked keys get a -inf score in the forward and both backward
kernels.
"""
import ctypes
import itertools
import os

import torch

from . import _native

HEAD_DIM = 64
_SITES = itertools.count(1)
_SEEDS = {}     # live per-device step counter (advanced in place: graph-replay safe)
_SNAPS = {}     # per device: the snapshot the current forward's dropout masks use


# Deferred dK / dV (the decoder's cross attentions): the K / V of all layers are column blocks
# of two shared buffers whose gradient only feeds transformer._MemoryKV's backward, which
# runs after every layer's attention backward.  A layer's backward computes dQ (and D) at
# once and queues its dK / dV job here; _MemoryKV.backward launches all of them in one
# ov3d_attn_bwd_dkdv_batch call before it reads the buffers.
_KV_JOBS = {}   # id(dK buffer) -> [((B, H, Lq, Lk, p), job struct, tensors kept alive), ...]
DEFER_KV = True   # off: every call computes its dK / dV at once (tests compare the two)


class _DkdvJob(ctypes.Structure):
    """mirror of ov3d_attn_dkdv_job (include/ov3d.h)"""
    _fields_ = [("q", ctypes.c_void_p), ("sq", ctypes.c_longlong), ("k", ctypes.c_void_p),
                ("sk", ctypes.c_longlong), ("v", ctypes.c_void_p), ("sv", ctypes.c_longlong),
                ("dout", ctypes.c_void_p), ("sdo", ctypes.c_longlong), ("lse", ctypes.c_void_p),
                ("dvec", ctypes.c_void_p), ("dropbits", ctypes.c_void_p), ("dk", ctypes.c_void_p),
                ("sdk", ctypes.c_longlong), ("dv", ctypes.c_void_p), ("sdv", ctypes.c_longlong)]


def defer_kv_grads(dk_buf):
    """attention calls whose K gradient goes to `dk_buf` queue their dK / dV (see _KV_JOBS)"""
    if len(_KV_JOBS) > 16:   # forwards without a backward (eval) leave empty entries
        for key in [k for k, v in _KV_JOBS.items() if not v]:
            del _KV_JOBS[key]
    _KV_JOBS[id(dk_buf)] = []


def flush_kv_grads(dk_buf):
    """launch the queued dK / dV of the calls writing `dk_buf` (one launch per shape)"""
    jobs = _KV_JOBS.pop(id(dk_buf), None)
    if not jobs:
        return
    lib = _native.load()
    by_shape = {}
    for dims, job, keep in jobs:
        by_shape.setdefault(dims, []).append((job, keep))
    for (B, H, Lq, Lk, p), lst in by_shape.items():
        arr = (_DkdvJob * len(lst))(*[j for j, _ in lst])
        rc = lib.ov3d_attn_bwd_dkdv_batch(ctypes.addressof(arr), len(lst), B, H, Lq, Lk,
                                          HEAD_DIM ** -0.5, p, _native._stream(lst[0][1][0]))
        if rc:
            raise _native.NativeError(f"ov3d_attn_bwd_dkdv_batch failed with status {rc}")
        _native.note("ov3d_attn_bwd_dkdv_batch")


def new_site():
    return next(_SITES)


def _live(device):
    t = _SEEDS.get(device)
    if t is None:
        # drawn from torch's generator (seeded per rank by the caller, main.py:415-418), and
        # offset by the rank so data-parallel replicas never share dropout masks
        rank = torch.distributed.get_rank() if (torch.distributed.is_available()
                                                and torch.distributed.is_initialized()) else 0
        v = int(torch.randint(0, 2 ** 40, (1,), dtype=torch.int64)) + (rank << 48)
        t = torch.tensor([v], dtype=torch.int64).to(device)
        _SEEDS[device] = t
    return t


def _seed(device):
    """The seed tensor of the CURRENT forward.  Attention saves the drop bits it drew from it
    on its autograd ctx (resnorm / FFN dropout save the seed object itself), so a backward
    never reads this function: a later forward (an EMA-teacher pass,
    forward-forward-backward) takes a new snapshot and leaves the saved masks untouched."""
    s = _SNAPS.get(device)
    if s is None:
        s = _live(device).clone()
        _SNAPS[device] = s
    return s


def next_step(device):
    """Advance the dropout seed of `device` and snapshot it for this forward (two tiny
    kernels, captured by a hipGraph like any other; call once per training forward)."""
    live = _live(device)
    snap = torch.empty_like(live)
    _native.call("ov3d_seed_next", live, snap, like=live)
    _SNAPS[device] = snap


# Drop bits generated ahead of the attention forward on a side stream (ov3d_attn_dropgen): the
# hash leaves the forward's vector-issue-bound loop (encoder forward 69 -> 52 us in the step).
# Off by default: beside the pre-encoder SA the side-stream pass slowed the step 1617 -> 1548
# scenes/s (same box, tools/ab_env.sh); OV3D_ATTN_PREGEN=1 enables it.
# (device, site) -> (bits, event, dims)
PREGEN = os.environ.get("OV3D_ATTN_PREGEN", "0") == "1"
_PREGEN = {}
_SIDE = {}


def pregen_dropout(device, jobs):
    """jobs: [(site, B, H, Lq, Lk, p)] of attention forwards later in this forward pass: their
    drop bits (this forward's seed) on a side stream, joined by the forward that uses them."""
    lib = _native.load()
    cur = torch.cuda.current_stream(device)
    side = _SIDE.get(device)
    if side is None:
        side = _SIDE[device] = torch.cuda.Stream(device=device)
    seed = _seed(device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        for site, B, H, Lq, Lk, p in jobs:
            nbits = lib.ov3d_attn_dropbits_words(B, H, Lq, Lk)
            with torch.cuda.stream(cur):   # allocated on the consumer's stream
                bits = torch.empty((nbits,), dtype=torch.int32, device=device)
            bits.record_stream(side)
            _native.call("ov3d_attn_dropgen", B, H, Lq, Lk, float(p), seed, site, bits, like=bits)
            ev = torch.cuda.Event()
            ev.record(side)
            _PREGEN[(device, site)] = (bits, ev, (B, H, Lq, Lk, float(p)))


def _take_pregen(device, site, dims):
    e = _PREGEN.pop((device, site), None)
    if e is None:
        return None
    bits, ev, d = e
    if d != dims:
        return None
    torch.cuda.current_stream(device).wait_event(ev)
    return bits


def clear_pregen():
    _PREGEN.clear()


class PackedMask:
    """An attention mask shared by the heads, packed for the kernels (ov3d_attn_mask_pack):
    ``words`` int32 (ov3d_attn_maskbits_words(B, Lq, Lk),), bit set = not attended."""

    def __init__(self, words, B, Lq, Lk):
        self.words, self.B, self.Lq, self.Lk = words, B, Lq, Lk


def pack_mask(src, thr=None, squared=False):
    """(B, Lq, Lk) bool mask (True = not attended), or fp32 distances with ``thr`` (not
    attended iff d >= thr: MaskedTransformerEncoder.compute_mask) -> PackedMask.
    squared: src is cdist's matmul-form squared distances (transformer.euclid_sq), packed as
    sqrt(max(src, 0)) >= thr — cdist's own clamp and sqrt, fused."""
    B, Lq, Lk = src.shape
    _native.check_device(src, "attention mask")
    lib = _native.load()
    n = lib.ov3d_attn_maskbits_words(B, Lq, Lk)
    if n <= 0:
        raise ValueError("pack_mask: query length must be a multiple of 32")
    src = src.contiguous()
    if thr is None:
        if src.dtype != torch.bool:
            raise ValueError("pack_mask: a bool mask, or distances with a threshold")
        kind, thr = 0, 0.0
    else:
        if src.dtype != torch.float32:
            raise ValueError("pack_mask: distances must be float32")
        kind = 2 if squared else 1
    words = torch.empty((n,), dtype=torch.int32, device=src.device)
    _native.call("ov3d_attn_mask_pack", src, kind, float(thr), B, Lq, Lk, words, like=src)
    return PackedMask(words, B, Lq, Lk)


def pack_mask_points(xyz, thr):
    """(B, L, 3) points -> PackedMask of cdist(xyz, xyz) >= thr computed in the packing launch
    (kind 3): the squared distances as cdist's matmul form, bit for bit, without the (B, L, L)
    distance matrix or its fp32 GEMM (MaskedTransformerEncoder.compute_mask)."""
    B, L, _ = xyz.shape
    _native.check_device(xyz, "attention mask points")
    lib = _native.load()
    n = lib.ov3d_attn_maskbits_words(B, L, L)
    if n <= 0:
        raise ValueError("pack_mask_points: point count must be a multiple of 32")
    with torch.autocast("cuda", enabled=False):
        x = xyz.float()
        pts = torch.cat([x, x.pow(2).sum(-1, keepdim=True)], -1).contiguous()   # euclid_sq's norms
    words = torch.empty((n,), dtype=torch.int32, device=xyz.device)
    _native.call("ov3d_attn_mask_pack", pts, 3, float(thr), B, L, L, words, like=pts)
    return PackedMask(words, B, L, L)


def supported(q_src, embed_dim, num_heads, attn_mask):
    """the HIP kernels: head_dim 64, no mask or a PackedMask, query length a multiple of 32"""
    return (q_src.is_cuda and (attn_mask is None or isinstance(attn_mask, PackedMask))
            and embed_dim == num_heads * HEAD_DIM and q_src.shape[0] % 32 == 0)


def _split(Lq, Lk, BH):
    """key splits so that the grid has >= ~256 workgroups (decoder: 128 queries)."""
    force = os.environ.get("OV3D_ATTN_SPLIT")    # measurement knob (tools/attn_time.py)
    if force:
        return max(1, min(int(force), Lk // 64))
    wgs = ((Lq + 127) // 128) * BH
    n = 1
    while wgs * n < 256 and Lk // (n * 2) >= 128:
        n *= 2
    return n


def _rows(src, off, E):
    """(contiguous source, column offset) -> (data pointer, row stride) for the kernel."""
    return src.data_ptr() + off * src.element_size(), src.shape[-1]


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, dims, H, dropout_p, site, ext, mask, token, *srcs):
        (qi, qo), (ki, ko), (vi, vo) = spec
        q, k, v = srcs[qi], srcs[ki], srcs[vi]
        Lq, Lk, B = dims
        E = H * HEAD_DIM
        dev = q.device
        o = torch.empty((Lq, B, E), dtype=torch.bfloat16, device=dev)
        lse = torch.empty((B * H, Lq), dtype=torch.float32, device=dev)
        nsplit = _split(Lq, Lk, B * H)
        ws_n = _native.load().ov3d_attn_fwd_workspace(B, H, Lq, Lk, nsplit)
        ws = torch.empty((max(ws_n, 1),), dtype=torch.float32, device=dev)
        seed = _seed(dev)
        bits = _take_pregen(dev, site, (B, H, Lq, Lk, float(dropout_p))) if dropout_p > 0 else None
        fn = _native.load().ov3d_attn_fwd_pregen
        if bits is None:
            nbits = _native.load().ov3d_attn_dropbits_words(B, H, Lq, Lk) if dropout_p > 0 else 0
            bits = torch.empty((max(nbits, 1),), dtype=torch.int32, device=dev)
            fn = _native.load().ov3d_attn_fwd_masked
        qp, sq = _rows(q, qo, E)
        kp, sk = _rows(k, ko, E)
        vp, sv = _rows(v, vo, E)
        mw = mask.words if mask is not None else None
        rc = fn(qp, kp, vp, sq, sk, sv, B, H, Lq, Lk, HEAD_DIM ** -0.5, float(dropout_p),
                _native._ptr(seed), site, _native._ptr(o), E, _native._ptr(lse), _native._ptr(bits),
                _native._ptr(ws), nsplit, _native._ptr(mw) if mw is not None else 0,
                _native._stream(q))
        if rc:
            raise _native.NativeError(f"ov3d_attn_fwd failed with status {rc}")
        _native.note("ov3d_attn_fwd_pregen" if fn is _native.load().ov3d_attn_fwd_pregen
                     else "ov3d_attn_fwd_masked")
        ctx.save_for_backward(*srcs, o, lse, bits, mw)
        ctx.meta = (spec, dims, H, float(dropout_p), site, len(srcs))
        ctx.ext = ext
        return o

    @staticmethod
    def backward(ctx, do):
        spec, (Lq, Lk, B), H, p, site, n = ctx.meta
        saved = ctx.saved_tensors
        srcs, o, lse, bits, mw = saved[:n], saved[n], saved[n + 1], saved[n + 2], saved[n + 3]
        (qi, qo), (ki, ko), (vi, vo) = spec
        q, k, v = srcs[qi], srcs[ki], srcs[vi]
        E = H * HEAD_DIM
        do = do.to(torch.bfloat16).contiguous()
        ext, tok_grad = ctx.ext if ctx.ext is not None else ((None,) * n, None)
        # every column of an own source is written below; external sources (shared K / V
        # of the decoder layers, transformer.MemoryKV) get their column block written into
        # the caller's gradient buffer
        grads = [e if e is not None else torch.empty_like(s) for s, e in zip(srcs, ext)]
        dvec = torch.empty((B * H, Lq), dtype=torch.float32, device=q.device)
        nsplit = _split(Lq, Lk, B * H)
        ws_n = _native.load().ov3d_attn_fwd_workspace(B, H, Lq, Lk, nsplit)
        ws = torch.empty((max(ws_n, 1),), dtype=torch.float32, device=q.device)
        qp, sq = _rows(q, qo, E)
        kp, sk = _rows(k, ko, E)
        vp, sv = _rows(v, vo, E)
        dqp, sdq = _rows(grads[qi], qo, E)
        dkp, sdk = _rows(grads[ki], ko, E)
        dvp, sdv = _rows(grads[vi], vo, E)
        # K and V gradients into shared buffers registered for deferral: dQ now, dK / dV
        # queued for the batched launch (flush_kv_grads)
        defer = (DEFER_KV and mw is None and ext[ki] is not None and ext[vi] is not None
                 and ki != qi and vi != qi and id(ext[ki]) in _KV_JOBS)
        rc = _native.load().ov3d_attn_bwd_masked(
            qp, kp, vp, sq, sk, sv, _native._ptr(o), E, _native._ptr(do), E, _native._ptr(lse),
            B, H, Lq, Lk, HEAD_DIM ** -0.5, p, _native._ptr(bits),
            _native._ptr(dvec), dqp, sdq, 0 if defer else dkp, sdk, 0 if defer else dvp, sdv,
            _native._ptr(ws), nsplit, _native._ptr(mw) if mw is not None else 0,
            _native._stream(q))
        if rc:
            raise _native.NativeError(f"ov3d_attn_bwd failed with status {rc}")
        _native.note("ov3d_attn_bwd_masked")
        if defer:
            job = _DkdvJob(qp, sq, kp, sk, vp, sv, _native._ptr(do), E, _native._ptr(lse),
                           _native._ptr(dvec), _native._ptr(bits) if p > 0 else 0,
                           dkp, sdk, dvp, sdv)
            _KV_JOBS[id(ext[ki])].append(((B, H, Lq, Lk, p), job,
                                          (q, k, v, do, lse, dvec, bits, ext[ki], ext[vi])))
        grads = [None if e is not None else g for g, e in zip(grads, ext)]
        return (None, None, None, None, None, None, None, tok_grad, *grads)


def attention_packed(srcs, spec, Lq, Lk, num_heads, dropout_p=0.0, site=0, ext=None, mask=None):
    """Attention over column ranges of projection outputs.

    srcs: contiguous (L, B, n*E) tensors (their rows l*B + b), spec: ((src index, column
    offset) for q, for k, for v).  Every column of every source must belong to one of
    q / k / v (their gradients are written column range by column range, not zeroed).
    ext: optional (grad buffers per source or None, token, token gradient): a source with
    a buffer is shared with other calls (it may have more columns than this call reads);
    its gradient columns go into the buffer and ``token`` (an output of the producer of
    the shared sources) carries the dependency instead.  mask: optional PackedMask of shape
    (B, Lq, Lk).  -> (Lq, B, E) bf16."""
    E = num_heads * HEAD_DIM
    B = srcs[spec[0][0]].shape[1]
    bufs = ext[0] if ext is not None else (None,) * len(srcs)
    for i, s in enumerate(srcs):
        cols = sorted(off for j, off in spec if j == i)
        shared = bufs[i] is not None
        if not s.is_contiguous() or s.dim() != 3 or s.shape[1] != B or \
                (not shared and cols != list(range(0, s.shape[-1], E))) or \
                (shared and (bufs[i].shape != s.shape or any(c + E > s.shape[-1] for c in cols))):
            raise ValueError("attention_packed: sources must be contiguous (L, B, n*E) tensors "
                             "fully covered by the q / k / v column ranges")
        _native.check_device(s, "attention input")
    if mask is not None and (mask.B, mask.Lq, mask.Lk) != (B, Lq, Lk):
        raise ValueError("attention_packed: mask shape does not match (B, Lq, Lk)")
    srcs = [s if s.dtype == torch.bfloat16 else s.to(torch.bfloat16) for s in srcs]
    if ext is None:
        return _Attention.apply(tuple(spec), (Lq, Lk, B), num_heads, dropout_p, site, None, mask,
                                None, *srcs)
    bufs, token, tok_grad = ext
    return _Attention.apply(tuple(spec), (Lq, Lk, B), num_heads, dropout_p, site,
                            (tuple(bufs), tok_grad), mask, token, *srcs)


def attention(q, k, v, num_heads, dropout_p=0.0, site=0, mask=None):
    """q (Lq, B, E), k / v (Lk, B, E) -> (Lq, B, E) bf16 = softmax(q k^T / 8) v per head,
    dropout on the probabilities (separate, contiguous copies of q, k, v); mask: optional
    PackedMask (B, Lq, Lk)."""
    if k.shape[1] != q.shape[1] or v.shape[:2] != k.shape[:2]:
        raise ValueError("attention: q, k, v batch / key lengths disagree")
    srcs = [t.contiguous() for t in (q, k, v)]
    return attention_packed(srcs, ((0, 0), (1, 0), (2, 0)), q.shape[0], k.shape[0], num_heads,
                            dropout_p, site, mask=mask)
