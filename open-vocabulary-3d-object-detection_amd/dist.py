"""Distributed helpers (API mirror of reference utils/dist.py:8-176) on
torch.distributed; on ROCm the "nccl" backend is RCCL over xGMI.

Same function names and semantics as the reference, plus
``all_reduce_coalesced`` (one collective for many scalars: the reference issues
one all-reduce for num_boxes, one for the loss and one for the stacked loss
dict every step, criterion.py:425 and engine.py:104-105).  One process per GPU;
the rendezvous comes from the environment (torchrun) or ``init_distributed``.
"""
import os
import pickle

import torch
import torch.distributed as dist


def is_distributed():
    return dist.is_available() and dist.is_initialized()


def get_rank():
    return dist.get_rank() if is_distributed() else 0


def is_primary():
    return get_rank() == 0


def get_world_size():
    return dist.get_world_size() if is_distributed() else 1


def barrier():
    if is_distributed():
        dist.barrier()


def setup_print_for_distributed(is_primary_rank):
    import builtins
    builtin_print = builtins.print

    def _print(*args, **kwargs):
        force = kwargs.pop("force", False)
        if is_primary_rank or force:
            builtin_print(*args, **kwargs)

    builtins.print = _print


def init_distributed(gpu_id, global_rank, world_size, dist_url, dist_backend):
    """reference dist.py:51-64 (dist_url e.g. tcp://127.0.0.1:12345 or env://)."""
    if torch.cuda.is_available() and dist_backend == "nccl":
        torch.cuda.set_device(gpu_id)
        capture_safe_env()
    dist.init_process_group(backend=dist_backend, init_method=dist_url, world_size=world_size,
                            rank=global_rank)
    dist.barrier()
    setup_print_for_distributed(is_primary())


def capture_safe_env():
    """Process-group settings for collectives captured in a hipGraph, set before the group is
    created.  ProcessGroupNCCL recycles the events of finished works (its event cache): an
    event of an eager work (graph warm-up) still on the watchdog's list could be handed to a
    work recorded during capture, and the watchdog's query of it then aborts the process
    ("operation not permitted on an event last recorded in a capturing stream").  Without the
    cache every work owns its events.  Forced, not defaulted: an environment that switches the
    cache on would re-arm the abort, so it is overridden (with a warning)."""
    prev = os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE")
    if prev not in (None, "0"):
        import warnings
        warnings.warn(f"TORCH_NCCL_CUDA_EVENT_CACHE={prev} overridden to 0: the captured step's "
                      "collectives need every work to own its events (dist.capture_safe_env)")
    os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] = "0"


_DEDICATED = {}


def dedicated_stream(device, role):
    """The process's stream for `role` on `device`: "eager" (StepGraph's warm-up, which issues
    eager collectives), "capture" (the stream a step graph is captured on), "bucket_eager" /
    "bucket_capture" (GradBuckets' side stream outside / inside a capture).

    Why (round 6, tools/pg_capture_probe.py on the GPU): a blocking (async_op=False) collective
    runs on the CURRENT stream and ProcessGroupNCCL records the work's end event there; the
    work stays on the group's watchdog list until a watchdog pass (~100 ms apart) sees the event
    complete.  If that stream joins a graph capture before that pass, HIP refuses the query
    (hipErrorCapturedEvent: "operation not permitted on an event last recorded in a capturing
    stream"), the watchdog rethrows and the process aborts.  Round 5's abort was exactly this:
    GradBuckets' one side stream carried the warm-up's eager bucket all-reduce and then joined
    the capture.  The probe aborts deterministically when eager works are issued from the stream
    that is then captured (whatever group the captured collective uses) and passes when they
    are issued from another stream.  So streams are dedicated by role: a stream that carried an
    eager collective never joins a capture.  They are HIP streams of their own
    (_native.stream_create), not torch.cuda.Stream() pool streams, which are recycled (32 per
    priority) and could alias across roles."""
    if role not in ("eager", "capture", "bucket_eager", "bucket_capture"):
        raise ValueError(f"dedicated_stream: unknown role {role!r}")
    device = torch.device(device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (device.index, role)
    s = _DEDICATED.get(key)
    if s is None:
        from . import _native
        s = _DEDICATED[key] = _native.stream_create(device)
    return s


def init_from_env(backend=None):
    """torchrun-style init (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* in the env)."""
    if is_distributed():
        return get_rank(), get_world_size(), int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            capture_safe_env()
        dist.init_process_group(backend=backend, init_method="env://", world_size=world, rank=rank)
    return rank, world, local


def all_reduce_sum(tensor):
    if not is_distributed():
        return tensor
    squeeze = tensor.ndim == 0
    if squeeze:
        tensor = tensor[None]
    dist.all_reduce(tensor)
    return tensor.squeeze(0) if squeeze else tensor


def all_reduce_average(tensor):
    return all_reduce_sum(tensor) / get_world_size()


def all_reduce_coalesced(tensors, average=True):
    """All-reduce a list of scalar / small tensors with ONE collective."""
    if not is_distributed():
        return list(tensors)
    flat = torch.cat([t.detach().reshape(-1).float() for t in tensors])
    dist.all_reduce(flat)
    if average:
        flat /= get_world_size()
    out, off = [], 0
    for t in tensors:
        n = t.numel()
        out.append(flat[off: off + n].view(t.shape))
        off += n
    return out


def reduce_dict(input_dict, average=True):
    """reference dist.py:82-108: sorted keys, one stacked all-reduce."""
    if get_world_size() < 2:
        return input_dict
    with torch.no_grad():
        names = sorted(input_dict.keys())
        values = torch.stack([input_dict[k] for k in names], dim=0)
        dist.all_reduce(values)
        if average:
            values /= get_world_size()
        return {k: v for k, v in zip(names, values)}


def all_gather_pickle(data, device):
    world = get_world_size()
    if world == 1:
        return [data]
    buf = torch.frombuffer(bytearray(pickle.dumps(data)), dtype=torch.uint8).to(device)
    size = torch.tensor([buf.numel()], device=device)
    sizes = [torch.zeros_like(size) for _ in range(world)]
    dist.all_gather(sizes, size)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    if buf.numel() < mx:
        buf = torch.cat([buf, torch.zeros(mx - buf.numel(), dtype=torch.uint8, device=device)])
    bufs = [torch.empty((mx,), dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(bufs, buf)
    return [pickle.loads(b.cpu().numpy().tobytes()[:s]) for b, s in zip(bufs, sizes)]


def all_gather_dict(data):
    if not isinstance(data, dict):
        raise TypeError("all_gather_dict expects a dict of tensors")
    out = {}
    for k, v in data.items():
        if isinstance(v, torch.Tensor):
            if is_distributed():
                v = v.contiguous()
                parts = [torch.empty_like(v) for _ in range(get_world_size())]
                dist.all_gather(parts, v)
                v = torch.cat(parts, dim=0)
            out[k] = v
    return out


class _SyncBNRows(torch.autograd.Function):
    """SyncBatchNorm over the rows of (R, C) on the host path (torch ops; the reference wraps
    the model with convert_sync_batchnorm, main.py:427-431).  The same arithmetic as the
    fused HIP BN launches (sa_fused.py / heads.py): float64 per-rank sums (Σx, Σx², R) and
    backward sums (Σdy, Σdy·x̂), ONE all-reduce each way over `group`, statistics with the
    global count; the weight / bias gradients stay rank-local (torch's SyncBatchNorm
    semantics: DDP averages them with the other gradients).  torch's SyncBatchNorm runs on
    GPU only; this keeps the CPU world>1 path (gloo tests) on the same semantics."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, group):
        xd = x.double()
        R, C = x.shape
        tot = torch.cat([xd.sum(0), (xd * xd).sum(0), xd.new_tensor([float(R)])])
        dist.all_reduce(tot, group=group)
        n = tot[2 * C]
        mean = tot[:C] / n
        var = (tot[C: 2 * C] / n - mean * mean).clamp_min(0)
        invstd = torch.rsqrt(var + eps)
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(1 - momentum).add_(momentum * mean.to(running_mean.dtype))
                running_var.mul_(1 - momentum).add_(
                    momentum * (var * n / (n - 1)).to(running_var.dtype))
        xhat = (xd - mean) * invstd
        y = xhat
        if weight is not None:
            y = y * weight.double()
        if bias is not None:
            y = y + bias.double()
        ctx.save_for_backward(xhat, weight, invstd, n)
        ctx.group = group
        ctx.bias_dtype = None if bias is None else bias.dtype
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        xhat, weight, invstd, n = ctx.saved_tensors
        dyd = dy.double()
        C = xhat.shape[1]
        s_dy = dyd.sum(0)
        s_dyx = (dyd * xhat).sum(0)
        tot = torch.cat([s_dy, s_dyx])
        dist.all_reduce(tot, group=ctx.group)
        scale = invstd if weight is None else weight.double() * invstd
        dx = scale * (dyd - tot[:C] / n - xhat * (tot[C:] / n))
        dw = None if weight is None else s_dyx.to(weight.dtype)
        db = None if ctx.bias_dtype is None else s_dy.to(ctx.bias_dtype)
        return dx.to(dy.dtype), dw, db, None, None, None, None, None


def sync_batch_norm_rows(bn, x):
    """train-mode SyncBatchNorm `bn` over rows x (R, C) across bn.process_group (host path)"""
    group = bn.process_group if bn.process_group is not None else dist.group.WORLD
    momentum = bn.momentum
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
        if momentum is None:  # torch's cumulative moving average (_BatchNorm.forward)
            momentum = 1.0 / float(bn.num_batches_tracked)
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return _SyncBNRows.apply(x, bn.weight, bn.bias, rm, rv,
                             momentum if momentum is not None else 0.0, bn.eps, group)


class GradBuckets:
    """The data-parallel gradient mean (DDP's, main.py:427-431) in buckets that start while
    the backward still runs.

    ``buckets``: disjoint parameter lists in launch order (Model3DETR.dp_buckets: the decoder
    side, whose gradients are final once the backward reaches the encoder output, then the
    encoder side).  Every parameter has a fixed view in ONE flat fp32 buffer (static for a
    captured step), a bucket's views are contiguous.  ``launch(i)`` copies bucket i's
    gradients into its views (one launch on the GPU) and starts ONE all-reduce (sum) of that
    region on ``group`` — a process group of its own (its own RCCL communicator), so the
    SyncBatchNorm all-reduces the encoder / SA backward issues on the BN's group are not
    queued behind it.  On the GPU the collective is issued from a side stream that first waits
    for the copy (a plain blocking-call all-reduce there: inside a capture it enqueues no work
    on the watchdog's list); the current stream runs on.  The side stream is
    ``dedicated_stream(.., "bucket_eager")`` outside a capture and ``"bucket_capture"`` inside
    one, so no stream that carried an eager bucket all-reduce joins a capture.  On the CPU
    (gloo) it is an ``async_op`` work.  ``finish()`` launches what is left, joins (the current
    stream waits for the side stream: capturable) and returns {id(param): summed gradient
    view} (the caller divides by the world size).  A parameter without a gradient contributes
    zeros."""

    def __init__(self, buckets, group=None):
        self.buckets = [list(b) for b in buckets]
        ids = [id(p) for b in self.buckets for p in b]
        if len(ids) != len(set(ids)):
            raise ValueError("GradBuckets: a parameter is in two buckets")
        self.group = group
        self.stream = None
        self.flat = None
        self.views = {}
        self.regions = []
        self._works = {}

    def _build(self, device):
        n = sum(p.numel() for b in self.buckets for p in b)
        self.flat = torch.zeros(n, dtype=torch.float32, device=device)
        o = 0
        for b in self.buckets:
            o0 = o
            for p in b:
                self.views[id(p)] = self.flat[o:o + p.numel()].view(p.shape)
                o += p.numel()
            self.regions.append(self.flat[o0:o])

    def launch(self, i):
        if i in self._works or not self.buckets[i]:
            return
        b = self.buckets[i]
        if self.flat is None:
            self._build(b[0].device)
        dst, src = [], []
        for p in b:
            v = self.views[id(p)]
            if p.grad is None:
                v.zero_()
            else:
                dst.append(v)
                src.append(p.grad)
        if self.flat.is_cuda:
            from . import _native
            if dst:
                _native.multi_copy(dst, src)
            # inside a capture the collective goes out on a stream that never carried an eager
            # one (dedicated_stream: an eager work's end event on a capturing stream aborts the
            # watchdog)
            role = "bucket_capture" if torch.cuda.is_current_stream_capturing() else "bucket_eager"
            self.stream = dedicated_stream(self.flat.device, role)
            cur = torch.cuda.current_stream(self.flat.device)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                dist.all_reduce(self.regions[i], group=self.group)
            self._works[i] = None
            return
        for d, s in zip(dst, src):
            d.copy_(s)
        self._works[i] = dist.all_reduce(self.regions[i], group=self.group, async_op=True)

    def launched(self, i):
        return i in self._works

    def finish(self):
        for i in range(len(self.buckets)):
            self.launch(i)
        for w in self._works.values():
            if w is not None:
                w.wait()
        if self.stream is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.stream)
        self._works.clear()
        return self.views


def stage_after_encoder(model, buckets, flush=None):
    """Start bucket 0 (the decoder side, Model3DETR.dp_buckets) as soon as the backward has
    produced the encoder output's gradient: a tensor hook on that output (Model3DETR.forward,
    ``encoder_grad_hook``) runs the deferred weight gradients queued so far (gemm.py: the
    decoder's and heads') and launches the bucket's all-reduce, which then overlaps the
    encoder and SA backward (~1.5 ms of the SUN step) instead of following it."""
    if flush is None:
        from . import gemm
        flush = gemm.flush_weight_grads

    def hook():
        flush()
        if buckets is not None:   # None: the staged flush alone (single-process A/B twin)
            buckets.launch(0)
    model.encoder_grad_hook = hook
    return hook
