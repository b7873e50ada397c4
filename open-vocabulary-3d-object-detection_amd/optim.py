"""AdamW with the gradient-norm clipping fused in: three HIP launches per step over all
parameter tensors (csrc/adamw.hip, ``ov3d_adamw_step``).

Reference: main.py builds ``torch.optim.AdamW(params, lr=base_lr,
weight_decay=weight_decay)``; engine.py:104-112 calls
``torch.nn.utils.clip_grad_norm_(model.parameters(), clip_gradient)`` (when > 0) and then
``optimizer.step()``.  ``FusedAdamW(params, lr, weight_decay=..., max_grad_norm=clip)``
does both in ``step()``: the clipped gradients are written back to ``p.grad`` as
clip_grad_norm_ does, ``last_grad_norm`` holds the total norm (device scalar) it returns,
and the state keeps torch's keys (``step``, ``exp_avg``, ``exp_avg_sq``).  Built with
``max_grad_norm=None`` it is a drop-in for AdamW after a separate clip_grad_norm_ call.
With ``allreduce_group`` (data parallel without DDP) the averaged, clipped gradients live
in the optimizer's flat buffer (``flat_grads()``) instead of ``p.grad``.

The bf16 copies of the parameters used by the autocast GEMMs (gemm.cast_param) are
rewritten by the same update launch, so no separate refresh copy runs.  Capturable: the
step counter and bias corrections live on the device, the per-tensor table (parameter,
moments, shadow, size, parameter group) is built by one eager step, and the gradient
addresses travel as kernel arguments of ov3d_adamw_set_grads, so a step graph carries its
own.  Each group's lr and weight decay live in a small device table (f64, as torch's
Python floats) that the update launch reads: ``sync_hyper()`` rewrites it from
``param_groups`` (step() does so itself when it runs eagerly; graphs.StepGraph calls it
before every replay), so the reference's per-iteration lr schedule (engine.py:79,
adjust_learning_rate: warmup then cosine) reaches a captured step.  Once a step has been
captured, the table and buffers are never reallocated (a change of the parameter set
raises instead of freeing memory the graph still uses).
"""
import ctypes

import torch

from . import _native
from . import gemm


class _Entry(ctypes.Structure):
    """mirror of ov3d_adamw_tensor (include/ov3d.h)"""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p),
                ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
                ("shadow", ctypes.c_void_p), ("numel", ctypes.c_longlong),
                ("group", ctypes.c_int), ("reserved", ctypes.c_int)]


class FusedAdamW(torch.optim.Optimizer):
    clips_grads = True        # step() includes clip_grad_norm_ (when max_grad_norm is set)
    writes_shadows = True     # step() refreshes gemm.py's bf16 parameter copies

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 max_grad_norm=None, allreduce_group=None, grad_buckets=None):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("FusedAdamW: invalid hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.max_grad_norm = max_grad_norm
        # data parallel without DDP (graphs.StepGraph at N > 1): the gradients are copied into
        # one flat buffer (one launch), all-reduced by ONE collective (sum) and averaged by
        # the update kernels (grad_scale = 1/world): DDP's gradient mean, main.py:427-431
        self.allreduce_group = allreduce_group
        # dist.GradBuckets: the same mean in buckets, the first one started during the backward
        # (dist.stage_after_encoder); its views replace the single flat buffer
        self.grad_buckets = grad_buckets
        if grad_buckets is not None and allreduce_group is None:
            raise ValueError("FusedAdamW: grad_buckets needs allreduce_group (the world size)")
        self.last_grad_norm = None
        self._key = None
        self._dev = None
        self._captured = False   # a graph holds the table / buffers: never reallocate them
        self._hyper = None       # device (ngroups, 2) f64 {lr, weight_decay}
        self._hyper_host = None

    def _params(self):
        out = []
        b = e = None
        for g in self.param_groups:
            if b is None:
                b, e = tuple(g["betas"]), g["eps"]
            elif tuple(g["betas"]) != b or g["eps"] != e:
                raise ValueError("FusedAdamW: betas / eps must be equal across param groups")
            for p in g["params"]:
                if p.grad is not None:
                    out.append((p, g))
        return out, b, e

    def _state(self, p, dev):
        st = self.state[p]
        if not st:
            if self._step_t is None:
                self._step_t = torch.zeros((), dtype=torch.float32, device=dev)
            st["step"] = self._step_t
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    _step_t = None

    def _table(self, items, dev):
        """entries without the gradient pointers (set per step by ov3d_adamw_set_grads)"""
        chunk = _native.load().ov3d_adamw_chunk()
        ents, blk_t, blk_c, key = [], [], [], []
        gid = {id(g): i for i, g in enumerate(self.param_groups)}
        for i, (p, g) in enumerate(items):
            if not (p.is_cuda and p.dtype == torch.float32 and p.grad.dtype == torch.float32
                    and p.is_contiguous() and p.grad.is_contiguous()
                    and p.grad.shape == p.shape):
                raise ValueError("FusedAdamW: fp32 contiguous device parameters and gradients only")
            st = self._state(p, dev)
            sh = gemm.shadow_of(p)
            n = p.numel()
            ents.append(_Entry(p.data_ptr(), 0, st["exp_avg"].data_ptr(),
                               st["exp_avg_sq"].data_ptr(), sh.data_ptr() if sh is not None else 0,
                               n, gid[id(g)], 0))
            nb = (n + chunk - 1) // chunk
            blk_t += [i] * nb
            blk_c += list(range(nb))
            key.append((p.data_ptr(), ents[-1].shadow, n, gid[id(g)]))
        return tuple(key), ents, blk_t, blk_c

    def sync_hyper(self):
        """Write every group's current lr / weight decay into the device table the update
        launch reads (stream-ordered, no host sync; only when a value changed).  Not during
        capture: call it before each replay of a captured step."""
        vals = [float(v) for g in self.param_groups for v in (g["lr"], g["weight_decay"])]
        if self._hyper is None or self._hyper.numel() != len(vals):
            if self._captured:
                raise RuntimeError("FusedAdamW: param groups changed after a step was captured")
            dev = self._dev or next(p.device for g in self.param_groups for p in g["params"])
            self._hyper = torch.empty(len(vals), dtype=torch.float64, device=dev)
            self._hyper_host = None
        if vals != self._hyper_host:
            src = torch.tensor(vals, dtype=torch.float64)
            if self._hyper.is_cuda:
                src = src.pin_memory()
            self._hyper.copy_(src, non_blocking=True)
            self._hyper_host = vals

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = [st["step"] for st in self.state.values() if "step" in st]
        if steps:
            dev = next(iter(self.state.values()))["exp_avg"].device
            self._step_t = torch.as_tensor(steps[0], dtype=torch.float32).to(dev).reshape(())
            for st in self.state.values():
                st["step"] = self._step_t
        self._key = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        items, (b1, b2), eps = self._params()
        if not items:
            return loss
        dev = items[0][0].device
        _native.check_device(items[0][0], "FusedAdamW parameters")
        key, ents, blk_t, blk_c = self._table(items, dev)
        capturing = torch.cuda.is_current_stream_capturing()
        if key != self._key or dev != self._dev:
            if capturing:
                raise RuntimeError("FusedAdamW: run one eager step before capturing a graph "
                                   "(the parameter table is built outside capture)")
            if self._captured:
                raise RuntimeError("FusedAdamW: the parameter set changed after a step was "
                                   "captured (the graph still uses the old table)")
            raw = (_Entry * len(ents))(*ents)
            nbytes = ctypes.sizeof(raw)
            host = torch.empty(nbytes + 8 * len(blk_t), dtype=torch.uint8)
            ctypes.memmove(host.data_ptr(), ctypes.addressof(raw), nbytes)
            host[nbytes:].view(torch.int32).copy_(torch.tensor(blk_t + blk_c, dtype=torch.int32))
            self._buf = host.to(dev)
            self._nbytes, self._nblocks, self._ntensors = nbytes, len(blk_t), len(ents)
            self._partials = torch.empty(len(blk_t), dtype=torch.float64, device=dev)
            self._coefs = torch.empty(4, dtype=torch.float64, device=dev)
            self._key, self._dev = key, dev
        scale = 1.0
        if self.grad_buckets is not None:
            import torch.distributed as dist
            views = self.grad_buckets.finish()
            missing = [p for p, _ in items if id(p) not in views]
            if missing:
                raise ValueError("FusedAdamW: a parameter with a gradient is in no bucket")
            self._flat_views = [views[id(p)] for p, _ in items]
            grad_src = self._flat_views
            scale = 1.0 / dist.get_world_size(self.allreduce_group)
        elif self.allreduce_group is not None:
            import torch.distributed as dist
            if getattr(self, "_flat", None) is None or self._flat_key != key:
                if capturing or self._captured:
                    raise RuntimeError("FusedAdamW: run one eager step before capturing a graph "
                                       "(and never change the parameter set after it)")
                self._flat = torch.empty(sum(p.numel() for p, _ in items), dtype=torch.float32,
                                         device=dev)
                self._flat_key = key
                views, o = [], 0
                for p, _ in items:
                    views.append(self._flat[o:o + p.numel()].view(p.shape))
                    o += p.numel()
                self._flat_views = views
            _native.multi_copy(self._flat_views, [p.grad for p, _ in items])
            dist.all_reduce(self._flat, group=self.allreduce_group)
            grad_src = self._flat_views
            scale = 1.0 / dist.get_world_size(self.allreduce_group)
        else:
            grad_src = [p.grad for p, _ in items]
        if capturing:
            self._captured = True
            if self._hyper is None:
                raise RuntimeError("FusedAdamW: run one eager step before capturing a graph")
        else:
            self.sync_hyper()
        grads = (ctypes.c_void_p * len(items))(*[g.data_ptr() for g in grad_src])
        _native.call("ov3d_adamw_set_grads", self._buf, len(items), ctypes.addressof(grads),
                     like=self._buf)
        idx = self._buf[self._nbytes:].view(torch.int32)
        clip = float(self.max_grad_norm) if self.max_grad_norm and self.max_grad_norm > 0 else 0.0
        _native.call("ov3d_adamw_step", self._buf, idx, idx[self._nblocks:], self._nblocks,
                     self._partials, clip, self._step_t, float(b1), float(b2), float(eps),
                     self._coefs, 1, float(scale), self._hyper, like=self._buf)
        self.last_grad_norm = self._coefs[3]   # fp64 view (no launch)
        for p, _ in items:
            torch.autograd.graph.increment_version(p)
            if clip and self.allreduce_group is None:
                torch.autograd.graph.increment_version(p.grad)
            gemm.mark_shadow_fresh(p)
        return loss

    def flat_grads(self):
        """the averaged, clipped gradients of the last all-reduced step, one view per parameter"""
        return getattr(self, "_flat_views", None)
