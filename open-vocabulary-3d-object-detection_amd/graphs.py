"""hipGraph capture of the 3DETR training step (single process).

``StepGraph`` captures the WHOLE step — forward, set criterion (device Hungarian,
no host sync), backward, gradient clipping and the fused AdamW update — once, and
replays it per batch: one graph launch instead of ~2400 kernel launches from
Python.  This is possible because nothing in the step synchronises with the host
(tests/test_model_gpu.py::test_step_has_no_host_sync_and_matcher_equals_scipy).
The batch is copied into the graph's static input buffers before each replay.

``GraphedModel`` (older, forward/backward only via make_graphed_callables) is
kept for callers that run their own criterion / optimizer eagerly.

---

A training step launches ~3000 small kernels; eager PyTorch pays ~2-4 us of host
time per launch, so the 8-scene step is host-bound in places.  The model's
forward and backward have no host synchronisation (the HIP sampling / grouping
kernels are plain stream launches, grouping's backward memset is a memset node),
so both are captured once with ``torch.cuda.make_graphed_callables`` and
replayed every step; the set criterion (which must sync for the host Hungarian
solver) and the optimizer stay eager between the two replays.  Results are the
eager results (same kernels, same order); dropout draws from the graph-safe
Philox generator.
"""
import os

import torch
import torch.nn as nn


OUT_KEYS = ("visual_embeds", "sem_cls_logits", "center_normalized", "center_unnormalized",
            "size_normalized", "size_unnormalized", "angle_logits", "angle_residual",
            "angle_residual_normalized", "angle_continuous", "objectness_prob", "sem_cls_prob",
            "box_corners")
IN_KEYS = ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")


class _Flat(nn.Module):
    def __init__(self, model, amp_dtype):
        super().__init__()
        self.model = model
        self.amp_dtype = amp_dtype

    def forward(self, pc, dmin, dmax):
        with torch.autocast("cuda", dtype=self.amp_dtype or torch.float32,
                            enabled=self.amp_dtype is not None, cache_enabled=False):
            out = self.model({"point_clouds": pc, "point_cloud_dims_min": dmin,
                              "point_cloud_dims_max": dmax})
        layers = [out["outputs"]] + list(out["aux_outputs"])
        return tuple(lay[k] for lay in layers for k in OUT_KEYS)


class GraphedModel:
    """Callable with the Model3DETR.forward contract, replaying captured graphs."""

    def __init__(self, model, sample_inputs, amp_dtype=torch.bfloat16, warmup_iters=3):
        self.model = model
        self.flat = _Flat(model, amp_dtype)
        args = tuple(sample_inputs[k] for k in IN_KEYS)
        from . import gemm
        # per-call casts inside the captured graph (see gemm.cast_param); the process-wide
        # cache is restored afterwards (the replays do not run the Python cast path)
        saved, gemm.SHADOW_CACHE = gemm.SHADOW_CACHE, False
        try:
            self.graphed = torch.cuda.make_graphed_callables(self.flat, args,
                                                             num_warmup_iters=warmup_iters)
        finally:
            gemm.SHADOW_CACHE = saved

    def __call__(self, inputs):
        flat = self.graphed(*(inputs[k] for k in IN_KEYS))
        n = len(OUT_KEYS)
        layers = [dict(zip(OUT_KEYS, flat[i:i + n])) for i in range(0, len(flat), n)]
        return {"outputs": layers[0], "aux_outputs": layers[1:]}


# "1" / "auto": split the step so that the plan starts after the encoder ("auto": only for the
# register-resident FPS, N <= 20480 points).  Default "0": the plan starts with the step.  Round 6
# (FPS 2.46 -> 2.25 ms): started after the encoder it ran into the encoder BACKWARD (attention
# dQ / dK/dV 68 / 95 -> 95-103 / 146-148 us beside it, the K = 2048 memory-gradient GEMM
# ~30 -> 94 us); started with the step it overlaps the SA / encoder forward instead and ends
# within the decoder: 1633-1636 -> 1642-1645 scenes/s (A/B on one box, tools/ab_plan_start.sh).
# ScanNet's 40000-point plan (~3.6 ms) must start with the step either way.
MID_START = os.environ.get("OV3D_PLAN_MID_START", "0")
MID_START_MAX_POINTS = 20480
SPLIT_AT = os.environ.get("OV3D_PLAN_SPLIT_AT", "encoder")   # or "memory_kv", "pre_encoder"


class StepGraph:
    """Replays forward + criterion + backward + clip_grad_norm_ + optimizer.step.

    model, crit: as for an eager step; opt: torch AdamW built with capturable=True, or
    optim.FusedAdamW (its step clips the gradients and rewrites the bf16 weight copies).
    sample: a batch dict (device tensors) fixing the static shapes.

    Sampling prefetch (prefetch_fps=True): the pre-encoder's furthest-point
    sampling depends on the input points only, and runs on 8 of the 256 CUs for
    ~3 ms; so do its ball query and the query FPS (Model3DETR.sampling_plan).  The
    plan is computed for the NEXT batch on its own stream, concurrently with this
    batch's graph replay, and handed to the next replay (as extra model inputs).  Each
    step still samples exactly one batch; results are identical.  step(batch, next_batch) keeps the
    pipeline primed; a batch that was not announced as `next_batch` (or whose point tensor
    was written in place after it was announced) is sampled eagerly first.  With an
    FusedAdamW optimizer each step first writes the groups' current lr / weight decay into
    the table the captured update reads (FusedAdamW.sync_hyper)."""

    def __init__(self, model, crit, opt, sample, amp_dtype=torch.bfloat16, clip=0.1,
                 warmup_iters=3, prefetch_fps=True, regionclip=None, before_capture=None):
        from . import gemm
        from . import pointnet2_utils as pu
        self.model, self.crit, self.opt = model, crit, opt
        self.regionclip = regionclip   # clip= of SetCriterion.forward (needs static_image_size)
        self.amp_dtype, self.clip = amp_dtype, clip
        self.static = {k: v.clone() for k, v in sample.items()}
        self.prefetch = prefetch_fps and hasattr(model, "pre_encoder")
        self._pu = pu
        self._expected = None
        if self.prefetch:
            self.npoint = model.pre_encoder.npoint
            self.next_pc = self.static["point_clouds"].clone()
            self.plan_cur = self._sample(self.static["point_clouds"])
        self.fps_stream = torch.cuda.Stream()
        # the next batch's sampling starts when this step's encoder forward is done: the
        # step is captured as TWO graphs split at Model3DETR.after_encoder (one memory pool),
        # and an event between their replays releases the side stream (ROCm PyTorch has no
        # external events inside a graph).  The FPS holds 8 CUs for ~2.5 ms; beside the
        # encoder's full-grid kernels it costs them a tail round (tools/contention.py:
        # attention forward 89 -> 127 us), beside the decoder's short launches ~nothing.
        npts = self.static["point_clouds"].shape[1]
        want = MID_START == "1" or (MID_START == "auto" and npts <= MID_START_MAX_POINTS)
        self.split = bool(self.prefetch and want and hasattr(model, "run_encoder"))
        self.mid_event = torch.cuda.Event() if self.split else None
        self.graph2 = None
        # warm-up and capture on streams dedicated to each role (dist.dedicated_stream): the
        # warm-up's eager collectives record their end events on the current stream, and a
        # stream holding one the process group's watchdog has not retired yet must never join
        # the capture (hipErrorCapturedEvent on the watchdog's query aborts the process)
        from . import dist as _dist
        dev = self.static["point_clouds"].device
        self.side = _dist.dedicated_stream(dev, "eager")
        cap = _dist.dedicated_stream(dev, "capture")
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            for _ in range(warmup_iters):
                self._body(gemm)
        torch.cuda.current_stream().wait_stream(self.side)
        if self.prefetch:
            self._set_plan(self._sample(self.static["point_clouds"]))
        if before_capture is not None:   # e.g. bench.py arms the in-kernel launch stamps here
            before_capture()
        self.graph = torch.cuda.CUDAGraph()
        self.opt.zero_grad(set_to_none=True)
        # with a process group the RCCL collectives are captured too; the watchdog thread of
        # the process group must not invalidate the capture ("thread_local" capture mode)
        pg = torch.distributed.is_available() and torch.distributed.is_initialized()
        mode = "thread_local" if pg else "global"
        if not self.split:
            with torch.cuda.graph(self.graph, stream=cap, capture_error_mode=mode):
                self.loss = self._body(gemm)
            return
        # split capture (the torch.cuda.graph context's steps, done by hand so the capture
        # can switch graphs in the middle of the forward)
        self.graph2 = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        cap.wait_stream(torch.cuda.current_stream())
        switched = []

        def switch():
            self.graph.capture_end()
            self.graph2.capture_begin(pool=self.graph.pool(), capture_error_mode=mode)
            switched.append(1)

        # split after the decoder's memory K / V GEMMs when the fused decoder runs (two
        # full-grid GEMMs that lose a tail round beside the FPS: 34 -> 53 us each), else
        # after the encoder
        dec = getattr(self.model, "decoder", None)
        if SPLIT_AT == "pre_encoder":
            target, attr = self.model, "after_pre_encoder"
        elif hasattr(dec, "_forward_fused") and SPLIT_AT == "memory_kv":
            target, attr = dec, "after_memory_kv"
        else:
            target, attr = self.model, "after_encoder"
        setattr(target, attr, switch)
        try:
            with torch.cuda.stream(cap):
                self.graph.capture_begin(capture_error_mode=mode)
                try:
                    self.loss = self._body(gemm)
                finally:
                    (self.graph2 if switched else self.graph).capture_end()
        finally:
            setattr(target, attr, None)
        torch.cuda.current_stream().wait_stream(cap)
        if len(switched) != 1:
            raise RuntimeError(f"StepGraph: the forward did not pass {attr} once")

    def _replay(self):
        self.graph.replay()
        if self.graph2 is not None:
            self.mid_event.record()
            self.graph2.replay()

    def _sample(self, pc):
        """-> dict of the step's point-only index work (extra model inputs)"""
        if hasattr(self.model, "sampling_plan"):
            return self.model.sampling_plan(pc)
        # the gather form: no host sync on the side stream (furthest_point_sample's eager
        # two-workgroup status check would block the host until the previous step retired)
        return {"pre_enc_inds": self._pu.furthest_point_sample_gather(
            pc[..., 0:3].contiguous(), self.npoint)[0]}

    def _set_plan(self, plan):
        from . import _native
        keys = list(self.plan_cur)
        _native.multi_copy([self.plan_cur[k] for k in keys], [plan[k] for k in keys])

    def _body(self, gemm):
        if not getattr(self.opt, "writes_shadows", False):
            gemm.refresh_shadows(force=True)   # captured: bf16 weight copies follow every update
        self.opt.zero_grad(set_to_none=True)
        inputs = {k: self.static[k] for k in IN_KEYS}
        if self.prefetch:
            inputs.update(self.plan_cur)
        with torch.autocast("cuda", dtype=self.amp_dtype or torch.float32,
                            enabled=self.amp_dtype is not None):
            out = self.model(inputs)
        loss, _ = self.crit(out, dict(self.static), clip=self.regionclip)
        loss.backward()
        if not getattr(self.opt, "clips_grads", False):
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.clip)
        self.opt.step()
        return loss.detach()

    def step(self, batch, next_batch=None):
        cur = torch.cuda.current_stream()
        if hasattr(self.opt, "sync_hyper"):
            self.opt.sync_hyper()   # this iteration's lr (engine.py:79) into the graph's table
        keys = list(self.static)
        dsts = [self.static[k] for k in keys]
        srcs = [batch[k] for k in keys]
        nb = next_batch if next_batch is not None else batch
        if self.prefetch:
            # the next batch's points ride in the same launch (the previous step's FPS, their
            # only reader, was joined at its end); a separate copy_ could land on a blit kernel
            # of ~0.3 ms on the critical path
            dsts.append(self.next_pc)
            srcs.append(nb["point_clouds"])
        if all(s.is_cuda and s.is_contiguous() and s.dtype == d.dtype and s.shape == d.shape
               for d, s in zip(dsts, srcs)):
            from . import _native
            _native.multi_copy(dsts, srcs)   # one launch
        else:
            for d, s in zip(dsts, srcs):
                d.copy_(s, non_blocking=True)
        if not self.prefetch:
            self.graph.replay()
            return self.loss
        # the prefetched plan is this batch's only if the announced tensor is the same object
        # AND was not written in place since (a loader refilling one device buffer bumps its
        # version counter): otherwise sample it now
        pc = batch["point_clouds"]
        if self._expected is None or pc is not self._expected[0] or \
                pc._version != self._expected[1]:
            self._set_plan(self._sample(self.static["point_clouds"]))
        self._expected = (nb["point_clouds"], nb["point_clouds"]._version)
        # the next batch's sampling plan runs on its own stream (own hardware queue),
        # concurrently with this step's graph; the graph reads plan_cur only
        if self.split:
            # the side-stream work is enqueued BEFORE the second graph (whose launch takes
            # the host ~0.2 ms, tools/graph_alone.py host), so the FPS is in its queue when
            # the first graph's last kernel retires (measured 1412 -> 1446 scenes/s)
            self.graph.replay()
            self.mid_event.record()
            self.fps_stream.wait_event(self.mid_event)   # after next_pc's copy, too
            with torch.cuda.stream(self.fps_stream):
                nxt = self._sample(self.next_pc)
            self.graph2.replay()
        else:
            self.fps_stream.wait_stream(cur)
            with torch.cuda.stream(self.fps_stream):
                nxt = self._sample(self.next_pc)
            self.graph.replay()
        cur.wait_stream(self.fps_stream)
        for t in nxt.values():
            t.record_stream(cur)
        self._set_plan(nxt)
        return self.loss
