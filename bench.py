"""Training-step throughput of the open-vocabulary 3DETR hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One step = forward (3DETR: FPS + ball query + grouping [HIP], SA-MLP,
3 encoder / 8 decoder layers, heads) + set criterion (GIoU [HIP] for all 8
layers, Hungarian matching, losses) + backward + clip_grad_norm_(0.1) + AdamW,
on a fresh synthetic SUN RGB-D-like batch (B=8 scenes x 20000 points per GPU,
nqueries=128, text embedding 21x640) already resident in HBM.  BASELINE.json
metric: scenes/sec (train step); weak scaling (8 scenes per GPU), DDP over RCCL.

Rank 0 prints ONE JSON line.  It carries a `roofline` object for the dominant
hand-written kernel (ov3d_fps, timed with HIP events on its launch stream; inside
the timed region in eager mode, right after it when the step replays a hipGraph) and a `cpu_baseline` (the CPU port of the same step: the
oracle's C restatement for the index kernels + PyTorch-CPU dense layers, a
bounded sample, rank 0 only, N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import ov3d_import  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BF16_DENSE_PEAK_TFLOPS = 2500.0
STEP_GFLOP_PER_SCENE = 113.64  # SURVEY §8d, fwd+bwd matmul/conv FLOPs, SUN config
SCANNET_GFLOP_PER_SCENE = 130.78


def default_args(**kw):
    """main.py defaults + the SUN RGB-D README / scripts/sunrgbd_ep1080.sh overrides."""
    a = dict(model_name="3detr", enc_type="vanilla", enc_nlayers=3, enc_dim=256, enc_ffn_dim=128,
             enc_dropout=0.1, enc_nhead=4, enc_activation="relu", dec_nlayers=8, dec_dim=256,
             dec_ffn_dim=256, dec_dropout=0.1, dec_nhead=4, mlp_dropout=0.3, preenc_npoints=2048,
             nqueries=128, use_color=False, matcher_giou_cost=3.0, matcher_cls_cost=1.0,
             matcher_center_cost=5.0, matcher_objectness_cost=5.0, loss_giou_weight=0.0,
             loss_sem_cls_weight=1.0, loss_no_object_weight=0.1, loss_angle_cls_weight=0.1,
             loss_angle_reg_weight=0.5, loss_center_weight=5.0, loss_size_weight=1.0,
             loss_2dalignment_weight=0.0, base_lr=7e-4, weight_decay=0.1, clip_gradient=0.1)
    a.update(kw)
    return argparse.Namespace(**a)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# C5 (BASELINE.json configs[4]): --use_image RegionCLIP RN50x4 ROI path + 2D
# alignment loss, bs=4/GPU (README.md:13-36: loss_2dalignment_weight 2e-4)
WORKLOADS = {
    "sun": dict(batch=8, use_image=False, args={}),
    "sun_image": dict(batch=4, use_image=True, args=dict(loss_2dalignment_weight=2e-4)),
    # C4 (BASELINE.json configs[3]): scripts/scannet_masked_ep1080.sh, ScanNet 40000 pts + colour
    # (scannet.py:181), masked encoder, 256 queries, differentiable GIoU loss
    "scannet": dict(batch=8, use_image=False, dataset="scannet", points=40000, queries=256,
                    args=dict(enc_type="masked", enc_dropout=0.3, nqueries=256, use_color=True,
                              base_lr=5e-4, matcher_giou_cost=2.0, matcher_cls_cost=1.0,
                              matcher_center_cost=0.0, matcher_objectness_cost=0.0,
                              loss_giou_weight=1.0, loss_no_object_weight=0.25)),
}


def build_regionclip(device):
    """RegionCLIP RN50x4 ROI-feature extractor (seed 11, no checkpoint offline), bf16."""
    from ov3d_amd import regionclip as rc
    clip, _ = rc.build_regionclip(compute_dtype=torch.bfloat16)
    clip = clip.to(device)
    clip.static_image_size = (530, 730)   # synthetic SUN images are all 530x730
    return clip


def regionclip_gflop_per_scene(batch, nqueries=128, layers=8):
    """algorithmic GFLOP/scene of the product's RegionCLIP pass (backbone once per image,
    res5 per ROI, reassociated pool) — tools/bench_regionclip.py counts the same terms."""
    backbone = 136.7                      # RN50x4 stem..res4 at 530x730 (conv FLOPs, per image)
    res5, pool = 9356.0e-3, 76.2e-3       # per 18x18 ROI
    return backbone + nqueries * layers * (res5 + pool)


def build(args, device, ddp=False, capturable=False, sync_bn=False, allreduce=False,
          dataset="sunrgbd", staged=True):
    """ddp: the reference's DistributedDataParallel + SyncBatchNorm (eager); sync_bn +
    allreduce: the same semantics for the captured step (SyncBatchNorm statistics
    all-reduced inside the fused BN kernels' launches, the gradient mean by ONE collective
    in FusedAdamW)."""
    ov3d = ov3d_import.load()
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import CONFIGS
    cfg = CONFIGS[dataset]()
    torch.manual_seed(0)
    model, _ = ov3d.build_model(args, cfg, text_embedding=synthetic.text_embedding(cfg.num_semcls + 1))
    model = model.to(device).train()
    if ddp or sync_bn:
        model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
    if ddp:
        model = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[device.index], bucket_cap_mb=32, gradient_as_bucket_view=True)
    crit = ov3d.build_criterion(args, cfg).to(device)
    params = [p for p in model.parameters() if p.requires_grad]
    if getattr(args, "optim", "fused") == "fused":
        # clip_grad_norm_(clip_gradient) + AdamW in three HIP launches (ov3d_amd/optim.py)
        from ov3d_amd.optim import FusedAdamW
        group = buckets = None
        if allreduce:
            import torch.distributed as tdist
            from ov3d_amd import dist as pdist
            group = tdist.group.WORLD
            if staged and hasattr(model, "dp_buckets"):
                # the decoder side's gradients all-reduced under the encoder / SA backward, on
                # a communicator of their own (dist.GradBuckets, dist.stage_after_encoder)
                bgroup = tdist.new_group(ranks=list(range(tdist.get_world_size())))
                buckets = pdist.GradBuckets(model.dp_buckets(), group=bgroup)
                pdist.stage_after_encoder(model, buckets)
        opt = FusedAdamW(params, lr=args.base_lr, weight_decay=args.weight_decay,
                         max_grad_norm=args.clip_gradient, allreduce_group=group,
                         grad_buckets=buckets)
        return model, crit, opt
    try:
        opt = torch.optim.AdamW(params, lr=args.base_lr, weight_decay=args.weight_decay, fused=True,
                                capturable=capturable)
    except Exception:  # fused AdamW unavailable -> multi-tensor
        opt = torch.optim.AdamW(params, lr=args.base_lr, weight_decay=args.weight_decay,
                                capturable=capturable)
    return model, crit, opt


def train_step(model, crit, opt, batch, args, amp_dtype, clip=None):
    opt.zero_grad(set_to_none=True)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    with torch.autocast("cuda", dtype=amp_dtype, enabled=amp_dtype is not None):
        out = model(inputs)
    loss, _ = crit(out, batch, clip=clip)
    loss.backward()
    if not getattr(opt, "clips_grads", False):
        torch.nn.utils.clip_grad_norm_(model.parameters(), args.clip_gradient)
    opt.step()
    return loss


def fps_launch_timings(pool, cli, reps=5):
    """Inside graph replays the kernel is not reachable by host events; time the same launch
    (pre-encoder FPS on the step's batch, same stream) right after the timed region."""
    from ov3d_amd import _native, pointnet2_utils as pu
    _native.timing_enable(["ov3d_fps"])
    for i in range(reps):
        pu.furthest_point_sample_gather(pool[i % len(pool)]["point_clouds"][..., 0:3].contiguous(), 2048)
    return _native.timing_collect()


def _gpu_busy(ms=3.0):
    """keep the stream busy (a spin kernel) while the host enqueues the timed launches, so
    the HIP events bracket kernel time, not host launch gaps"""
    try:
        torch.cuda._sleep(int(ms * 2.4e6))
    except Exception:
        pass


def attn_launch_timings(B, L, H=4, p=0.1, reps=5):
    """The roofline kernel: the encoder self-attention (flash attention, csrc/attn.hip) at the
    step's shape.  Inside graph replays it is not reachable by host events, so the same
    launches (forward kernel; backward = dQ + dK/dV kernels) run right after the timed region
    on the step's stream, bracketed by HIP events."""
    from ov3d_amd import attention as A
    E = H * A.HEAD_DIM
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn((L, B, 3 * E), device="cuda", dtype=torch.bfloat16, generator=g)
    x.requires_grad_(True)
    gout = torch.randn((L, B, E), device="cuda", dtype=torch.bfloat16, generator=g)
    spec = ((0, 0), (0, E), (0, 2 * E))
    st = torch.cuda.current_stream()
    fwd, bwd = [], []
    for i in range(reps + 1):          # the first pair warms the allocator
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        _gpu_busy()
        ev[0].record(st)
        o = A.attention_packed([x], spec, L, L, H, p, site=1)
        ev[1].record(st)
        o.backward(gout)
        ev[2].record(st)
        ev[2].synchronize()
        x.grad = None
        if i:
            fwd.append(ev[0].elapsed_time(ev[1]))
            bwd.append(ev[1].elapsed_time(ev[2]))
    return float(np.mean(fwd)), float(np.mean(bwd))


def gemm_ceiling(n=8192, reps=10):
    """measured bf16 GEMM ceiling of this box: hipBLASLt (torch.matmul) n x n x n on random
    data, HIP events around `reps` back-to-back launches (SURVEY §8d asks for it beside the
    vendor peak)"""
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.randn((n, n), device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn((n, n), device="cuda", dtype=torch.bfloat16, generator=g)
    for _ in range(3):
        torch.matmul(a, b)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    _gpu_busy(1.0)
    e0.record(st)
    for _ in range(reps):
        torch.matmul(a, b)
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"tflops": round(2.0 * n ** 3 / (ms * 1e-3) / 1e12, 1), "shape": f"{n}x{n}x{n} bf16",
            "ms": round(ms, 4), "how": "torch.matmul (hipBLASLt), random data, HIP events"}


def _timed(fn, reps):
    """HIP events around `reps` back-to-back calls queued behind a spin kernel (kernel time, not
    host launch gaps) -> ms per call"""
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    _gpu_busy(2.0)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def index_kernel_rates(batch, npoint=2048, radius=0.2, nsample=64, L=8, Q=128, reps=5):
    """Per-kernel HBM figures for the index / geometry kernels (BASELINE.md:62):
    algorithmic bytes under the streaming formulation / measured time (HIP events, the step's
    shapes on its batch)."""
    from ov3d_amd import nms, pointnet2_utils as pu
    from ov3d_amd.box_util import generalized_box3d_iou
    xyz = batch["point_clouds"][..., 0:3].contiguous()
    B, N, _ = xyz.shape
    _, new_xyz = pu.furthest_point_sample_gather(xyz, npoint)
    idx = pu.ball_query(radius, nsample, xyz, new_xyz)
    grouper = pu.QueryAndGroup(radius, nsample, normalize_xyz=True)
    corners = batch["gt_box_corners"]                                   # (B, G, 8, 3)
    G = corners.shape[1]
    g = torch.Generator(device="cuda").manual_seed(3)
    pred = corners[:, torch.randint(0, G, (Q,), device="cuda", generator=g)]
    pred = (pred + 0.05 * torch.randn(pred.shape, device="cuda", generator=g)).repeat(L, 1, 1, 1)
    gt = corners.repeat(L, 1, 1, 1)
    nums = batch["gt_box_present"].sum(1).int().repeat(L)
    boxes = nms.nms_boxes_from_corners(pred[:B], torch.rand((B, Q), device="cuda", generator=g),
                                       torch.randint(0, 10, (B, Q), device="cuda", generator=g))
    scanned = ball_query_scanned(idx, N)
    # FPS is a serial chain of dependent argmax rounds over register-resident points: it is
    # reported as microseconds per sampling iteration against its latency floor ("fps" below),
    # not as a byte rate
    rows = {
        "ov3d_ball_query": (lambda: pu.ball_query(radius, nsample, xyz, new_xyz),
                            B * N * 12 + B * npoint * nsample * 4,
                            f"r={radius} S={nsample}: the scene's points read from HBM once (B*N*12 B) + "
                            f"the indices written (B*M*S*4 B); the reference's scans ({scanned} points "
                            f"over the B*M centroids, each stopping at the S-th in-radius point, SURVEY "
                            f"Appendix A.2) are replaced by a per-scene cell index (csrc/group.hip "
                            f"bq_cells_*: 27 cells per centroid, L2-resident): scan_points_per_s is "
                            f"the reference-scan-equivalent rate"),
        "ov3d_group_fwd": (lambda: grouper.rows(xyz, new_xyz, None, idx=idx),
                           B * npoint * nsample * (3 * 4 + 4),
                           "(B,M,S,3) fp32 rows out + idx in"),
        "ov3d_giou3d": (lambda: generalized_box3d_iou(pred, gt, nums), L * B * ((Q + G) * 96 + Q * G * 4),
                        f"{L} layers x B x (({Q} + {G}) boxes x 96 B corners + {Q} x {G} x 4 B out)"),
        "ov3d_nms3d": (lambda: nms.nms3d_batched(boxes, 0.25), B * Q * Q * 56,
                       f"B x K^2 x 56 B (K={Q}, fp64 boxes)"),
    }
    out = {}
    for name, (fn, nbytes, what) in rows.items():
        ms = _timed(fn, reps)
        out[name] = {"ms": round(ms, 4), "alg_bytes": nbytes, "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                     "frac_hbm": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "bytes": what}
    # ball query is bound by the distance tests over the L2-resident scene, not by HBM: the
    # reference scan's point count per second (points each centroid's scan reads until its S-th
    # hit) is its throughput figure
    bq = out["ov3d_ball_query"]
    bq["scanned_points"] = scanned
    bq["scan_points_per_s"] = round(scanned / (bq["ms"] * 1e-3), 1)
    return out


def ball_query_scanned(idx, N):
    """points the reference scan reads (per centroid, in index order, until
    the nsample-th strict d^2 < r^2 hit, else all N), summed over every scene and centroid, from
    the ball-query indices themselves (bit-exact against the C restatement, tests/
    test_kernels_gpu.py): a full row's S-th index is the last point scanned; a row that never
    filled (its padding repeats the first hit, so the indices stop increasing) scanned all N."""
    idx = idx.long()
    S = idx.shape[-1]
    full = (idx[..., 1:] > idx[..., :-1]).all(dim=-1) if S > 1 else torch.ones_like(idx[..., 0], dtype=torch.bool)
    stop = torch.where(full, idx[..., -1] + 1, torch.full_like(idx[..., -1], N))
    return int(stop.sum().item())


def fps_latency_floor(B, M, reps=3):
    """FPS iteration cost with one point per thread (N = M): what the per-iteration barrier /
    reduction / LDS chain costs with (almost) no distance work -- the kernel's latency floor"""
    from ov3d_amd import pointnet2_utils as pu
    xyz = torch.rand((B, M, 3), device="cuda") + 0.1
    st = torch.cuda.current_stream()
    ts = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        pu.furthest_point_sample_gather(xyz, M)
        e1.record(st)
        e1.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    return float(np.mean(ts))


def cpu_baseline(args, rounds=5, b8_steps=2):
    """The reference step on the host cores: product host code on CPU with the
    C oracle for FPS / ball query / grouping / GIoU (test-infrastructure
    injection, oracle/torch_shim.py), fp32, a bounded sample.  Every setting is warmed by one
    untimed step first; then `rounds` interleaved pairs of B=1 steps with torch.autograd anomaly
    detection off and on (the reference's default is on: main.py:499, quirk Q7), then
    `b8_steps` B=8 steps (the GPU workload's batch; capped: a B=8 step is ~10-15 s on 16
    cores).  value = B=1 (config C1) scenes / median step time (BASELINE.md:58-60)."""
    from oracle import torch_shim
    ov3d = ov3d_import.load()
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    threads = len(os.sched_getaffinity(0))
    threads = max(1, min(threads, 16))  # the GPU box's CPU share
    torch.set_num_threads(threads)
    saved = torch_shim.install(ov3d)
    try:
        cfg = SunrgbdDatasetConfig()
        torch.manual_seed(0)
        model, _ = ov3d.build_model(args, cfg, text_embedding=synthetic.text_embedding())
        model.train()
        crit = ov3d.build_criterion(args, cfg)
        opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=args.base_lr,
                                weight_decay=args.weight_decay)

        def step(b, anomaly=False):
            t0 = time.perf_counter()
            with torch.autograd.set_detect_anomaly(anomaly, check_nan=True):
                opt.zero_grad(set_to_none=True)
                out = model({k: b[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
                loss, _ = crit(out, b)
                loss.backward()
                torch.nn.utils.clip_grad_norm_(model.parameters(), args.clip_gradient)
                opt.step()
            return time.perf_counter() - t0

        # warm-up: every batch size and anomaly setting once, untimed
        step(synthetic.make_batch(1, seed=97))
        step(synthetic.make_batch(1, seed=98), anomaly=True)
        step(synthetic.make_batch(8, seed=99))
        ts = {"B=1": [], "B=1 anomaly": [], "B=8": []}
        for i in range(rounds):   # interleaved, so drift hits both settings alike
            ts["B=1"].append(step(synthetic.make_batch(1, seed=100 + i)))
            ts["B=1 anomaly"].append(step(synthetic.make_batch(1, seed=200 + i), anomaly=True))
        for i in range(b8_steps):
            ts["B=8"].append(step(synthetic.make_batch(8, seed=300 + i)))
    finally:
        torch_shim.uninstall(saved)
    bs = {"B=1": 1, "B=1 anomaly": 1, "B=8": 8}
    rates = {k: bs[k] / float(np.median(v)) for k, v in ts.items()}
    return {"value": round(rates["B=1"], 4), "unit": "scenes/s", "cores": threads, "kind": "port",
            "by_batch": {k: {"value": round(rates[k], 4), "steps": len(ts[k]),
                             "step_s": [round(t, 3) for t in ts[k]]} for k in ts},
            "anomaly_cost": round(float(np.median(ts["B=1 anomaly"])) / float(np.median(ts["B=1"])), 3),
            "sample": (f"after one untimed warm-up step per setting: {rounds} interleaved pairs of B=1 "
                       f"train steps with torch.autograd anomaly detection off / on (the reference "
                       f"default is on, main.py:499), then {b8_steps} B=8 steps (capped: ~10-15 s "
                       "each); 20000-pt scenes, fp32, oracle C for FPS/ball-query/grouping/GIoU + "
                       "PyTorch-CPU dense layers; value: B=1 scenes / median step time")}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)      # >= 50 timed steps
    p.add_argument("--warmup", type=int, default=10)     # after 10 warm-up steps
    p.add_argument("--workload", default="sun", choices=sorted(WORKLOADS),
                   help="sun = BASELINE metric config (C2/C3); sun_image = C5 (RegionCLIP ROI path)")
    p.add_argument("--batch", type=int, default=None, help="scenes per GPU (default: workload's)")
    p.add_argument("--points", type=int, default=None, help="points per scene (default: workload's)")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--pool", type=int, default=4, help="distinct synthetic batches cycled")
    p.add_argument("--no-prefetch", action="store_true",
                   help="do not overlap the next batch's pre-encoder FPS with this step")
    p.add_argument("--eager", "--no-graph", dest="eager", action="store_true",
                   help="launch the step eagerly (DDP at N>1); by default the whole step is "
                        "captured once and replayed as one hipGraph (graphs.StepGraph), "
                        "with the RCCL collectives inside it at N>1")
    p.add_argument("--dp-collectives", action="store_true",
                   help="run the data-parallel collectives (SyncBN statistics, gradient all-reduce) "
                        "even at world size 1 (tests the captured collectives on one GPU)")
    p.add_argument("--no-staged-allreduce", action="store_true",
                   help="data parallel: all-reduce every gradient at the end of the step instead of "
                        "starting the decoder side's bucket under the encoder backward")
    p.add_argument("--no-defer-wgrad", action="store_true",
                   help="compute each linear layer's dW / db inside its backward instead of one "
                        "grouped launch at the end of the backward pass (gemm.DEFER_WGRAD)")
    p.add_argument("--optim", default="fused", choices=["fused", "torch"],
                   help="fused: clip + AdamW in three HIP launches (ov3d_amd.optim.FusedAdamW); "
                        "torch: clip_grad_norm_ + torch.optim.AdamW(fused=True)")
    cli = p.parse_args()
    # stdout carries exactly ONE JSON line: native libraries' banners (RCCL's version block at
    # communicator init) are sent to stderr by pointing fd 1 there; the result line is written
    # to the saved descriptor
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    wl = WORKLOADS[cli.workload]
    if cli.batch is None:
        cli.batch = wl["batch"]
    if cli.points is None:
        cli.points = wl.get("points", 20000)
    dataset = wl.get("dataset", "sunrgbd")

    ov3d = ov3d_import.load()
    from ov3d_amd import _native, dist, synthetic
    if cli.dp_collectives and "WORLD_SIZE" not in os.environ:
        # a one-rank RCCL group so the captured step holds real collectives (single-GPU test)
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=os.environ.get("MASTER_PORT", "29517"))
        torch.cuda.set_device(0)
        dist.capture_safe_env()
        torch.distributed.init_process_group(backend="nccl", init_method="env://", world_size=1,
                                             rank=0)
    rank, world, local = dist.init_from_env()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    args = default_args(**wl["args"])
    args.optim = cli.optim
    amp = torch.bfloat16 if cli.dtype == "bf16" else None
    # N >= 1: the whole step is one captured hipGraph; at N > 1 it holds the SyncBN and the
    # gradient collectives (RCCL), no DDP wrapper.  --eager: the DDP path.
    use_graph = not cli.eager
    dp = (world > 1 or cli.dp_collectives) and use_graph
    if dp and cli.dp_collectives:
        from ov3d_amd import sa_fused
        sa_fused.FORCE_SYNC = True   # collectives even at world 1 (capture test)
    if cli.optim != "fused" and dp:
        raise SystemExit("the captured data-parallel step needs --optim fused")
    model, crit, opt = build(args, device, ddp=world > 1 and not use_graph, capturable=use_graph,
                             sync_bn=dp, allreduce=dp, dataset=dataset,
                             staged=not cli.no_staged_allreduce)
    if not cli.no_defer_wgrad and not (world > 1 and not use_graph):
        from ov3d_amd import gemm
        gemm.DEFER_WGRAD = True   # one grouped weight-gradient launch per backward (not under DDP)
    clip = build_regionclip(device) if wl["use_image"] else None
    pool = [synthetic.make_batch(cli.batch, seed=1000 * rank + i, num_points=cli.points, device=device,
                                 use_image=wl["use_image"], dataset=dataset,
                                 use_color=bool(args.use_color))
            for i in range(cli.pool)]

    graphed = None
    stamp_buf = None
    if use_graph:
        from ov3d_amd.graphs import StepGraph
        # the encoder attention launches captured into the step carry in-kernel wall-clock
        # stamps (csrc/common.h ov3d_stamp): the roofline kernel is timed inside the step
        # (armed after the eager warm-up, so the launch table holds the captured launches only)
        stamp_buf = torch.zeros((1 << 21,), dtype=torch.int64, device=device)
        try:
            graphed = StepGraph(model, crit, opt, pool[0], amp_dtype=amp, clip=args.clip_gradient,
                                prefetch_fps=not cli.no_prefetch, regionclip=clip,
                                before_capture=lambda: _native.stamps_arm(stamp_buf, min_work=1 << 20))
        finally:
            _native.stamps_arm(None)

    def step(i):
        if graphed is not None:
            return graphed.step(pool[i % cli.pool], pool[(i + 1) % cli.pool])
        return train_step(model, crit, opt, pool[i % cli.pool], args, amp, clip=clip)

    for i in range(cli.warmup):
        step(i)
    torch.cuda.synchronize()
    dist.barrier()

    if graphed is None:
        _native.timing_enable(["ov3d_fps"])
    torch.cuda.synchronize()
    dist.barrier()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(cli.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(cli.steps):
        loss = step(i)
        marks[i + 1].record()
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    # in-step kernel times: the last timed step's captured launches, then 5 more replays
    stamped = []
    if stamp_buf is not None:
        stamped.append(_native.stamps_read(stamp_buf))
        for i in range(5):
            stamp_buf.zero_()
            step(cli.steps + i)
            torch.cuda.synchronize()
            stamped.append(_native.stamps_read(stamp_buf))
    timings = _native.timing_collect() if graphed is None else fps_launch_timings(pool, cli)
    att = None
    rates = gemm_ref = None
    if rank == 0 and dataset in ("sunrgbd", "scannet"):
        att = attn_launch_timings(cli.batch, args.preenc_npoints, args.enc_nhead, args.enc_dropout)
        fps_floor_ms = fps_latency_floor(cli.batch, args.preenc_npoints)
        gemm_ref = gemm_ceiling()
        if dataset == "sunrgbd":
            rates = index_kernel_rates(pool[0], npoint=args.preenc_npoints, Q=args.nqueries,
                                       L=args.dec_nlayers)
    el = torch.tensor([elapsed], device=device, dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())
    if not torch.isfinite(loss).item():
        raise RuntimeError("non-finite loss")

    if rank != 0:
        return
    scenes = cli.batch * world * cli.steps
    value = scenes / elapsed
    # per-step times on this rank (HIP events between steps; SURVEY §8d asks for the median)
    per_step = [marks[i].elapsed_time(marks[i + 1]) for i in range(cli.steps)]
    # roofline: the encoder flash attention (the largest kernel family on the step's critical
    # path; FPS runs on the side stream).  Algorithmic flops per launch: 4 * L^2 * d per
    # (scene, head) forward (Q K^T and P V); the backward 10 * L^2 * d (dV, dP, dS->dQ, dK:
    # 2.5x the forward, the usual flash-attention count; the S recompute is not counted)
    roof, extra = None, {}
    if att is not None:
        L, H, d = args.preenc_npoints, args.enc_nhead, 64
        fwd_ms, bwd_ms = att
        fl_fwd = 4.0 * L * L * d * cli.batch * H
        # in-step launch times (stamps): the encoder layers at L (C4: the first masked layer;
        # its interim layers run at L/2 and are not averaged in)
        per = {k: [] for k in _native.STAMP_KINDS}
        for rec in stamped:
            for k, ms, work in rec:
                if k in ("fwd", "dq", "dkdv") and work == L * L:
                    per[k].append(ms)
        in_step = {k: float(np.mean(v)) for k, v in per.items() if v}
        fwd_in = in_step.get("fwd")
        use_ms = fwd_in if fwd_in else fwd_ms
        ach = fl_fwd / (use_ms * 1e-3) / 1e12
        traffic, tsrc = None, None
        # the latest PMC record of the shipped kernel (tools/attn_traffic.py over gpu_pmc.sh)
        for rec_name in ("r04_attn_pmc.json", "r03_attn_pmc.json"):
            pmc = os.path.join(ROOT, "profiles", rec_name)
            if os.path.exists(pmc) and (cli.batch, L, H) == (8, 2048, 4) and dataset == "sunrgbd":
                traffic = json.load(open(pmc)).get("fwd_traffic_bytes_per_launch")
                tsrc = f"profiles/{rec_name} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)"
                break
        kname = "attn_fwd_kernel (encoder self-attention, B=%d H=%d L=%d d=64, dropout %.1f%s)" % (
            cli.batch, H, L, args.enc_dropout, ", radius mask" if dataset == "scannet" else "")
        roof = {"bound": "mfma", "achieved": round(ach, 1), "peak": BF16_DENSE_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(ach / BF16_DENSE_PEAK_TFLOPS, 4),
                "traffic": traffic, "traffic_source": tsrc, "kernel": kname,
                "flop_per_launch": fl_fwd, "avg_launch_ms": round(use_ms, 4),
                "launches": len(per["fwd"]) if fwd_in else 5,
                "timing": ("in-step: in-kernel wall-clock stamps (first-wave entry to last-wave exit) "
                           "of the captured step's launches, the last timed step + 5 replays"
                           if fwd_in else "standalone relaunch after the timed region, HIP events"),
                "standalone_relaunch_ms": round(fwd_ms, 4)}
        if gemm_ref:
            roof["measured_gemm_ceiling_tflops"] = gemm_ref["tflops"]
            roof["frac_of_measured_gemm"] = round(ach / gemm_ref["tflops"], 4)
            extra["gemm_ceiling"] = gemm_ref
        fl_bwd = 2.5 * fl_fwd
        bwd_in = in_step.get("dq", 0.0) + in_step.get("dkdv", 0.0) if "dq" in in_step else None
        use_b = bwd_in if bwd_in else bwd_ms
        extra["attn_bwd"] = {"kernels": "attn_bwd_dq_kernel + attn_bwd_dkdv_kernel",
                             "avg_ms": round(use_b, 4), "flop": fl_bwd,
                             "dq_ms": round(in_step["dq"], 4) if "dq" in in_step else None,
                             "dkdv_ms": round(in_step["dkdv"], 4) if "dkdv" in in_step else None,
                             "achieved_tflops": round(fl_bwd / (use_b * 1e-3) / 1e12, 1),
                             "frac": round(fl_bwd / (use_b * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS, 4),
                             "timing": "in-step stamps" if bwd_in else "standalone relaunch",
                             "standalone_relaunch_ms": round(bwd_ms, 4)}
    if wl["use_image"]:
        # C5: the dominant kernel is the 256 x 256 tile GEMM (every RegionCLIP backbone / res5
        # convolution and attention-pool product, ~3/4 of the step): its in-step stamps, summed
        # over the step's launches (flops 2 M N K per launch, from the launch table)
        recs = [[(ms, work) for k, ms, work in rec if k == "gemm256"] for rec in stamped]
        recs = [r for r in recs if r]
        if recs:
            step_ms = float(np.mean([sum(ms for ms, _ in r) for r in recs]))
            step_fl = float(np.mean([sum(w for _, w in r) for r in recs]))
            nl = int(round(np.mean([len(r) for r in recs])))
            ach = step_fl / (step_ms * 1e-3) / 1e12
            big = max(recs[0], key=lambda t: t[1])
            if roof is not None:
                extra["encoder_attention"] = roof
            roof = {"bound": "mfma", "achieved": round(ach, 1), "peak": BF16_DENSE_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / BF16_DENSE_PEAK_TFLOPS, 4),
                    "traffic": None,
                    "kernel": ("gemm256_kernel (csrc/gemm256.hip: every RegionCLIP RN50x4 backbone / "
                               "res5 convolution, implicit-GEMM 3x3 and 1x1, and the attention-pool "
                               "products of the C5 step)"),
                    "flop_per_launch": round(step_fl / nl), "avg_launch_ms": round(step_ms / nl, 4),
                    "launches": nl, "flop_per_step": step_fl, "ms_per_step": round(step_ms, 3),
                    "largest_launch": {"flop": big[1], "ms": round(big[0], 4),
                                       "tflops": round(big[1] / (big[0] * 1e-3) / 1e12, 1)},
                    "timing": ("in-step: in-kernel wall-clock stamps (first-wave entry to last-wave "
                               "exit) of every captured gemm256 launch, summed per step, the last "
                               "timed step + 5 replays")}
            if gemm_ref:
                roof["measured_gemm_ceiling_tflops"] = gemm_ref["tflops"]
                roof["frac_of_measured_gemm"] = round(ach / gemm_ref["tflops"], 4)
    if rates:
        extra["index_kernels_hbm"] = rates
    # FPS (side stream): a serial chain of M - 1 dependent iterations, reported per iteration
    # against the same kernel's cost with one point per thread (its latency floor)
    fps = timings.get("ov3d_fps", [])
    pre = [t for t in fps if t["shape"][1] == cli.points]
    if pre and att is not None:
        B, N, M = pre[0]["shape"]
        avg_ms = float(np.mean([t["ms"] for t in pre]))
        kern = "fps_cull_kernel" if N <= 20480 else "fps_pair_kernel"
        extra["fps"] = {"kernel": "%s (pre-encoder, B=%d N=%d M=%d, side stream)" % (kern, B, N, M),
                        "avg_launch_ms": round(avg_ms, 4),
                        "us_per_iteration": round(avg_ms * 1e3 / (M - 1), 4),
                        "floor_us_per_iteration": round(fps_floor_ms * 1e3 / (M - 1), 4),
                        "floor": f"same kernel, N = M = {M} (one point per thread)"}
    gflop_scene = STEP_GFLOP_PER_SCENE
    metric = "scenes/sec (train step) SUN RGB-D 20k pts nqueries=128"
    workload = (f"SUN RGB-D train step, bs={cli.batch}/GPU, {cli.points} pts, nqueries=128, "
                "3DETR 256-d enc3/dec8, text-emb 640, AdamW + clip 0.1")
    if dataset == "scannet":
        gflop_scene = SCANNET_GFLOP_PER_SCENE
        metric = "scenes/sec (train step) ScanNet 40k pts + colour nqueries=256 masked encoder (C4)"
        workload = (f"ScanNet train step (scannet_masked_ep1080.sh), bs={cli.batch}/GPU, {cli.points} "
                    "pts + colour, nqueries=256, masked encoder, GIoU loss, AdamW + clip 0.1")
    if wl["use_image"]:
        gflop_scene += regionclip_gflop_per_scene(cli.batch)
        metric += " +RegionCLIP RN50x4 2D alignment (C5)"
        workload += ", --use_image: RegionCLIP RN50x4 ROI features (8 layers x 128 boxes) + 2D alignment loss 2e-4"
    step_tflops = gflop_scene * value / 1e3
    res = {
        "metric": metric,
        "value": round(value, 3), "unit": "scenes/s", "n_gpus": world, "steps": cli.steps,
        "warmup": cli.warmup, "ms_per_step": round(elapsed / cli.steps * 1e3, 3),
        "ms_per_step_median": round(float(np.median(per_step)), 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": cli.dtype,
        "data": "synthetic SUN RGB-D-like scenes (numpy PCG64), random-init weights",
        "config": {"workload": workload,
                   "global_batch": cli.batch * world, "points": cli.points, "parallelism": f"dp{world}"},
        "roofline": roof,
        **extra,
        "step_mfma": {"achieved_tflops": round(step_tflops, 2), "peak_tflops": BF16_DENSE_PEAK_TFLOPS,
                      "frac": round(step_tflops / (world * BF16_DENSE_PEAK_TFLOPS), 5)},
    }
    if dataset == "scannet":
        res["data"] = "synthetic ScanNet-like scenes (numpy PCG64, axis-aligned boxes), random-init weights"
    if wl["use_image"]:
        res["cpu_baseline"] = {"value": None, "note": "not run for C5: the RN50x4 ROI path is "
                               f"{regionclip_gflop_per_scene(cli.batch) / 1e3:.1f} TFLOP/scene"}
    elif world == 1 and not cli.no_cpu_baseline and dataset == "sunrgbd":
        try:
            res["cpu_baseline"] = cpu_baseline(default_args())
        except Exception as e:  # report, never fake
            res["cpu_baseline"] = {"value": None, "error": repr(e)}
    os.write(result_fd, (json.dumps(res) + "\n").encode())


if __name__ == "__main__":
    main()
