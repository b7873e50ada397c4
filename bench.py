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
          dataset="sunrgbd"):
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
        group = None
        if allreduce:
            import torch.distributed as tdist
            group = tdist.group.WORLD
        opt = FusedAdamW(params, lr=args.base_lr, weight_decay=args.weight_decay,
                         max_grad_norm=args.clip_gradient, allreduce_group=group)
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


def cpu_baseline(args, batch_size=1, steps=2):
    """The reference step on the host cores: product host code on CPU with the
    C oracle for FPS / ball query / grouping / GIoU (test-infrastructure
    injection, oracle/torch_shim.py), fp32, bounded sample."""
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
        batches = [synthetic.make_batch(batch_size, seed=100 + i) for i in range(steps + 1)]

        def step(b):
            opt.zero_grad(set_to_none=True)
            out = model({k: b[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
            loss, _ = crit(out, b)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), args.clip_gradient)
            opt.step()

        step(batches[0])  # warm-up
        t0 = time.perf_counter()
        for i in range(steps):
            step(batches[i + 1])
        dt = time.perf_counter() - t0
    finally:
        torch_shim.uninstall(saved)
    return {"value": round(batch_size * steps / dt, 4), "unit": "scenes/s", "cores": threads,
            "kind": "port",
            "sample": f"{steps} train steps x {batch_size} scene(s) of 20000 pts (B={batch_size}), fp32, "
                      "oracle C for FPS/ball-query/grouping/GIoU + PyTorch-CPU dense layers"}


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
                             sync_bn=dp, allreduce=dp, dataset=dataset)
    if use_graph and not cli.no_defer_wgrad:
        from ov3d_amd import gemm
        gemm.DEFER_WGRAD = True   # one grouped weight-gradient launch per backward (not under DDP)
    clip = build_regionclip(device) if wl["use_image"] else None
    pool = [synthetic.make_batch(cli.batch, seed=1000 * rank + i, num_points=cli.points, device=device,
                                 use_image=wl["use_image"], dataset=dataset,
                                 use_color=bool(args.use_color))
            for i in range(cli.pool)]

    graphed = None
    if use_graph:
        from ov3d_amd.graphs import StepGraph
        graphed = StepGraph(model, crit, opt, pool[0], amp_dtype=amp, clip=args.clip_gradient,
                            prefetch_fps=not cli.no_prefetch, regionclip=clip)

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
    t0 = time.perf_counter()
    for i in range(cli.steps):
        loss = step(i)
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    timings = _native.timing_collect() if graphed is None else fps_launch_timings(pool, cli)
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
    # roofline of ov3d_fps: launches alternate pre-encoder (N=20000 -> 2048) and query (2048 -> 128)
    fps = timings.get("ov3d_fps", [])
    pre = [t for t in fps if t["shape"][1] == cli.points]
    roof = None
    if pre:
        B, N, M = pre[0]["shape"]
        avg_ms = float(np.mean([t["ms"] for t in pre]))
        algo_bytes = B * M * N * 16.0      # per scene M*N*(12 B coords + 4 B running min)
        achieved = algo_bytes / (avg_ms * 1e-3) / 1e9
        traffic, tsrc = None, None
        pmc = os.path.join(ROOT, "profiles", "r02_fps_pmc.json")
        if os.path.exists(pmc) and (B, N, M) == (8, 20000, 2048):
            traffic = json.load(open(pmc))["traffic_bytes_per_launch"]
            tsrc = "profiles/r02_fps_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, gfx950-corrected)"
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                "kernel": "ov3d_fps (pre-encoder, B=%d N=%d M=%d)" % (B, N, M),
                "avg_launch_ms": round(avg_ms, 4), "launches": len(pre)}
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
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": cli.dtype,
        "data": "synthetic SUN RGB-D-like scenes (numpy PCG64), random-init weights",
        "config": {"workload": workload,
                   "global_batch": cli.batch * world, "points": cli.points, "parallelism": f"dp{world}"},
        "roofline": roof,
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
