"""Data-parallel path on CPU: world_size 2 over gloo (the GPU path is the same code on
RCCL).  Covers the reference utils/dist.py API mirror and one DDP training step whose
averaged gradients must equal the single-process gradients on the whole batch
(the reference's num_boxes all-reduce, criterion.py:425, makes the box-normalised
losses batch-split invariant)."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from helpers import ROOT, batch_from_fixture, build_model_from_fixture, fixture, ov3d, rel_err

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    from ov3d_amd import dist
    r, w, _ = dist.init_from_env(backend="gloo")
    assert (r, w) == (rank, WORLD)
    return dist


def _collectives(rank, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import ov3d_import
    ov3d_import.load()
    dist = _init(rank, port)
    res = {}
    res["sum"] = dist.all_reduce_sum(torch.tensor(float(rank + 1))).item()
    res["avg"] = dist.all_reduce_average(torch.tensor([2.0 * rank, 4.0])).tolist()
    co = dist.all_reduce_coalesced([torch.tensor(1.0 + rank), torch.full((2, 2), 3.0 * rank)])
    res["co0"] = co[0].item()
    res["co1"] = co[1].tolist()
    rd = dist.reduce_dict({"b": torch.tensor(float(rank)), "a": torch.tensor(10.0 * rank)})
    res["rd"] = {k: v.item() for k, v in rd.items()}
    res["gather"] = dist.all_gather_pickle({"rank": rank, "pay": "x" * (5 + 100 * rank)}, "cpu")
    res["gdict"] = dist.all_gather_dict({"t": torch.full((1, 3), float(rank))})["t"].tolist()
    with open(os.path.join(out_dir, f"coll{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    torch.distributed.destroy_process_group()


def test_collectives_world2():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_collectives, args=(_free_port(), d), nprocs=WORLD, join=True)
        for rank in range(WORLD):
            with open(os.path.join(d, f"coll{rank}.json")) as f:
                r = json.load(f)
            assert r["sum"] == 3.0
            assert r["avg"] == [1.0, 4.0]
            assert r["co0"] == 1.5 and r["co1"] == [[1.5, 1.5], [1.5, 1.5]]
            assert r["rd"] == {"a": 5.0, "b": 0.5}
            assert [g["rank"] for g in r["gather"]] == [0, 1]
            assert len(r["gather"][1]["pay"]) == 105
            assert r["gdict"] == [[0.0] * 3, [1.0] * 3]


def _step(model, crit, batch):
    out = model({k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
    loss, ld = crit(out, batch)
    loss.backward()
    return loss


def _ddp_rank(rank, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    torch.set_num_threads(2)
    from oracle import torch_shim
    from helpers import batch_from_fixture as bff, build_model_from_fixture as bmf, fixture as fxl, ov3d as pkg
    _init(rank, port)
    torch_shim.install(pkg)
    from ov3d_amd.criterion import build_criterion
    fx = fxl("model_sun.npz")
    model, cfg, args = bmf(fx, "cpu", "sunrgbd")
    args.loss_2dalignment_weight = 0.0
    model.eval()     # running-stat BN, no dropout: per-scene independent forward
    ddp = torch.nn.parallel.DistributedDataParallel(model)
    crit = build_criterion(args, cfg)
    batch = {k: v[rank: rank + 1] for k, v in bff(fx, "cpu").items()}
    loss = _step(ddp, crit, batch)
    grads = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    torch.save({"loss": loss.detach(), "grads": grads}, os.path.join(out_dir, f"ddp{rank}.pt"))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.fixture()
def shim():
    from oracle import torch_shim
    saved = torch_shim.install(ov3d)
    yield
    torch_shim.uninstall(saved)


def test_ddp_gradients_equal_rank_average(shim, monkeypatch):
    """DDP step == the mean of the per-scene gradients, each computed with the GLOBAL
    average num_boxes (what criterion.py:425's all_reduce_average yields on every rank).
    Other loss terms are per-rank means (reference semantics), so the comparison target
    is the rank average, not a single whole-batch step."""
    from ov3d_amd import criterion as crit_mod
    torch.set_num_threads(4)
    fx = fixture("model_sun.npz")
    full = batch_from_fixture(fx, "cpu")
    nbox = full["gt_box_present"].sum(dim=1)
    monkeypatch.setattr(crit_mod, "all_reduce_average", lambda t: nbox.sum() / WORLD)
    ref, losses = {}, []
    for r in range(WORLD):
        model, cfg, args = build_model_from_fixture(fx, "cpu", "sunrgbd")
        args.loss_2dalignment_weight = 0.0
        model.eval()
        crit = crit_mod.build_criterion(args, cfg)
        losses.append(_step(model, crit, {k: v[r: r + 1] for k, v in full.items()}).item())
        for n, p in model.named_parameters():
            if p.grad is not None:
                ref[n] = ref.get(n, 0) + p.grad / WORLD
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ddp_rank, args=(_free_port(), d), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(d, f"ddp{r}.pt"), weights_only=True) for r in range(WORLD)]
    assert set(res[0]["grads"]) == set(ref)
    checked = 0
    for n, g in ref.items():
        g0, g1 = res[0]["grads"][n], res[1]["grads"][n]
        assert torch.equal(g0, g1), n          # DDP leaves identical gradients on every rank
        if g.abs().max() > 1e-8:
            assert rel_err(g0.numpy(), g.numpy()) < 1e-4, n
            checked += 1
    assert checked > 50
    for r in range(WORLD):
        assert abs(res[r]["loss"].item() - losses[r]) <= 1e-5 * abs(losses[r])


def _slice_outputs(out, r):
    """scene r of the model outputs (every tensor is (B, Q, ...))"""
    def one(d):
        return {k: v[r: r + 1] for k, v in d.items()}
    return {"outputs": one(out["outputs"]), "aux_outputs": [one(a) for a in out["aux_outputs"]]}


def _train_rank(rank, port, out_dir, mode="coalesced"):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    torch.set_num_threads(2)
    from oracle import torch_shim
    from helpers import batch_from_fixture as bff, build_model_from_fixture as bmf, fixture as fxl, ov3d as pkg
    _init(rank, port)
    torch_shim.install(pkg)
    from ov3d_amd.criterion import build_criterion
    fx = fxl("model_sun.npz")
    from full_fixture import float64_host
    model, cfg, args = bmf(fx, "cpu", "sunrgbd")
    args.loss_2dalignment_weight = 0.0
    model = model.double().train()   # batch-statistics BN; the fixture's dropouts are all 0
    # the reference's data-parallel semantics (main.py:427-431): SyncBatchNorm + the DDP
    # gradient mean.  The product's step has no DDP wrapper (torch's refuses SyncBatchNorm on
    # CPU modules anyway): ONE all-reduce of every gradient, averaged (FusedAdamW on the GPU,
    # dist.all_reduce_coalesced here)
    from ov3d_amd import dist as pdist
    model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
    crit = build_criterion(args, cfg)
    batch = {k: (v.double() if v.is_floating_point() else v)[rank: rank + 1]
             for k, v in bff(fx, "cpu").items()}
    order = {}
    if mode == "buckets":
        # dist.GradBuckets on a group of its own, bucket 0 (decoder side) started by the hook on
        # the encoder output's gradient; record what was final when it fired
        gb = pdist.GradBuckets(model.dp_buckets(),
                               group=torch.distributed.new_group(ranks=list(range(WORLD))))

        def flush():
            order["enc_grads_at_hook"] = sum(p.grad is not None for p in model.dp_buckets()[1])
            order["dec_grads_at_hook"] = sum(p.grad is not None for p in model.dp_buckets()[0])
        pdist.stage_after_encoder(model, gb, flush=flush)
    with float64_host():
        loss = _step(model, crit, batch)
    named = [(n, p) for n, p in model.named_parameters() if p.grad is not None]
    if mode == "buckets":
        order["launched_before_step"] = gb.launched(0)
        views = gb.finish()
        avg = [views[id(p)] / WORLD for _, p in named]
    else:
        avg = pdist.all_reduce_coalesced([p.grad for _, p in named], average=True)
    grads = {n: g.clone() for (n, _), g in zip(named, avg)}
    bufs = {n: b.clone() for n, b in model.named_buffers()}
    torch.save({"loss": loss.detach(), "grads": grads, "bufs": bufs, "order": order},
               os.path.join(out_dir, f"tr{rank}.pt"))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("mode", ["coalesced", "buckets"])
def test_ddp_syncbn_train_step_equals_global_batch(shim, monkeypatch, mode):
    """§8(e): 2 ranks x 1 scene (train mode: SyncBatchNorm batch statistics over both ranks,
    the gradient mean by one all-reduce, num_boxes all-reduced) == 1 process x 2 scenes,
    both in float64 (so ReLU / max-pool decisions cannot flip between the two orders of
    summation and the comparison is of the semantics: 1e-6, the few float32 roundings left
    on the host path -- the index ops' coordinates, the matcher cost -- turn 1e-16 summation-
    order differences into single float32 ulps): the same B=2 forward (BatchNorm
    over both scenes), each scene's loss with the global num_boxes, their mean backpropagated
    (what DDP's gradient average of the per-rank losses is).  Gradients, losses and the BN
    running statistics."""
    from ov3d_amd import criterion as crit_mod
    torch.set_num_threads(4)
    from full_fixture import float64_host
    fx = fixture("model_sun.npz")
    full = {k: (v.double() if v.is_floating_point() else v)
            for k, v in batch_from_fixture(fx, "cpu").items()}
    nbox = full["gt_box_present"].sum(dim=1)
    monkeypatch.setattr(crit_mod, "all_reduce_average", lambda t: nbox.sum() / WORLD)
    model, cfg, args = build_model_from_fixture(fx, "cpu", "sunrgbd")
    args.loss_2dalignment_weight = 0.0
    model = model.double().train()
    crit = crit_mod.build_criterion(args, cfg)
    with float64_host():
        out = model({k: full[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
        losses = []
        for r in range(WORLD):
            loss_r, _ = crit(_slice_outputs(out, r), {k: v[r: r + 1] for k, v in full.items()})
            losses.append(loss_r)
        (sum(losses) / WORLD).backward()
    ref = {n: p.grad for n, p in model.named_parameters() if p.grad is not None}
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_train_rank, args=(_free_port(), d, mode), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(d, f"tr{r}.pt"), weights_only=True) for r in range(WORLD)]
    if mode == "buckets":
        # bucket 0 left during the backward: the decoder side complete, the encoder side not
        # started (its gradients came after the hook)
        for r in range(WORLD):
            o = res[r]["order"]
            assert o["launched_before_step"] and o["enc_grads_at_hook"] == 0, o
            assert o["dec_grads_at_hook"] > 50, o
    assert set(res[0]["grads"]) == set(ref)
    checked = 0
    for n, g in ref.items():
        g0, g1 = res[0]["grads"][n], res[1]["grads"][n]
        assert torch.equal(g0, g1), n
        if g.abs().max() > 1e-8:
            err = (g0.double() - g.double()).norm() / g.double().norm()
            assert err < 1e-6, (n, err.item())
            checked += 1
    assert checked > 50
    for r in range(WORLD):
        assert abs(res[r]["loss"].item() - losses[r].item()) <= 1e-9 * abs(losses[r].item())
    # SyncBN running statistics == plain BN's over the whole batch, identical on both ranks
    nb = 0
    for n, b in model.named_buffers():
        if n.endswith(("running_mean", "running_var")):
            torch.testing.assert_close(res[0]["bufs"][n], b, rtol=1e-7, atol=1e-12, msg=n)
            assert torch.equal(res[0]["bufs"][n], res[1]["bufs"][n]), n
            nb += 1
    assert nb >= 16


def _syncbn_rank(rank, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import ov3d_import
    ov3d_import.load()
    dist = _init(rank, port)
    res = {}
    for name, kw in (("cma", dict(momentum=None)), ("noaffine", dict(affine=False)),
                     ("plain", dict())):
        g = torch.Generator().manual_seed(5)
        xs = [torch.randn(2, 7, 6, generator=g, dtype=torch.float64) * 3 + 1 for _ in range(2)]
        bn = torch.nn.SyncBatchNorm(6, **kw).double()
        if bn.weight is not None:
            with torch.no_grad():
                bn.weight.uniform_(0.5, 1.5, generator=g)
                bn.bias.uniform_(-1, 1, generator=g)
        bn.train()
        outs = []
        for x in xs:   # two steps: the cumulative-average momentum changes between them
            xr = x[rank].clone().requires_grad_(True)
            y = dist.sync_batch_norm_rows(bn, xr)
            (y * torch.arange(1.0, 7.0, dtype=torch.float64)).sum().backward()
            outs.append(y.detach())
        res[name] = dict(y=torch.stack(outs).tolist(), gx=xr.grad.tolist(),
                         rm=bn.running_mean.tolist(), rv=bn.running_var.tolist(),
                         gw=None if bn.weight is None else bn.weight.grad.tolist())
    with open(os.path.join(out_dir, f"sbn{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    torch.distributed.destroy_process_group()


def test_syncbn_rows_momentum_none_and_no_affine_world2():
    """dist.sync_batch_norm_rows at world 2 equals torch BatchNorm1d on the global batch for
    momentum=None (cumulative average, 1/num_batches_tracked) and affine=False;
    the weight gradient is rank-local as in torch's SyncBatchNorm (sum over ranks = global)."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_syncbn_rank, args=(_free_port(), d), nprocs=WORLD, join=True)
        got = [json.load(open(os.path.join(d, f"sbn{r}.json"))) for r in range(WORLD)]
    for name, kw in (("cma", dict(momentum=None)), ("noaffine", dict(affine=False)),
                     ("plain", dict())):
        g = torch.Generator().manual_seed(5)
        xs = [torch.randn(2, 7, 6, generator=g, dtype=torch.float64) * 3 + 1 for _ in range(2)]
        bn = torch.nn.BatchNorm1d(6, **kw).double()
        if bn.weight is not None:
            with torch.no_grad():
                bn.weight.uniform_(0.5, 1.5, generator=g)
                bn.bias.uniform_(-1, 1, generator=g)
        bn.train()
        for step, x in enumerate(xs):
            xr = x.reshape(14, 6).clone().requires_grad_(True)
            y = bn(xr)
            (y * torch.arange(1.0, 7.0, dtype=torch.float64)).sum().backward()
            for r in range(WORLD):
                np.testing.assert_allclose(got[r][name]["y"][step], y.detach()[7 * r: 7 * r + 7],
                                           rtol=1e-9, atol=1e-9)
        for r in range(WORLD):
            np.testing.assert_allclose(got[r][name]["gx"], xr.grad[7 * r: 7 * r + 7], atol=1e-9)
            np.testing.assert_allclose(got[r][name]["rm"], bn.running_mean, rtol=1e-9, atol=1e-12)
            np.testing.assert_allclose(got[r][name]["rv"], bn.running_var, rtol=1e-9, atol=1e-12)
        if bn.weight is not None:
            gw = np.add(got[0][name]["gw"], got[1][name]["gw"])
            np.testing.assert_allclose(gw, bn.weight.grad, rtol=1e-9, atol=1e-9)
        else:
            assert got[0][name]["gw"] is None


def test_capture_safe_env_forces_event_cache_off(monkeypatch):
    """dist.capture_safe_env overrides an environment that switched ProcessGroupNCCL's event
    cache on (a recycled event inside a captured step aborted the process, DESIGN.md Multi-GPU)"""
    from ov3d_amd import dist as pdist
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "1")
    with pytest.warns(UserWarning, match="TORCH_NCCL_CUDA_EVENT_CACHE"):
        pdist.capture_safe_env()
    assert os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] == "0"
    monkeypatch.delenv("TORCH_NCCL_CUDA_EVENT_CACHE")
    pdist.capture_safe_env()
    assert os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] == "0"
