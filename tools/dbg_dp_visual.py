"""Debug: where do the two-rank and the one-process bf16 steps part for the visual head?
Compares, per scene, the final layer's sem_cls_logits / visual_embeds and their gradients."""
import os
import sys
import tempfile

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import test_dp_world2_gpu as T  # noqa: E402

KEYS = ("sem_cls_logits", "visual_embeds", "center_normalized")


def _rank(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE="2", LOCAL_RANK="0")
    torch.distributed.init_process_group("gloo", init_method="env://", world_size=2, rank=rank)
    model, crit, batch, dev = T._setup()
    model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
    b = {k: v[rank: rank + 1] for k, v in batch.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = model(T._inputs(b))
    st = out["_layers_stacked"]
    for k in KEYS:
        st[k].retain_grad()
    loss, _ = crit(out, b)
    loss.backward()
    g0 = lambda t: (t.grad if t.grad is not None else torch.zeros_like(t)).float().cpu()  # noqa: E731
    torch.save({k: (st[k].detach().float().cpu(), g0(st[k])) for k in KEYS},
               os.path.join(out_dir, f"r{rank}.pt"))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def main():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank, args=(T._free_port(), d), nprocs=2, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]
    from ov3d_amd import criterion as crit_mod
    from ov3d_amd import dist as pdist
    model, crit, batch, dev = T._setup()
    nbox = batch["gt_box_present"].sum(dim=1)
    crit_mod.all_reduce_average = pdist.all_reduce_average = lambda t: nbox.sum() / 2
    pdist.get_world_size = lambda: 2
    for amp in (True, False):
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = model(T._inputs(batch))
        st = out["_layers_stacked"]
        for k in KEYS:
            st[k].retain_grad()
        losses = [crit(T._slice_outputs(out, r), {k: v[r: r + 1] for k, v in batch.items()})[0]
                  for r in range(2)]
        (sum(losses) / 2).backward()
        for k in KEYS:
            for r in range(2):
                v, g = res[r][k]
                gg = st[k].grad if st[k].grad is not None else torch.zeros_like(st[k])
                sv, sg = st[k].detach().float().cpu()[:, r:r + 1], gg.float().cpu()[:, r:r + 1] * 2
                ev = ((v - sv).norm() / sv.norm()).item()
                eg = ((g - sg).norm() / sg.norm().clamp_min(1e-30)).item()
                print("amp" if amp else "fp32", k, "scene", r, "value err %.3e grad err %.3e |g| %.3e/%.3e"
                      % (ev, eg, g.norm().item(), sg.norm().item()))


if __name__ == "__main__":
    main()
