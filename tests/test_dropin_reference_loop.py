"""Drop-in proof: the REFERENCE's own training and evaluation loops
(/root/reference/engine.py:47-150 train_one_epoch, :154-231 evaluate), imported unchanged,
drive the product model and criterion through INTEGRATION.md §2's bindings:
``build_model`` / ``build_criterion`` from ov3d_amd and ``utils.dist`` aliased to
ov3d_amd.dist.  The HIP index ops come from the C oracle (oracle/torch_shim.py: this is the
CPU suite).  The losses the loop computes equal a direct product step on the same weights
and batches, and the reference's own APCalculator consumes the product's outputs.

Runs in this container only (it imports /root/reference; skipped where that is absent,
e.g. on the GPU box)."""
import argparse
import copy
import importlib.util
import os
import sys

import pytest
import torch

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference sources")


class _Logger:
    def __init__(self):
        self.scalars = []

    def log_scalars(self, d, step, prefix=None):
        self.scalars.append((prefix, step, {k: float(v) for k, v in d.items()}))


def _args():
    return argparse.Namespace(
        model_name="3detr", enc_type="vanilla", enc_nlayers=3, enc_dim=64, enc_ffn_dim=64,
        enc_dropout=0.0, enc_nhead=4, enc_activation="relu", dec_nlayers=8, dec_dim=64,
        dec_ffn_dim=64, dec_dropout=0.0, dec_nhead=4, mlp_dropout=0.0, preenc_npoints=256,
        nqueries=32, use_color=False, matcher_giou_cost=3.0, matcher_cls_cost=1.0,
        matcher_center_cost=5.0, matcher_objectness_cost=5.0, loss_giou_weight=0.0,
        loss_sem_cls_weight=1.0, loss_no_object_weight=0.1, loss_angle_cls_weight=0.1,
        loss_angle_reg_weight=0.5, loss_center_weight=5.0, loss_size_weight=1.0,
        loss_2dalignment_weight=2e-4,
        # engine.py's schedule / logging arguments (main.py defaults)
        base_lr=5e-4, warm_lr=1e-6, warm_lr_epochs=9, final_lr=1e-6, max_epoch=720,
        clip_gradient=0.1, log_every=10, log_metrics_every=20, use_pseudo_labels=False)


@pytest.fixture()
def reference_engine(monkeypatch):
    from helpers import ov3d
    from ref_loader import load_reference
    from oracle import torch_shim
    load_reference()
    import ov3d_amd.dist
    # the reference's utils/dist.py -> ov3d_amd.dist
    monkeypatch.setitem(sys.modules, "utils.dist", ov3d_amd.dist)
    spec = importlib.util.spec_from_file_location("ref_engine", os.path.join(REF, "engine.py"))
    eng = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(eng)
    saved = torch_shim.install(ov3d)
    # engine.py logs torch.cuda.max_memory_allocated() (0 on the host)
    monkeypatch.setattr(torch.cuda, "max_memory_allocated", lambda *a, **k: 0)
    yield eng
    torch_shim.uninstall(saved)


def _batches():
    from ov3d_amd import synthetic
    from make_golden import small_images
    out = []
    for s in (31, 32):
        b = synthetic.make_batch(2, seed=s, num_points=2048)
        out.append(small_images(b, 2))
    return out


def test_reference_train_and_eval_loops_drive_the_product(reference_engine):
    from fake_clip import FakeRegionCLIP
    from ov3d_amd import build_criterion, build_model, synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    torch.set_num_threads(8)
    args = _args()
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(7)
    model, _ = build_model(args, cfg, text_embedding=synthetic.text_embedding(21, 640))
    twin = copy.deepcopy(model)
    crit = build_criterion(args, cfg)
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=args.base_lr, weight_decay=0.1)
    batches = _batches()
    seen = []

    class Recording(torch.nn.Module):          # the loop's criterion, recording its losses
        def __init__(self, c):
            super().__init__()
            self.c = c

        def forward(self, *a, **k):
            loss, ld = self.c(*a, **k)
            seen.append((loss.item(), len(ld)))
            return loss, ld

    logger = _Logger()
    apc = reference_engine.train_one_epoch(args, 0, model, FakeRegionCLIP(), None, opt,
                                           Recording(crit), cfg,
                                           [{k: v.clone() for k, v in b.items()} for b in batches],
                                           logger)
    assert len(seen) == 2 and all(n == 56 for _, n in seen)
    assert apc.scan_cnt == 2        # the reference's APCalculator metered the product's outputs
    assert any(p == "Train/" for p, _, _ in logger.scalars)
    # the same two steps called directly on the product (twin weights, same optimizer)
    opt2 = torch.optim.AdamW([p for p in twin.parameters() if p.requires_grad], lr=args.base_lr,
                             weight_decay=0.1)
    for it, b in enumerate(batches):
        lr = reference_engine.compute_learning_rate(args, it / (args.max_epoch * 2))
        for g in opt2.param_groups:
            g["lr"] = lr
        opt2.zero_grad()
        out = twin({k: b[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
        loss, _ = crit(out, dict(b), clip=FakeRegionCLIP())
        loss.backward()
        torch.nn.utils.clip_grad_norm_(twin.parameters(), args.clip_gradient)
        opt2.step()
        assert loss.item() == seen[it][0], (it, loss.item(), seen[it][0])
    for (n, p), (_, q) in zip(model.named_parameters(), twin.named_parameters()):
        assert torch.equal(p, q), n
    # evaluation loop (exact AP calculator of the reference) over the product's eval outputs
    apc = reference_engine.evaluate(args, 1, model, FakeRegionCLIP(), crit, cfg,
                                    [{k: v.clone() for k, v in b.items()} for b in batches],
                                    _Logger(), 2)
    assert apc.scan_cnt == 4   # 2 batches x 2 scenes
