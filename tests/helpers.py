"""Shared test helpers: fixture loading and building the product model from a
reference fixture (state dict loaded strict, so key compatibility is tested)."""
import argparse
import ast
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)

import ov3d_import  # noqa: E402

ov3d = ov3d_import.load()


def fixture(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def fixture_args(fx):
    items = ast.literal_eval(str(fx["args"]))
    return argparse.Namespace(**dict(items))


def fixture_prefix(fx, prefix):
    return {k[len(prefix):]: v for k, v in fx.items() if k.startswith(prefix)}


def build_model_from_fixture(fx, device, dataset):
    from ov3d_amd.dataset_config import CONFIGS
    from ov3d_amd.model_3detr import build_3detr
    args = fixture_args(fx)
    cfg = CONFIGS[dataset]()
    model, _ = build_3detr(args, cfg, text_embedding=torch.from_numpy(fx["text"]))
    sd = {k: torch.from_numpy(v) for k, v in fixture_prefix(fx, "sd/").items()}
    missing, unexpected = model.load_state_dict(sd, strict=True)
    assert not missing and not unexpected
    return model.to(device), cfg, args


def batch_from_fixture(fx, device):
    return {k: torch.from_numpy(v).to(device) for k, v in fixture_prefix(fx, "in/").items()}


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))
