"""Deterministic stand-in for RegionCLIP's ``clip.inference`` (test infrastructure).

RegionCLIP (detectron2 CLIPFastRCNN + RN50x4 weights) is not available
offline, so the parity fixtures pin the 2D-alignment branch with a fixed,
box-dependent feature map: feats = tanh(((box / [w,h,w,h]) - 0.5) @ W), W seeded.
This pins the projection (quirk Q4), the clamp, the scene-major/box-minor row
order and the cosine loss of criterion.py:132-140, 366-398.
"""
import torch


class FakeRegionCLIP:
    def __init__(self, dim=640, seed=11):
        g = torch.Generator().manual_seed(seed)
        self.W = torch.randn(4, dim, generator=g)
        self.calls = 0

    def inference(self, batch, do_postprocess=False):
        self.calls += 1
        feats = []
        for d in batch:
            inst = d["instances"]
            boxes = inst.gt_boxes.tensor.to(torch.float32)   # float32 features in any run
            H, W = d["image"].shape[1], d["image"].shape[2]
            scale = torch.tensor([W, H, W, H], dtype=boxes.dtype, device=boxes.device)
            feats.append(torch.tanh((boxes / scale - 0.5) @ self.W.to(boxes.device)))
        return torch.cat(feats, 0)
