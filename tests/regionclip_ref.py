"""Plain-PyTorch fp32 restatement of CLIPFastRCNN.inference for the GT-crop feature
extraction used at criterion.py:397 [upstream RegionCLIP; PARITY UNPINNED: RegionCLIP,
detectron2 and its weights are not available offline].

Test infrastructure only.  It runs the module's own reference-formulation layers:
NCHW convolutions with unfolded frozen BN, per-image preprocessing and padding,
ROIAlign from the C oracle (oracle/ov3d_oracle.c), ``layer4`` as res5 and CLIP's
AttentionPool2d through ``F.multi_head_attention_forward`` — i.e. none of the
product's fusions (folded BN, NHWC rows, one backbone pass, reassociated pool).
"""
import numpy as np
import torch

from oracle import oracle as O


def preprocess(model, images):
    """list of (3,H,W) 0-255 -> (N,3,Hp,Wp) normalised, zero padded (ImageList.from_tensors)."""
    xs = [((im.float() / 255.0) - model.pixel_mean.to(im.device)) / model.pixel_std.to(im.device)
          for im in images]
    H = max(x.shape[1] for x in xs)
    W = max(x.shape[2] for x in xs)
    out = xs[0].new_zeros((len(xs), 3, H, W))
    for i, x in enumerate(xs):
        out[i, :, : x.shape[1], : x.shape[2]] = x
    return out


@torch.no_grad()
def inference(model, batched_inputs):
    """-> (sum Q, output_dim) f32, same contract as RegionCLIP.inference."""
    bb = model.backbone
    images = [x["image"] for x in batched_inputs]
    x = preprocess(model, images)
    res4 = bb(x.float())["res4"]                                       # NCHW f32
    feats = res4.permute(0, 2, 3, 1).contiguous().cpu().numpy()
    outs = []
    for i, inp in enumerate(batched_inputs):
        boxes = inp["instances"].gt_boxes.tensor.float().cpu().numpy()
        if boxes.shape[0] == 0:
            continue
        rois = O.roi_align(feats[i:i + 1], boxes, per_image=boxes.shape[0], nimages=1,
                           spatial_scale=model.spatial_scale, pooled=model.pooler_resolution)
        r = torch.from_numpy(np.ascontiguousarray(rois.transpose(0, 3, 1, 2))).to(res4.device)
        outs.append(bb.attnpool(bb.layer4(r)))
    return torch.cat(outs)
