"""Plain-PyTorch fp32 restatement of CLIPFastRCNN.inference for the GT-crop feature
extraction used at criterion.py:397 [upstream RegionCLIP; PARITY UNPINNED: RegionCLIP,
detectron2 and its weights are not available offline].

Test infrastructure only.  Functional: it reads the weight tensors from the module's
state dict by their upstream key names and runs its own statement of the published
architecture [upstream CLIP model.py ModifiedResNet / Bottleneck / AttentionPool2d,
detectron2 FrozenBatchNorm2d, RegionCLIP CLIPRes5ROIHeads with ROIAlignV2] with
torch.nn.functional ops: NCHW convolutions with unfolded frozen BN, per-image
preprocessing and padding, ROIAlign from the C oracle (oracle/ov3d_oracle.c), res5 as
the backbone's layer4 blocks and the attention pool through
``F.multi_head_attention_forward`` over all 82 tokens.  None of the product's modules
(``backbone``, ``layer4``, ``attnpool`` forward methods) and none of its fusions (folded
BN, NHWC rows, one backbone pass, the first-query pool) are used.
"""
import re

import numpy as np
import torch
import torch.nn.functional as F

from oracle import oracle as O

BN_EPS = 1e-5   # detectron2 FrozenBatchNorm2d default


def frozen_bn(sd, prefix, x):
    """detectron2 FrozenBatchNorm2d: x * w / sqrt(var + eps) + (b - mean * w / sqrt(var + eps))"""
    scale = sd[prefix + ".weight"] * (sd[prefix + ".running_var"] + BN_EPS).rsqrt()
    shift = sd[prefix + ".bias"] - sd[prefix + ".running_mean"] * scale
    return x * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)


def bottleneck(sd, prefix, x, stride):
    """CLIP Bottleneck: 1x1 -> 3x3 (stride 1) -> avgpool(stride) -> 1x1 (x4), downsample
    branch avgpool(stride) -> 1x1 -> BN whenever it exists in the weights"""
    out = F.relu(frozen_bn(sd, prefix + ".bn1", F.conv2d(x, sd[prefix + ".conv1.weight"])))
    out = F.relu(frozen_bn(sd, prefix + ".bn2", F.conv2d(out, sd[prefix + ".conv2.weight"], padding=1)))
    if stride > 1:
        out = F.avg_pool2d(out, stride)
    out = frozen_bn(sd, prefix + ".bn3", F.conv2d(out, sd[prefix + ".conv3.weight"]))
    idn = x
    if prefix + ".downsample.0.weight" in sd:
        idn = F.avg_pool2d(x, stride) if stride > 1 else x
        idn = frozen_bn(sd, prefix + ".downsample.1", F.conv2d(idn, sd[prefix + ".downsample.0.weight"]))
    return F.relu(out + idn)


def res_layer(sd, name, x):
    """layer1 (stride 1) / layer2..4 (stride 2 in the first block), blocks from the keys"""
    n = 1 + max(int(m.group(1)) for k in sd
                for m in [re.match(re.escape(name) + r"\.(\d+)\.conv1\.weight$", k)] if m)
    stride = 1 if name.endswith("layer1") else 2
    for i in range(n):
        x = bottleneck(sd, f"{name}.{i}", x, stride if i == 0 else 1)
    return x


def stem(sd, p, x):
    x = F.relu(frozen_bn(sd, p + "bn1", F.conv2d(x, sd[p + "conv1.weight"], stride=2, padding=1)))
    x = F.relu(frozen_bn(sd, p + "bn2", F.conv2d(x, sd[p + "conv2.weight"], padding=1)))
    x = F.relu(frozen_bn(sd, p + "bn3", F.conv2d(x, sd[p + "conv3.weight"], padding=1)))
    return F.avg_pool2d(x, 2)


def attnpool(sd, p, x, num_heads):
    """CLIP AttentionPool2d on NCHW x: mean token + positional embedding, full MHA over all
    tokens, token 0 of the output"""
    x = x.flatten(start_dim=2).permute(2, 0, 1)                 # (HW, N, C)
    x = torch.cat([x.mean(dim=0, keepdim=True), x], dim=0)
    x = x + sd[p + "positional_embedding"][:, None, :]
    out, _ = F.multi_head_attention_forward(
        query=x, key=x, value=x, embed_dim_to_check=x.shape[-1], num_heads=num_heads,
        q_proj_weight=sd[p + "q_proj.weight"], k_proj_weight=sd[p + "k_proj.weight"],
        v_proj_weight=sd[p + "v_proj.weight"], in_proj_weight=None,
        in_proj_bias=torch.cat([sd[p + "q_proj.bias"], sd[p + "k_proj.bias"], sd[p + "v_proj.bias"]]),
        bias_k=None, bias_v=None, add_zero_attn=False, dropout_p=0.0,
        out_proj_weight=sd[p + "c_proj.weight"], out_proj_bias=sd[p + "c_proj.bias"],
        use_separate_proj_weight=True, training=False, need_weights=False)
    return out[0]


def preprocess(mean, std, images):
    """list of (3,H,W) 0-255 -> (N,3,Hp,Wp) normalised, zero padded (ImageList.from_tensors)."""
    xs = [((im.float() / 255.0) - mean.to(im.device)) / std.to(im.device) for im in images]
    H = max(x.shape[1] for x in xs)
    W = max(x.shape[2] for x in xs)
    out = xs[0].new_zeros((len(xs), 3, H, W))
    for i, x in enumerate(xs):
        out[i, :, : x.shape[1], : x.shape[2]] = x
    return out


@torch.no_grad()
def inference(model, batched_inputs):
    """-> (sum Q, output_dim) f32, same contract as RegionCLIP.inference."""
    sd = {k: v.float() for k, v in model.state_dict().items()}
    p = "backbone."
    heads = model.backbone.attnpool.num_heads
    images = [x["image"] for x in batched_inputs]
    x = preprocess(model.pixel_mean.float(), model.pixel_std.float(), images)
    x = stem(sd, p, x.float())
    for name in ("layer1", "layer2", "layer3"):
        x = res_layer(sd, p + name, x)
    res4 = x                                                            # NCHW f32, stride 16
    feats = res4.permute(0, 2, 3, 1).contiguous().cpu().numpy()
    outs = []
    for i, inp in enumerate(batched_inputs):
        boxes = inp["instances"].gt_boxes.tensor.float().cpu().numpy()
        if boxes.shape[0] == 0:
            continue
        rois = O.roi_align(feats[i:i + 1], boxes, per_image=boxes.shape[0], nimages=1,
                           spatial_scale=model.spatial_scale, pooled=model.pooler_resolution)
        r = torch.from_numpy(np.ascontiguousarray(rois.transpose(0, 3, 1, 2))).to(res4.device)
        outs.append(attnpool(sd, p + "attnpool.", res_layer(sd, p + "layer4", r), heads))
    return torch.cat(outs)
