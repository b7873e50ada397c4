"""RegionCLIP ROI-feature extractor for the 2D-alignment loss.

Replaces ``build_model(args, cfg, model_name="regionclip")`` (main.py:422 ->
models/model_regionclip.py:15-22), i.e. detectron2's ``CLIPFastRCNN`` with
``CLIPRes5ROIHeads_FeatureExtraction`` and ``CROP_REGION_TYPE GT`` as configured
in README.md:29-36, and its one call site ``clip.inference(batched_inputs,
do_postprocess=False)`` (criterion.py:397).  RegionCLIP/detectron2 are not
vendored and no weights are available offline: the architecture below restates
the published upstream code [upstream RegionCLIP clip_backbone.ModifiedResNet
+ CLIPRes5ROIHeads; CLIP RN50x4], numerics are "parity unpinned", and the
module is random-initialised (seeded) unless a checkpoint is loaded.

    images (B,3,H,W) float 0-255 -> (v/255 - mean)/std, zero-pad to the batch max
    -> ModifiedResNet stem + res2..res4 (stride 16, 1280 ch; frozen BN)
    -> ROIAlignV2 18x18 (aligned, adaptive sampling) of each GT box
    -> res5 = backbone.layer4 (2560 ch, 9x9) -> attnpool (CLIP AttentionPool2d) -> 640-d

MI355X path (``region_features``), output-identical up to float rounding:
  * the backbone runs ONCE per training step: the reference calls
    ``clip.inference`` once per decoder layer (8x, criterion.py:432-442) on the
    same images;
  * image unpack + normalise + pad is one HIP kernel (``ov3d_clip_preprocess``),
    activations stay channels-last (NHWC) end to end, frozen BN is folded into
    the convolution weights;
  * ROIAlign for all L*B*Q boxes is one HIP launch (``ov3d_roi_align_fwd``)
    writing the (R,18,18,1280) rows the res5 GEMMs read;
  * res5 runs once over all L*B*Q ROIs on the hand-written 256 x 256 tile kernel
    (csrc/gemm256.hip: 1x1 convs as GEMMs on rows with bias / identity / ReLU in the
    epilogue, 3x3 convs as implicit GEMMs over the NHWC rows), bf16 with fp32
    accumulation; the backbone's narrow 3x3 convs (Cin % 64 != 0) as HIP im2col +
    the same kernel;
  * the attention pool only ever needs its first query (``x[0]``): with
    a_h = Wk_h^T q_h the scores are a_h . t_j (the q_h . bk_h term is constant
    over j and cancels in the softmax) and the output is Wv_h (sum_j p_hj t_j)
    + bv_h, so neither K nor V is projected for the 82 tokens: 2.2 GFLOP ->
    0.08 GFLOP per ROI; the scores, softmax and p.t of all heads are one HIP
    launch that builds the token rows on chip (csrc/attnpool.hip).
"""
import math
import os
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native
from . import gemm

# RegionCLIP CLIP configs: PIXEL_MEAN / PIXEL_STD of CLIP, images divided by 255
CLIP_PIXEL_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_PIXEL_STD = (0.26862954, 0.26130258, 0.27577711)
# MODEL.RESNETS.DEPTH -> (layers, width) [upstream build_clip_resnet_backbone]
CLIP_RESNETS = {50: ((3, 4, 6, 3), 64), 101: ((3, 4, 23, 3), 64), 200: ((4, 6, 10, 6), 80)}


class FrozenBatchNorm2d(nn.Module):
    """detectron2.layers.FrozenBatchNorm2d: y = x * scale + shift with fixed statistics."""

    def __init__(self, num_features, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.register_buffer("weight", torch.ones(num_features))
        self.register_buffer("bias", torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features) - eps)

    def scale_shift(self):
        scale = self.weight * (self.running_var + self.eps).rsqrt()
        return scale, self.bias - self.running_mean * scale

    def forward(self, x):
        scale, shift = self.scale_shift()
        return x * scale.view(1, -1, 1, 1).to(x.dtype) + shift.view(1, -1, 1, 1).to(x.dtype)


class Bottleneck(nn.Module):
    """CLIP ModifiedResNet bottleneck: anti-aliased strided conv (avgpool before the
    stride-1 conv3) and an avgpool + 1x1 conv downsample."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = FrozenBatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1, bias=False)
        self.bn2 = FrozenBatchNorm2d(planes)
        self.avgpool = nn.AvgPool2d(stride) if stride > 1 else nn.Identity()
        self.conv3 = nn.Conv2d(planes, planes * self.expansion, 1, bias=False)
        self.bn3 = FrozenBatchNorm2d(planes * self.expansion)
        self.stride = stride
        self.downsample = None
        if stride > 1 or inplanes != planes * self.expansion:
            self.downsample = nn.Sequential(OrderedDict([
                ("-1", nn.AvgPool2d(stride)),
                ("0", nn.Conv2d(inplanes, planes * self.expansion, 1, stride=1, bias=False)),
                ("1", FrozenBatchNorm2d(planes * self.expansion))]))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.avgpool(out)
        out = self.bn3(self.conv3(out))
        identity = x if self.downsample is None else self.downsample(x)
        return F.relu(out + identity)


class AttentionPool2d(nn.Module):
    """CLIP AttentionPool2d (mean token + positional embedding, MHA, output of token 0)."""

    def __init__(self, spacial_dim, embed_dim, num_heads, output_dim=None):
        super().__init__()
        self.positional_embedding = nn.Parameter(torch.randn(spacial_dim ** 2 + 1, embed_dim)
                                                 / embed_dim ** 0.5)
        self.k_proj = nn.Linear(embed_dim, embed_dim)
        self.q_proj = nn.Linear(embed_dim, embed_dim)
        self.v_proj = nn.Linear(embed_dim, embed_dim)
        self.c_proj = nn.Linear(embed_dim, output_dim or embed_dim)
        self.num_heads = num_heads

    def forward(self, x):
        """Reference formulation (NCHW input) -> (N, output_dim)."""
        x = x.flatten(start_dim=2).permute(2, 0, 1)
        x = torch.cat([x.mean(dim=0, keepdim=True), x], dim=0)
        x = x + self.positional_embedding[:, None, :].to(x.dtype)
        x, _ = F.multi_head_attention_forward(
            query=x, key=x, value=x, embed_dim_to_check=x.shape[-1], num_heads=self.num_heads,
            q_proj_weight=self.q_proj.weight, k_proj_weight=self.k_proj.weight,
            v_proj_weight=self.v_proj.weight, in_proj_weight=None,
            in_proj_bias=torch.cat([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias]),
            bias_k=None, bias_v=None, add_zero_attn=False, dropout_p=0.0,
            out_proj_weight=self.c_proj.weight, out_proj_bias=self.c_proj.bias,
            use_separate_proj_weight=True, training=self.training, need_weights=False)
        return x[0]


class ModifiedResNet(nn.Module):
    """CLIP ModifiedResNet as RegionCLIP's C4 backbone (out_features ['res4'], layer4 and
    attnpool reused by the ROI heads)."""

    def __init__(self, layers=(4, 6, 10, 6), output_dim=640, heads=40, input_resolution=288,
                 width=80):
        super().__init__()
        self.conv1 = nn.Conv2d(3, width // 2, 3, stride=2, padding=1, bias=False)
        self.bn1 = FrozenBatchNorm2d(width // 2)
        self.conv2 = nn.Conv2d(width // 2, width // 2, 3, padding=1, bias=False)
        self.bn2 = FrozenBatchNorm2d(width // 2)
        self.conv3 = nn.Conv2d(width // 2, width, 3, padding=1, bias=False)
        self.bn3 = FrozenBatchNorm2d(width)
        self.avgpool = nn.AvgPool2d(2)
        self._inplanes = width
        self.layer1 = self._make_layer(width, layers[0])
        self.layer2 = self._make_layer(width * 2, layers[1], stride=2)
        self.layer3 = self._make_layer(width * 4, layers[2], stride=2)
        self.layer4 = self._make_layer(width * 8, layers[3], stride=2)
        self.attnpool = AttentionPool2d(input_resolution // 32, width * 32, heads, output_dim)
        self.size_divisibility = 0

    def _make_layer(self, planes, blocks, stride=1):
        layers = [Bottleneck(self._inplanes, planes, stride)]
        self._inplanes = planes * Bottleneck.expansion
        layers += [Bottleneck(self._inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def stem(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.relu(self.bn2(self.conv2(x)))
        x = F.relu(self.bn3(self.conv3(x)))
        return self.avgpool(x)

    def forward(self, x):
        x = self.stem(x.to(self.conv1.weight.dtype))
        return {"res4": self.layer3(self.layer2(self.layer1(x)))}


def init_synthetic_(model, seed=11):
    """Seeded random weights for a checkpoint-free run (RN50x4 random-init,
    seed 11).  Convs: He-normal on fan-in; frozen BN: mild random affine statistics with
    the last BN of every residual branch at 0.5 so activations stay O(1) through 26
    blocks; attention pool as CLIP's initialize_parameters (std = C^-1/2)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, m in model.named_modules():
            if isinstance(m, nn.Conv2d):
                fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1]
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * math.sqrt(2.0 / fan_in))
            elif isinstance(m, FrozenBatchNorm2d):
                n = m.weight.numel()
                gain = 0.5 if name.startswith("layer") and name.endswith(".bn3") else 1.0
                m.weight.copy_(gain * (1 + 0.1 * torch.randn(n, generator=g)))
                m.bias.copy_(0.1 * torch.randn(n, generator=g))
                m.running_mean.copy_(0.1 * torch.randn(n, generator=g))
                m.running_var.copy_(1 + 0.1 * torch.rand(n, generator=g))
            elif isinstance(m, AttentionPool2d):
                C = m.q_proj.in_features
                std = C ** -0.5
                m.positional_embedding.copy_(torch.randn(m.positional_embedding.shape, generator=g) * std)
                for lin in (m.q_proj, m.k_proj, m.v_proj, m.c_proj):
                    lin.weight.copy_(torch.randn(lin.weight.shape, generator=g) * std)
                    lin.bias.copy_(0.02 * torch.randn(lin.bias.shape, generator=g))
    return model


class _Folded:
    """Inference weights: frozen BN folded into each conv (w*scale, shift), in the compute
    dtype; 1x1 convs as (Cout, Cin) matrices, 3x3 convs channels-last."""

    def __init__(self, backbone, dtype):
        self.dtype = dtype
        self.conv = {}
        for name, m in backbone.named_modules():
            if isinstance(m, Bottleneck):
                self._fold(name + ".conv1", m.conv1, m.bn1)
                self._fold(name + ".conv2", m.conv2, m.bn2)
                self._fold(name + ".conv3", m.conv3, m.bn3)
                if m.downsample is not None:
                    self._fold(name + ".down", m.downsample[1], m.downsample[2])
        self._fold("conv1", backbone.conv1, backbone.bn1)
        self._fold("conv2", backbone.conv2, backbone.bn2)
        self._fold("conv3", backbone.conv3, backbone.bn3)
        ap = backbone.attnpool
        C, H = ap.q_proj.in_features, ap.num_heads
        d = C // H
        f32 = torch.float32
        self.heads, self.head_dim = H, d
        self.pos = ap.positional_embedding.detach().to(dtype).contiguous()          # (T, C)
        self.wq = (ap.q_proj.weight.detach().float() * d ** -0.5).to(dtype)          # scaled q
        self.bq = (ap.q_proj.bias.detach().float() * d ** -0.5).to(dtype)
        self.wk = ap.k_proj.weight.detach().to(dtype).view(H, d, C)                 # (H, d, C)
        self.wkt = self.wk.transpose(1, 2).contiguous()                              # (H, C, d)
        self.wv = ap.v_proj.weight.detach().to(dtype).contiguous()                   # (H*d, C)
        self.wvt = ap.v_proj.weight.detach().to(dtype).view(H, d, C).transpose(1, 2).contiguous()
        self.bv = ap.v_proj.bias.detach().to(f32)
        self.wc = ap.c_proj.weight.detach().to(dtype)
        self.bc = ap.c_proj.bias.detach().to(dtype)

    def _fold(self, key, conv, bn):
        scale, shift = bn.scale_shift()
        w = conv.weight.detach().float() * scale.float().view(-1, 1, 1, 1)
        cout, cin = w.shape[:2]
        if w.shape[-1] == 1:
            w = w.view(cout, cin)
        else:   # (Cout, ky, kx, Cin) -> (Cout, Kpad): the im2col column order, K zero-padded
            kpad = (9 * cin + 15) // 16 * 16
            wm = w.new_zeros((cout, kpad))
            wm[:, : 9 * cin] = w.permute(0, 2, 3, 1).reshape(cout, 9 * cin)
            w = wm
        self.conv[key] = (w.to(self.dtype), shift.detach().to(self.dtype))


def _nchw(x):
    """(N,H,W,C) contiguous -> channels-last NCHW view (no copy)."""
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    """channels-last NCHW -> (N,H,W,C) view (copies only if x is not channels-last)."""
    return x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)


def _conv1x1(x, w, b, relu, residual=None):
    """1x1 conv on NHWC rows as one GEMM: (rows, Cin) @ (Cout, Cin)^T + b (+ residual), the
    bias and ReLU in the GEMM epilogue; with a residual (bf16) the identity is the GEMM's C.

    bf16 on the device (the product path) has ONE backend, the hand-written 256 x 256 tile
    kernel (csrc/gemm256.hip); a shape it rejects raises instead of falling back to a library
    GEMM.  fp32 (the parity tests' restatement dtype) runs torch's GEMM + ov3d_bias_residual_act."""
    shp = x.shape
    rows = x.reshape(-1, shp[-1])
    res = residual.reshape(-1, w.shape[0]) if residual is not None else None
    if x.dtype == torch.bfloat16 and x.is_cuda:
        if not gemm.gemm256_ok(rows, w, residual=res):
            raise _native.NativeError(
                f"regionclip 1x1 conv: gemm256 rejects rows {tuple(rows.shape)} stride "
                f"{rows.stride()} x weight {tuple(w.shape)} stride {w.stride()} (bf16 rows, "
                "K % 8 == 0, N % 8 == 0, 16-byte aligned; OV3D_GEMM256=1)")
        return gemm.gemm256(rows, w, bias=b, residual=res, relu=relu).view(*shp[:-1], w.shape[0])
    if res is None:
        y = torch._addmm_activation(b, rows, w.t()) if relu else torch.addmm(b, rows, w.t())
    else:
        res = _native.check(res, "residual", ndim=2)
        y = torch.mm(rows, w.t())
        _native.call("ov3d_bias_residual_act", y, y.element_size(), y.shape[0], y.shape[1], b,
                     res, int(relu), like=y)
    return y.view(*shp[:-1], w.shape[0])


# im2col chunk budget.  Whole convolutions (16 GB: res5's first 3x3 over 4096 ROIs is 15.3 GB of
# columns) beat Infinity-Cache-sized 96 MB chunks: one K = 5760 GEMM reaches ~1130 TFLOP/s where
# 8100-row chunks ran at ~650, and the columns' HBM round trip costs less than the difference
# (C5 step 70.3 -> 67.6 ms).  OV3D_IM2COL_CHUNK_MB overrides.
IM2COL_CHUNK_BYTES = int(os.environ.get("OV3D_IM2COL_CHUNK_MB", "16384")) << 20


# im2col of chunk i + 1 on a side stream while the GEMM of chunk i runs (two column buffers):
# the byte-moving im2col hides behind the matrix-core GEMM (OV3D_CONV_OVERLAP=0: in series)
CONV_OVERLAP = os.environ.get("OV3D_CONV_OVERLAP", "1") != "0"

# the attention pool's scores / softmax / p.t in one launch over on-chip token rows
# (csrc/attnpool.hip); OV3D_FUSED_POOL=0: the token rows + library bmm's (_pool_tokens)
FUSED_POOL = os.environ.get("OV3D_FUSED_POOL", "1") != "0"
_SIDE = {}


def _side_stream(device):
    s = _SIDE.get(device)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _SIDE[device] = s
    return s


_BUDGET = {}


def _im2col_budget(device):
    """the column-buffer budget: IM2COL_CHUNK_BYTES, at most an eighth of the device's memory
    (two buffers are live when the chunks overlap; the caching allocator keeps them)"""
    b = _BUDGET.get(device)
    if b is None:
        total = torch.cuda.get_device_properties(device).total_memory
        b = _BUDGET[device] = min(IM2COL_CHUNK_BYTES, total // 8)
    return b


def _conv3x3(x, w, b, stride=1):
    """3x3 conv (pad 1) + bias + ReLU on NHWC: HIP im2col of a chunk of images / ROIs,
    then one hipBLASLt GEMM with the ReLU epilogue writing the chunk's output rows; with
    several chunks the next chunk's im2col runs on a side stream beside this chunk's GEMM."""
    N, H, W, C = x.shape
    cout, kpad = w.shape
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    x = _native.check(x.contiguous(), "conv input", ndim=4)
    if stride == 1 and gemm.conv3x3_ok(x, w):
        # implicit GEMM: the 3x3 taps are read straight from the NHWC rows (no column matrix)
        return gemm.conv3x3_gemm256(x, w, bias=b, relu=True)
    out = torch.empty((N, Ho, Wo, cout), dtype=x.dtype, device=x.device)
    per_img = Ho * Wo * kpad * x.element_size()
    step = max(1, _im2col_budget(x.device) // per_img)
    starts = list(range(0, N, step))
    overlap = CONV_OVERLAP and len(starts) > 1
    cols = [torch.empty((min(step, N) * Ho * Wo, kpad), dtype=x.dtype, device=x.device)
            for _ in range(2 if overlap else 1)]
    wt = w.t()
    main = torch.cuda.current_stream(x.device) if overlap else None
    side = _side_stream(x.device) if overlap else None
    freed = [None, None]    # event: the GEMM that last read column buffer j has been issued
    for ci, n0 in enumerate(starts):
        n = min(step, N - n0)
        c = cols[ci % len(cols)][: n * Ho * Wo]
        if overlap:
            j = ci % 2
            with torch.cuda.stream(side):
                side.wait_event(freed[j]) if freed[j] is not None else side.wait_stream(main)
                _native.call("ov3d_im2col3x3", x[n0:n0 + n], x.element_size(), n, H, W, C, stride,
                             kpad, c, like=x)
                ready = torch.cuda.Event()
                ready.record(side)
            main.wait_event(ready)
        else:
            _native.call("ov3d_im2col3x3", x[n0:n0 + n], x.element_size(), n, H, W, C, stride, kpad, c,
                         like=x)
        o = out[n0:n0 + n].view(-1, cout)
        if gemm.gemm256_ok(c, w, out=o):   # the columns on the tile kernel, ReLU in its epilogue
            gemm.gemm256(c, w, bias=b, relu=True, out=o)
        else:
            torch.ops.aten._addmm_activation.out(b, c, wt, out=o)
        if overlap:
            freed[ci % 2] = torch.cuda.Event()
            freed[ci % 2].record(main)
    return out


def _avgpool2(x):
    """nn.AvgPool2d(2) on NHWC rows: HIP (16-byte channel runs), torch's arithmetic."""
    N, H, W, C = x.shape
    if C % (16 // x.element_size()):
        return _nhwc(F.avg_pool2d(_nchw(x), 2))
    x = _native.check(x.contiguous(), "avgpool input", ndim=4)
    out = torch.empty((N, H // 2, W // 2, C), dtype=x.dtype, device=x.device)
    _native.call("ov3d_avgpool2_nhwc", x, x.element_size(), N, H, W, C, out, like=x)
    return out


class RegionCLIP(nn.Module):
    """CLIPFastRCNN (GT crop regions, CLIPRes5ROIHeads_FeatureExtraction, attnpool) with
    the reference's ``inference`` API plus the batched ``region_features`` used by the
    criterion.  ``compute_dtype``: torch.bfloat16 (training step) or torch.float32."""

    def __init__(self, depth=200, output_dim=640, pooler_resolution=18, pixel_mean=CLIP_PIXEL_MEAN,
                 pixel_std=CLIP_PIXEL_STD, div_pixel=True, compute_dtype=torch.bfloat16,
                 layers=None, width=None, heads=None, max_rois_per_chunk=8192):
        super().__init__()
        lay, wid = CLIP_RESNETS[depth] if layers is None else (layers, width)
        heads = heads if heads is not None else wid * 32 // 64
        self.backbone = ModifiedResNet(lay, output_dim, heads, pooler_resolution * 16, wid)
        self.register_buffer("pixel_mean", torch.tensor(pixel_mean).view(-1, 1, 1), persistent=False)
        self.register_buffer("pixel_std", torch.tensor(pixel_std).view(-1, 1, 1), persistent=False)
        self._norm = (tuple(float(v) for v in pixel_mean), tuple(float(v) for v in pixel_std))
        self.div_pixel = div_pixel
        self.pooler_resolution = pooler_resolution
        self.spatial_scale = 1.0 / 16
        self.sampling_ratio = 0
        self.compute_dtype = compute_dtype
        self.max_rois_per_chunk = max_rois_per_chunk
        # Optional (H, W) promise that every batch's largest image has exactly this size
        # (e.g. SUN RGB-D batches holding a 530x730 image): the padded batch shape is then
        # known without reading image_height / image_width back to the host, which keeps
        # the step free of host syncs (hipGraph capture).  None = read them (reference).
        self.static_image_size = None
        self._folded = None
        self.eval()

    # -- weights -------------------------------------------------------------------------
    def _load_from_state_dict(self, *a, **k):
        self._folded = None
        return super()._load_from_state_dict(*a, **k)

    def _apply(self, fn, *a, **k):
        self._folded = None
        return super()._apply(fn, *a, **k)

    def folded(self):
        if self._folded is None or self._folded.pos.device != self.backbone.conv1.weight.device:
            self._folded = _Folded(self.backbone, self.compute_dtype)
        return self._folded

    # -- reference API -------------------------------------------------------------------
    @torch.no_grad()
    def inference(self, batched_inputs, detected_instances=None, do_postprocess=False):
        """criterion.py:397: list of {"image": (3,H,W) 0-255, "instances": Instances(gt_boxes)}
        -> (sum_i Q_i, output_dim) f32 region features, scene-major / box-minor."""
        if do_postprocess:
            raise NotImplementedError("only the feature-extraction form (do_postprocess=False) "
                                      "is used by the reference (criterion.py:397)")
        boxes = [x["instances"].gt_boxes.tensor for x in batched_inputs]
        counts = [int(b.shape[0]) for b in boxes]
        images = [x["image"] for x in batched_inputs]
        feats = self._features(self._preprocess_list(images))
        return self._roi_features(feats, torch.cat(boxes).float().contiguous(), counts=counts)

    # -- batched training-step path -------------------------------------------------------
    @torch.no_grad()
    def region_features(self, images_1d, heights, widths, boxes):
        """Every decoder layer's region features from ONE backbone pass.

        images_1d (B, cap) f32 padded 1-D images (criterion.py:371-375), heights/widths (B,)
        ints (a host list or a tensor; the padded batch shape is their max, as
        ImageList.from_tensors makes it), boxes (L, B, Q, 4) image-pixel boxes
        -> (L, B, Q, output_dim) f32 == stacking clip.inference over the L layers."""
        L, B, Q, _ = boxes.shape
        if self.static_image_size is not None:
            hmax, wmax = self.static_image_size
        else:
            hmax = max(heights.tolist() if torch.is_tensor(heights) else list(heights))
            wmax = max(widths.tolist() if torch.is_tensor(widths) else list(widths))
        x = self._preprocess_1d(images_1d, heights, widths, hmax, wmax)
        feats = self._features(x)
        out = self._roi_features(feats, boxes.reshape(-1, 4).float().contiguous(), per_image=Q,
                                 nimages=B)
        return out.view(L, B, Q, -1)

    # -- stages ----------------------------------------------------------------------------
    def _pad_hw(self, h, w):
        d = self.backbone.size_divisibility
        if d > 1:
            h, w = (h + d - 1) // d * d, (w + d - 1) // d * d
        return h, w

    def _preprocess_1d(self, images_1d, heights, widths, hmax, wmax):
        dev = images_1d.device
        Hp, Wp = self._pad_hw(int(hmax), int(wmax))
        B = images_1d.shape[0]
        hts = torch.as_tensor(heights, dtype=torch.int32, device=dev).contiguous()
        wts = torch.as_tensor(widths, dtype=torch.int32, device=dev).contiguous()
        images_1d = _native.check(images_1d.float().contiguous(), "images", ndim=2)
        out = torch.empty((B, Hp, Wp, 3), dtype=self.compute_dtype, device=dev)
        m, s = self._norm      # host constants: no device read in the (capturable) step
        _native.call("ov3d_clip_preprocess", images_1d, images_1d.stride(0), hts, wts, B, Hp, Wp,
                     255.0 if self.div_pixel else 1.0, *m, *s,
                     int(self.compute_dtype == torch.bfloat16), out, like=images_1d)
        return out

    def _preprocess_list(self, images):
        """preprocess_image for a list of (3,H,W) tensors: one HIP launch on the HWC data."""
        hs = [int(im.shape[1]) for im in images]
        ws = [int(im.shape[2]) for im in images]
        cap = max(h * w for h, w in zip(hs, ws)) * 3
        flat = torch.zeros((len(images), cap), dtype=torch.float32, device=images[0].device)
        for i, im in enumerate(images):
            flat[i, : hs[i] * ws[i] * 3] = im.permute(1, 2, 0).reshape(-1)
        return self._preprocess_1d(flat, hs, ws, max(hs), max(ws))

    def _features(self, x):
        """NHWC image batch -> res4 (N, H/16, W/16, 4*width) NHWC."""
        fw = self.folded()
        c = fw.conv
        x = _conv3x3(x, *c["conv1"], stride=2)
        x = _conv3x3(x, *c["conv2"])
        x = _conv3x3(x, *c["conv3"])
        x = _avgpool2(x)
        for lname in ("layer1", "layer2", "layer3"):
            x = self._res_layer(x, lname)
        return x

    def _res_layer(self, x, lname, x_pooled=None):
        """x_pooled: _avgpool2(x) when the caller already has it (the ROIAlign launch)"""
        fw = self.folded()
        for i, blk in enumerate(getattr(self.backbone, lname)):
            key = f"{lname}.{i}"
            c = fw.conv
            out = _conv1x1(x, *c[key + ".conv1"], relu=True)
            out = _conv3x3(out, *c[key + ".conv2"])
            if blk.stride > 1:
                out = _avgpool2(out)
            if blk.downsample is not None:
                if blk.stride > 1:
                    xi = x_pooled if (i == 0 and x_pooled is not None) else _avgpool2(x)
                else:
                    xi = x
                identity = _conv1x1(xi, *c[key + ".down"], relu=False)
            else:
                identity = x
            x = _conv1x1(out, *c[key + ".conv3"], relu=True, residual=identity)
        return x

    def _roi_features(self, feats, boxes, counts=None, per_image=None, nimages=None):
        """ROIAlign (HIP) + res5 + attention pool over all boxes, chunked by ROI count."""
        N, H, W, C = feats.shape
        if counts is not None:   # list form: rows grouped by image
            outs = []
            start = 0
            for i, n in enumerate(counts):
                if n:
                    outs.append(self._roi_chunked(feats[i:i + 1], boxes[start:start + n], n, 1))
                start += n
            return torch.cat(outs) if outs else boxes.new_zeros((0, self.backbone.attnpool.c_proj.out_features))
        return self._roi_chunked(feats, boxes, per_image, nimages)

    def _roi_chunked(self, feats, boxes, per_image, nimages):
        R = boxes.shape[0]
        step = max(per_image, (self.max_rois_per_chunk // per_image) * per_image)
        outs = []
        for r0 in range(0, R, step):
            b = boxes[r0:r0 + step]
            # rows r0.. map to image ((r0 + r) / per_image) % nimages; r0 is a multiple of per_image
            first = (r0 // per_image) % nimages
            f = feats if first == 0 else torch.roll(feats, -first, 0)
            outs.append(self._roi_block(f, b, per_image, nimages))
        return torch.cat(outs) if len(outs) > 1 else outs[0]

    def _roi_block(self, feats, boxes, per_image, nimages):
        P = self.pooler_resolution
        N, H, W, C = feats.shape
        R = boxes.shape[0]
        feats = _native.check(feats.contiguous(), "res4 features", ndim=4)
        boxes = _native.check(boxes.contiguous(), "boxes", dtype=torch.float32, ndim=2)
        x = torch.empty((R, P, P, C), dtype=feats.dtype, device=feats.device)
        if os.environ.get("OV3D_ROI_STATS") == "1" and not torch.cuda.is_current_stream_capturing():
            # diagnostic: ROI extents in feature pixels and ROIAlign samples per bin (host sync)
            wh = (boxes[:, 2:] - boxes[:, :2]).float() * self.spatial_scale
            g = torch.ceil(wh / P).clamp(min=1)
            qs = torch.tensor([0.1, 0.5, 0.9, 1.0], device=boxes.device)
            print("ROI_STATS R=%d map=%dx%d w_q=%s h_q=%s samples/bin mean=%.2f" % (
                R, H, W, torch.quantile(wh[:, 0], qs).tolist(), torch.quantile(wh[:, 1], qs).tolist(),
                (g[:, 0] * g[:, 1]).mean().item()), flush=True)
        blk0 = self.backbone.layer4[0]
        xp = None
        if P % 2 == 0 and blk0.stride > 1 and blk0.downsample is not None:
            # the first block's identity pool comes out of the ROIAlign launch itself
            xp = torch.empty((R, P // 2, P // 2, C), dtype=feats.dtype, device=feats.device)
            _native.call("ov3d_roi_align_pool2_fwd", feats, int(feats.dtype == torch.bfloat16), N, H,
                         W, C, boxes, R, per_image, nimages, self.spatial_scale, P,
                         self.sampling_ratio, 1, x, xp, like=feats)
        else:
            _native.call("ov3d_roi_align_fwd", feats, int(feats.dtype == torch.bfloat16), N, H, W,
                         C, boxes, R, per_image, nimages, self.spatial_scale, P,
                         self.sampling_ratio, 1, x, like=feats)
        x = self._res_layer(x, "layer4", x_pooled=xp)
        return self._attnpool(x)

    def _attnpool(self, x):
        """AttentionPool2d, first query only, reassociated (module docstring)."""
        if self._fused_pool_ok(x):
            return self._pool_fused(x)
        return self._pool_tokens(self._tokens(x))

    def _fused_pool_ok(self, x):
        fw = self.folded()
        R, h, w, C = x.shape
        return (FUSED_POOL and x.is_cuda and x.dtype == torch.bfloat16 and fw.pos.dtype == torch.bfloat16
                and bool(_native.load().ov3d_attnpool_fused_supported(h * w, C, fw.heads)))

    def _pool_fused(self, x):
        """_pool_tokens without the token rows (csrc/attnpool.hip): the mean token t0, q and
        a = Wk_h^T q_h as before, then scores, softmax and p.t for all heads in one launch that
        builds the token rows on chip; the value / output projections as before."""
        fw = self.folded()
        R, h, w, C = x.shape
        Hh, d = fw.heads, fw.head_dim
        x = _native.check(x.contiguous(), "attnpool input", ndim=4)
        t0 = torch.empty((R, C), dtype=x.dtype, device=x.device)
        _native.call("ov3d_attnpool_mean", x, R, h * w, C, fw.pos, t0, like=x)
        tiles = gemm.gemm256_ok(t0, fw.wq) and d % 8 == 0
        q = (gemm.gemm256(t0, fw.wq, bias=fw.bq) if tiles
             else torch.addmm(fw.bq, t0, fw.wq.t()))                     # (R, C), scaled
        a = torch.empty((Hh, R, C), dtype=x.dtype, device=x.device)
        if tiles:   # a_h = q_h Wk_h for every head in one tile-kernel launch (K = d)
            gemm.gemm256_batched(q, C, d, fw.wkt, d, C * d, a, C, R * C, R, C, d, Hh)
        else:
            torch.bmm(q.view(R, Hh, d).transpose(0, 1), fw.wk, out=a)
        y = torch.empty((Hh, R, C), dtype=x.dtype, device=x.device)
        _native.call("ov3d_attnpool_fused", x, t0, fw.pos, a, a.stride(0), a.stride(1), R, h * w, C,
                     Hh, y, like=x)
        if tiles:   # o_h = y_h Wv_h^T + bv_h, one launch, written as (R, H*d) rows
            o = torch.empty((R, C), dtype=x.dtype, device=x.device)
            gemm.gemm256_batched(y, C, R * C, fw.wv, C, d * C, o, C, d, R, d, C, Hh, bias=fw.bv,
                                 sbias=d)
            return gemm.gemm256(o, fw.wc, bias=fw.bc).float()
        o = torch.bmm(y, fw.wvt).transpose(0, 1)                         # (R, H, d)
        o = (o.float() + fw.bv.view(Hh, d)).to(x.dtype).reshape(R, C)
        return torch.addmm(fw.bc, o, fw.wc.t()).float()

    def _tokens(self, x):
        """(R, h, w, C) res5 rows -> (R, h*w + 1, C) token rows [mean; x] + pos (one HIP pass)."""
        fw = self.folded()
        R, h, w, C = x.shape
        t = torch.empty((R, h * w + 1, C), dtype=x.dtype, device=x.device)
        x = _native.check(x.contiguous(), "attnpool input", ndim=4)
        _native.call("ov3d_attnpool_tokens", x, x.element_size(), R, h * w, C, fw.pos, t, like=x)
        return t

    def _pool_tokens(self, t):
        """the pool's first query over the token rows t (R, T, C) -> (R, output_dim) f32"""
        fw = self.folded()
        R, _, C = t.shape
        Hh, d = fw.heads, fw.head_dim
        q = torch.addmm(fw.bq, t[:, 0], fw.wq.t())                        # (R, C), scaled
        a = torch.bmm(q.view(R, Hh, d).transpose(0, 1), fw.wk)             # (H, R, C)
        s = torch.bmm(a.transpose(0, 1), t.transpose(1, 2))                # (R, H, T)
        p = torch.softmax(s.float(), dim=-1).to(t.dtype)
        y = torch.bmm(p, t)                                                # (R, H, C)
        o = torch.bmm(y.transpose(0, 1), fw.wvt).transpose(0, 1)           # (R, H, d)
        o = (o.float() + fw.bv.view(Hh, d)).to(t.dtype).reshape(R, C)
        return torch.addmm(fw.bc, o, fw.wc.t()).float()


def build_regionclip(args=None, dataset_config=None, compute_dtype=torch.bfloat16, seed=11, **kw):
    """models/model_regionclip.py:15-22 counterpart -> (model, None).  Loads
    ``args.region_clip_ckpt_path`` with torch.load(weights_only=True) when the file exists
    (detectron2 checkpoint keys 'model' -> 'backbone.*'), else seeded synthetic weights."""
    model = RegionCLIP(compute_dtype=compute_dtype, **kw)
    init_synthetic_(model.backbone, seed=seed)
    path = getattr(args, "region_clip_ckpt_path", None) if args is not None else None
    if path:
        import os
        if os.path.exists(path):
            sd = torch.load(path, map_location="cpu", weights_only=True)
            sd = sd.get("model", sd)
            model.load_state_dict({k: v for k, v in sd.items() if k.startswith("backbone.")},
                                  strict=False)
    return model.eval(), None
