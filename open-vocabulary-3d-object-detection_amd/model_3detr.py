"""3DETR with open-vocabulary classification head (mirror of reference
models/model_3detr.py), on the ov3d HIP kernels for sampling / grouping.

API kept identical for main.py / engine.py:
  * ``build_3detr(args, dataset_config) -> (Model3DETR, BoxProcessor)``
    (model_3detr.py:421-438);
  * ``Model3DETR.forward(inputs, encoder_only=False)`` returning
    ``{"outputs": {13 keys}, "aux_outputs": [7 dicts]}`` (model_3detr.py:317-350);
  * state-dict keys of the reference (pre_encoder.mlp_module.layer*, encoder.layers.*,
    decoder.layers.*, mlp_heads.*, pos_embedding.gauss_B, ...).
Reference quirks reproduced by default:
  * Q6: ``sem_cls_head`` = Linear(640, T, bias=False) holding the frozen text
    embedding; logits are raw dot products;
  * Q8: the reference reshapes the (L*B, T, Q) transposed logits straight to
    (L, B, Q, T) (model_3detr.py:238, 253), which scrambles the (query, class)
    layout; ``cls_logits_layout="reference"`` keeps that, ``"fixed"`` undoes it.
"""
import math
from functools import partial

import numpy as np
import torch
import torch.nn as nn

from . import _native
from . import attention as flash
from . import heads as heads_mod
from . import pointnet2_utils as pu
from .helpers import GenericMLP
from .pc_util import scale_points, shift_scale_points
from .pointnet2_modules import PointnetSAModuleVotes
from .position_embedding import PositionEmbeddingCoordsSine
from .transformer import (MaskedTransformerEncoder, TransformerDecoder, TransformerDecoderLayer,
                          TransformerEncoder, TransformerEncoderLayer)


class BoxProcessor:
    """Head outputs -> boxes (reference model_3detr.py:19-69)."""

    def __init__(self, dataset_config):
        self.dataset_config = dataset_config

    def compute_predicted_center(self, center_offset, query_xyz, point_cloud_dims):
        center_unnormalized = query_xyz + center_offset
        return shift_scale_points(center_unnormalized, src_range=point_cloud_dims), center_unnormalized

    def compute_predicted_size(self, size_normalized, point_cloud_dims):
        scene_scale = torch.clamp(point_cloud_dims[1] - point_cloud_dims[0], min=1e-1)
        return scale_points(size_normalized, mult_factor=scene_scale)

    def compute_predicted_angle(self, angle_logits, angle_residual):
        if angle_logits.shape[-1] == 1:
            # no-rotation datasets: keep the heads in the graph (DDP), angle = 0
            return (angle_logits * 0 + angle_residual * 0).squeeze(-1).clamp(min=0)
        per_cls = 2 * np.pi / self.dataset_config.num_angle_bin
        cls = angle_logits.argmax(dim=-1).detach()
        angle = per_cls * cls + angle_residual.gather(2, cls.unsqueeze(-1)).squeeze(-1)
        return torch.where(angle > np.pi, angle - 2 * np.pi, angle)

    def compute_objectness_and_cls_prob(self, cls_logits):
        if cls_logits.shape[-1] != self.dataset_config.num_semcls + 1:
            raise ValueError("class logits must have num_semcls + 1 entries")
        prob = torch.softmax(cls_logits, dim=-1)
        return prob[..., :-1], 1 - prob[..., -1]

    def box_parametrization_to_corners(self, box_center_unnorm, box_size_unnorm, box_angle):
        return self.dataset_config.box_parametrization_to_corners(box_center_unnorm, box_size_unnorm,
                                                                  box_angle)


class _BoxParam(torch.autograd.Function):
    """BoxProcessor (model_3detr.py:19-69) + corners for all L*B*Q proposals in one HIP launch
    each way (csrc/boxparam.hip) from the fused heads' raw rows
    [center 3 | size 3 | angle logits NB | angle residual NB]."""

    @staticmethod
    def forward(ctx, raw, qxyz, dmin, dmax, logits, B, Q, NB):
        R = raw.shape[0]
        dev = raw.device
        T = logits.shape[-1]
        f = dict(dtype=torch.float32, device=dev)
        outs = [torch.empty((R, 3), **f) for _ in range(4)] + \
            [torch.empty((R, NB), **f) for _ in range(3)] + \
            [torch.empty((R,), **f), torch.empty((R, 8, 3), **f),
             torch.empty((R, T - 1), **f), torch.empty((R,), **f)]
        qxyz, dmin, dmax = (t.float().contiguous() for t in (qxyz, dmin, dmax))
        lg = logits.detach().float().reshape(R, T).contiguous()
        _native.call("ov3d_box_param_fwd", R, B, Q, NB, T, raw, raw.stride(0), qxyz, dmin, dmax,
                     lg, *outs, like=raw)
        ctx.save_for_backward(raw, qxyz, dmin, dmax)
        ctx.meta = (B, Q, NB)
        ctx.mark_non_differentiable(outs[9], outs[10])
        ctx.set_materialize_grads(False)   # unused outputs: no zero-filled gradients
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        raw, qxyz, dmin, dmax = ctx.saved_tensors
        B, Q, NB = ctx.meta
        R = raw.shape[0]
        g = [t.float().contiguous() if t is not None else None for t in grads[:9]]
        draw = torch.empty_like(raw)
        if draw.shape[1] > 6 + 2 * NB:
            draw.zero_()
        _native.call("ov3d_box_param_bwd", R, B, Q, NB, raw, raw.stride(0), qxyz, dmin, dmax, *g,
                     draw, draw.stride(0), like=raw)
        return draw, None, None, None, None, None, None, None


class Model3DETR(nn.Module):
    def __init__(self, pre_encoder, encoder, decoder, dataset_config, text_embedding, encoder_dim=256,
                 decoder_dim=256, position_embedding="fourier", mlp_dropout=0.3, num_queries=256,
                 cls_logits_layout="reference"):
        super().__init__()
        self.pre_encoder = pre_encoder
        self.encoder = encoder
        self.class_num = dataset_config.num_semcls + 1
        hidden = [encoder_dim] if hasattr(encoder, "masking_radius") else [encoder_dim, encoder_dim]
        self.encoder_to_decoder_projection = GenericMLP(
            input_dim=encoder_dim, hidden_dims=hidden, output_dim=decoder_dim, norm_fn_name="bn1d",
            activation="relu", use_conv=True, output_use_activation=True, output_use_norm=True,
            output_use_bias=False)
        self.pos_embedding = PositionEmbeddingCoordsSine(d_pos=decoder_dim, pos_type=position_embedding,
                                                         normalize=True)
        self.query_projection = GenericMLP(input_dim=decoder_dim, hidden_dims=[decoder_dim],
                                           output_dim=decoder_dim, use_conv=True,
                                           output_use_activation=True, hidden_use_bias=True)
        self.decoder = decoder
        self._build_heads(dataset_config, decoder_dim, mlp_dropout, text_embedding)
        self.num_queries = num_queries
        self.box_processor = BoxProcessor(dataset_config)
        if cls_logits_layout not in ("reference", "fixed"):
            raise ValueError(cls_logits_layout)
        self.cls_logits_layout = cls_logits_layout
        self.fuse_heads = True   # heads.py under bf16 autocast training (False: per-head MLPs)

    def _build_heads(self, cfg, dim, dropout, text_embedding):
        mlp = partial(GenericMLP, norm_fn_name="bn1d", activation="relu", use_conv=True,
                      hidden_dims=[dim, dim], dropout=dropout, input_dim=dim)
        sem = nn.Linear(cfg.clip_embed_length, self.class_num, bias=False)
        if tuple(sem.weight.shape) != tuple(text_embedding.shape):
            raise ValueError(f"text embedding {tuple(text_embedding.shape)} != {tuple(sem.weight.shape)}")
        sem.weight = nn.Parameter(text_embedding.float().clone(), requires_grad=False)
        self.mlp_heads = nn.ModuleDict([
            ("visual_embed_head", mlp(output_dim=cfg.clip_embed_length)),
            ("sem_cls_head", sem),
            ("center_head", mlp(output_dim=3)),
            ("size_head", mlp(output_dim=3)),
            ("angle_cls_head", mlp(output_dim=cfg.num_angle_bin)),
            ("angle_residual_head", mlp(output_dim=cfg.num_angle_bin)),
        ])

    # ------------------------------------------------------------------ encoder
    def get_query_embeddings(self, encoder_xyz, point_cloud_dims):
        """-> query_xyz (B,Q,3), query_embed (B, C, Q) (reference layout)."""
        query_xyz, rows = self._query_rows(encoder_xyz, point_cloud_dims)
        return query_xyz, rows.permute(0, 2, 1)

    def _query_rows(self, encoder_xyz, point_cloud_dims, query_xyz=None, seq_first=False):
        """-> query_xyz (B, Q, 3), query embedding (B, Q, C) or, seq_first, (Q, B, C) (the
        projection is per row: the PE launch writes the rows in the decoder's order)"""
        if query_xyz is None:
            _, query_xyz = pu.furthest_point_sample_gather(encoder_xyz, self.num_queries)
        pe = self.pos_embedding.rows(query_xyz, input_range=point_cloud_dims, seq_first=seq_first)
        n0, n1, C = pe.shape
        return query_xyz, self.query_projection.rows(pe.reshape(n0 * n1, C)).view(n0, n1, -1)

    @staticmethod
    def _break_up_pc(pc):
        xyz = pc[..., 0:3].contiguous()
        feats = pc[..., 3:].transpose(1, 2).contiguous() if pc.size(-1) > 3 else None
        return xyz, feats

    # index work that depends on the input points only (sampling_plan)
    PLAN_KEYS = ("pre_enc_inds", "pre_enc_xyz", "pre_enc_ball", "query_xyz", "interim_inds",
                 "interim_xyz", "interim_ball", "interim_inv_off", "interim_inv_rows")

    def _encoder_keeps_xyz(self):
        from .transformer import MaskedTransformerEncoder
        return not isinstance(self.encoder, MaskedTransformerEncoder)

    def _interim_sa(self):
        """the masked encoder's interim downsampling SA (None for the vanilla encoder)"""
        return None if self._encoder_keeps_xyz() else getattr(self.encoder, "interim_downsampling",
                                                               None)

    @torch.no_grad()
    def sampling_plan(self, point_clouds):
        """The step's sampling and neighbourhood indices, which depend on the input points
        only: pre-encoder FPS (indices + points), its ball query, and (when the encoder keeps
        its input points) the query FPS.  graphs.StepGraph computes the next batch's plan on
        a side stream while this batch trains; forward(inputs | plan) gives results
        identical to forward(inputs)."""
        xyz = point_clouds[..., 0:3].contiguous()
        pe = self.pre_encoder
        inds, pre_xyz = pu.furthest_point_sample_gather(xyz, pe.npoint)
        plan = {"pre_enc_inds": inds, "pre_enc_xyz": pre_xyz,
                "pre_enc_ball": pu.ball_query(pe.grouper.radius, pe.grouper.nsample, xyz, pre_xyz)}
        if self._encoder_keeps_xyz():
            plan["query_xyz"] = pu.furthest_point_sample_gather(pre_xyz, self.num_queries)[1]
        elif self._interim_sa() is not None:
            # masked encoder (transformer.py:192-197): its interim SA samples the pre-encoder
            # points, so its FPS / ball query and the query FPS on its output points are also
            # functions of the input points
            ids = self._interim_sa()
            i_inds, i_xyz = pu.furthest_point_sample_gather(pre_xyz, ids.npoint)
            ball = pu.ball_query(ids.grouper.radius, ids.grouper.nsample, pre_xyz, i_xyz)
            # the ball's inverse (rows per point) for the gather-form grouping backward
            inv_off, inv_rows = pu.group_inverse(ball, pre_xyz.shape[1])
            plan.update(interim_inds=i_inds, interim_xyz=i_xyz, interim_ball=ball,
                        interim_inv_off=inv_off, interim_inv_rows=inv_rows,
                        query_xyz=pu.furthest_point_sample_gather(i_xyz, self.num_queries)[1])
        return plan

    def run_encoder(self, point_clouds, pre_enc_inds=None, plan=None):
        """pre_enc_inds / plan: the pre-encoder's sampling computed ahead of time (they
        depend on the input points only; see sampling_plan).  Identical results."""
        plan = plan or {}
        pre_enc_inds = plan.get("pre_enc_inds", pre_enc_inds)
        xyz, feats = self._break_up_pc(point_clouds)
        pre_xyz, pre_feats, pre_inds = self.pre_encoder(
            xyz, feats, inds=pre_enc_inds,
            new_xyz=plan.get("pre_enc_xyz") if pre_enc_inds is not None else None,
            ball=plan.get("pre_enc_ball") if pre_enc_inds is not None else None)
        hook = getattr(self, "after_pre_encoder", None)
        if hook is not None:   # graphs.StepGraph (OV3D_PLAN_SPLIT_AT=pre_encoder)
            hook()
        # (B, C, M) view of channels-last rows -> seq-first (M, B, C)
        src = pre_feats.permute(2, 0, 1).contiguous()
        if "interim_inds" in plan:
            enc_xyz, enc_feats, enc_inds = self.encoder(
                src, xyz=pre_xyz, interim_plan=(plan["interim_inds"], plan["interim_xyz"],
                                                plan["interim_ball"],
                                                (plan["interim_inv_off"], plan["interim_inv_rows"])))
        else:
            enc_xyz, enc_feats, enc_inds = self.encoder(src, xyz=pre_xyz)
        if enc_inds is None:
            enc_inds = pre_inds
        else:
            enc_inds = torch.gather(pre_inds.long(), 1, enc_inds.long())
        hook = getattr(self, "after_encoder", None)
        if hook is not None:   # graphs.StepGraph: the point in the step the side stream waits for
            hook()
        return enc_xyz, enc_feats, enc_inds

    # -------------------------------------------------------------------- heads
    def get_box_predictions(self, query_xyz, point_cloud_dims, box_features):
        """Heads for all L decoder layers at once (the reference loops over layers,
        model_3detr.py:264-306).  Training under bf16 autocast: the five MLP heads run as
        one fused MLP (heads.py); the box parametrisation is evaluated in fp32 like the
        reference, even under autocast."""
        L, Q, B, C = box_features.shape
        # heads on channels-last rows ordered (l, b, q): BatchNorm1d statistics are over all
        # L*B*Q positions exactly as on the reference's (L*B, C, Q) conv input
        rows = box_features.permute(0, 2, 1, 3).reshape(L * B * Q, C)
        pre = None
        if self._heads_fused_ok(rows):
                # the text alignment folds into the heads' output launch (Q8 layout written
                # there when the reference layout is kept)
                pre = heads_mod.fused_heads(self._head_pack, rows, sem=self.mlp_heads["sem_cls_head"],
                                            lq=Q if self.cls_logits_layout == "reference" else 0)
        with torch.autocast(device_type=box_features.device.type, enabled=False):
            return self._box_predictions(query_xyz.float(), point_cloud_dims, rows, (L, Q, B), pre)

    def dp_buckets(self):
        """parameters in gradient all-reduce order (dist.GradBuckets): everything downstream of
        the encoder output (decoder, heads, projections: final when the backward reaches that
        output), then the encoder and the pre-encoder SA"""
        early = {id(p) for m in (self.pre_encoder, self.encoder) for p in m.parameters()}
        ps = [p for p in self.parameters() if p.requires_grad]
        return [[p for p in ps if id(p) not in early], [p for p in ps if id(p) in early]]

    def _heads_fused_ok(self, x):
        """True when the five heads run as the fused launch (heads.supported) on x's device"""
        if not self.fuse_heads:
            return False
        if getattr(self, "_head_pack", None) is None:
            self._head_pack = heads_mod.HeadPack(self.mlp_heads)
        return heads_mod.supported(self._head_pack, x)

    def _box_predictions(self, query_xyz, point_cloud_dims, rows, dims_lqb, pre=None):
        L, Q, B = dims_lqb
        heads = self.mlp_heads
        if pre is not None and "_raw" in pre and pre["_raw"].is_cuda and \
                pre["_raw"].dtype == torch.float32 and pre["_raw"].stride(1) == 1:
            return self._box_predictions_fused(query_xyz, point_cloud_dims, pre, L, Q, B)

        if rows is not None:
            rows = rows.float()   # the heads in fp32 (the decoder's bf16 rows under autocast)

        def head(name):
            if pre is not None:
                return pre[name].view(L, B, Q, -1)
            return heads[name].rows(rows).view(L, B, Q, -1)

        visual = head("visual_embed_head")                                  # (L, B, Q, 640)
        if pre is not None and "sem_cls_logits" in pre:   # the heads' launch, final layout
            logits = pre["sem_cls_logits"].view(L, B, Q, -1)
        else:
            logits = heads["sem_cls_head"](visual)                          # (L, B, Q, T)
            if self.cls_logits_layout == "reference":
                logits = logits.reshape(L * B, Q, -1).transpose(1, 2).reshape(L, B, Q, -1)   # Q8
        center_offset = head("center_head").sigmoid() - 0.5
        size_norm = head("size_head").sigmoid()
        angle_logits = head("angle_cls_head")
        angle_res_norm = head("angle_residual_head")
        angle_res = angle_res_norm * (np.pi / angle_res_norm.shape[-1])

        # BoxProcessor over the stacked (L*B) batch: dims repeated per layer
        dims = [point_cloud_dims[0].repeat(L, 1), point_cloud_dims[1].repeat(L, 1)]
        bp = self.box_processor
        center_n, center_u = bp.compute_predicted_center(center_offset.reshape(L * B, Q, 3),
                                                         query_xyz.repeat(L, 1, 1), dims)
        angle = bp.compute_predicted_angle(angle_logits.reshape(L * B, Q, -1),
                                           angle_res.reshape(L * B, Q, -1))
        size_u = bp.compute_predicted_size(size_norm.reshape(L * B, Q, 3), dims)
        corners = bp.box_parametrization_to_corners(center_u, size_u, angle)
        with torch.no_grad():
            sem_prob, obj_prob = bp.compute_objectness_and_cls_prob(logits)
        center_n = center_n.view(L, B, Q, 3)
        center_u = center_u.view(L, B, Q, 3)
        size_u = size_u.view(L, B, Q, 3)
        angle = angle.view(L, B, Q)
        corners = corners.view(L, B, Q, 8, 3)
        stacked = {
            "visual_embeds": visual, "sem_cls_logits": logits, "center_normalized": center_n,
            "center_unnormalized": center_u, "size_normalized": size_norm, "size_unnormalized": size_u,
            "angle_logits": angle_logits, "angle_residual": angle_res,
            "angle_residual_normalized": angle_res_norm, "angle_continuous": angle,
            "objectness_prob": obj_prob, "sem_cls_prob": sem_prob, "box_corners": corners,
        }
        # per-layer dicts as views (unbind: ONE stack in backward per key, not L selects that
        # each zero-fill a full-size gradient)
        per_key = {k: v.unbind(0) for k, v in stacked.items()}
        outs = [{k: per_key[k][l] for k in stacked} for l in range(L)]
        # "_layers_stacked": the same tensors stacked over decoder layers (natural order, last =
        # final); the set criterion consumes them directly instead of re-concatenating
        return {"outputs": outs[-1], "aux_outputs": outs[:-1], "_layers_stacked": stacked}

    def _box_predictions_fused(self, query_xyz, point_cloud_dims, pre, L, Q, B):
        """same outputs as _box_predictions, the parametrisation in one HIP launch each way"""
        visual = pre["visual_embed_head"].view(L, B, Q, -1)
        if "sem_cls_logits" in pre:   # computed by the heads' output launch, final layout
            logits = pre["sem_cls_logits"].view(L, B, Q, -1)
        else:
            logits = self.mlp_heads["sem_cls_head"](visual)                 # (L, B, Q, T)
            if self.cls_logits_layout == "reference":
                logits = logits.reshape(L * B, Q, -1).transpose(1, 2).reshape(L, B, Q, -1)   # Q8
        NB = self.box_processor.dataset_config.num_angle_bin
        (center_n, center_u, size_n, size_u, angle_logits, angle_res_norm, angle_res, angle,
         corners, sem_prob, obj_prob) = _BoxParam.apply(pre["_raw"], query_xyz, point_cloud_dims[0],
                                                       point_cloud_dims[1], logits, B, Q, NB)
        v = lambda t, *tail: t.view(L, B, Q, *tail)   # noqa: E731
        stacked = {
            "visual_embeds": visual, "sem_cls_logits": logits, "center_normalized": v(center_n, 3),
            "center_unnormalized": v(center_u, 3), "size_normalized": v(size_n, 3),
            "size_unnormalized": v(size_u, 3), "angle_logits": v(angle_logits, NB),
            "angle_residual": v(angle_res, NB), "angle_residual_normalized": v(angle_res_norm, NB),
            "angle_continuous": v(angle), "objectness_prob": v(obj_prob),
            "sem_cls_prob": v(sem_prob, -1), "box_corners": v(corners, 8, 3),
        }
        per_key = {k: t.unbind(0) for k, t in stacked.items()}
        outs = [{k: per_key[k][l] for k in stacked} for l in range(L)]
        return {"outputs": outs[-1], "aux_outputs": outs[:-1], "_layers_stacked": stacked}

    def _pregen_encoder_dropout(self, pc):
        """The plain encoder's self-attention drop bits for this step, generated on a side
        stream beside the pre-encoder (attention.pregen_dropout): the layers' forwards read
        them instead of hashing.  Bit-identical masks (same seed, site and hash)."""
        from .transformer import TransformerEncoder
        enc = self.encoder
        if not (flash.PREGEN and type(enc) is TransformerEncoder and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            return
        L = getattr(self.pre_encoder, "npoint", None)
        if not L or L % 32:
            return
        B = pc.shape[0]
        jobs = []
        for layer in enc.layers:
            a = getattr(layer, "self_attn", None)
            if a is None or not getattr(a, "site", None) or a.dropout <= 0 or \
                    a.embed_dim != a.num_heads * flash.HEAD_DIM:
                return
            jobs.append((a.site, B, a.num_heads, L, L, float(a.dropout)))
        flash.pregen_dropout(pc.device, jobs)

    def forward(self, inputs, encoder_only=False):
        pc = inputs["point_clouds"]
        if self.training and pc.is_cuda:
            flash.next_step(pc.device)   # fresh attention-dropout stream for this step
            self._pregen_encoder_dropout(pc)
        plan = {k: inputs[k] for k in self.PLAN_KEYS if k in inputs}
        enc_xyz, enc_feats, _ = self.run_encoder(pc, plan=plan)   # (N', B, C)
        hook = getattr(self, "encoder_grad_hook", None)
        if hook is not None and enc_feats.requires_grad:
            # data parallel: the decoder side's gradients are final when this fires (dist.py
            # stage_after_encoder starts their all-reduce under the encoder's backward)
            enc_feats.register_hook(lambda g: hook())
        Np, B, C = enc_feats.shape
        enc_feats = self.encoder_to_decoder_projection.rows(enc_feats.reshape(Np * B, C)).view(Np, B, -1)
        if encoder_only:
            return enc_xyz, enc_feats.transpose(0, 1)
        dims = [inputs["point_cloud_dims_min"].float(), inputs["point_cloud_dims_max"].float()]
        # (Q, B, C) and (N', B, C) rows, sequence-first as the decoder reads them
        query_xyz, query_embed = self._query_rows(enc_xyz, dims, plan.get("query_xyz"),
                                                  seq_first=True)
        enc_pos = self.pos_embedding.rows(enc_xyz, input_range=dims, seq_first=True)
        tgt = _zeros_like_cached(query_embed)
        # the fused decoder writes its layer outputs as bf16 rows only for the fused heads
        # launch; the per-head fp32 path (eval, other head shapes) gets the fp32 rows
        self.decoder.rows_bf16 = self._heads_fused_ok(tgt)
        box_features = self.decoder(tgt, enc_feats, query_pos=query_embed, pos=enc_pos)[0]
        return self.get_box_predictions(query_xyz, dims, box_features)


_ZERO_TGT = {}


def _zeros_like_cached(t):
    """the decoder's initial target (zeros, read-only): allocated once per shape instead of
    zero-filled in every step"""
    key = (tuple(t.shape), t.dtype, t.device)
    z = _ZERO_TGT.get(key)
    if z is None:
        z = torch.zeros_like(t)
        _ZERO_TGT[key] = z
    return z


# ---------------------------------------------------------------- builders
def build_preencoder(args):
    return PointnetSAModuleVotes(radius=0.2, nsample=64, npoint=args.preenc_npoints,
                                 mlp=[3 * int(args.use_color), 64, 128, args.enc_dim],
                                 normalize_xyz=True)


def build_encoder(args):
    layer = TransformerEncoderLayer(d_model=args.enc_dim, nhead=args.enc_nhead,
                                    dim_feedforward=args.enc_ffn_dim, dropout=args.enc_dropout,
                                    activation=args.enc_activation)
    if args.enc_type == "vanilla":
        return TransformerEncoder(encoder_layer=layer, num_layers=args.enc_nlayers)
    if args.enc_type == "masked":
        interim = PointnetSAModuleVotes(radius=0.4, nsample=32, npoint=args.preenc_npoints // 2,
                                        mlp=[args.enc_dim, 256, 256, args.enc_dim], normalize_xyz=True)
        return MaskedTransformerEncoder(encoder_layer=layer, num_layers=3,
                                        interim_downsampling=interim,
                                        masking_radius=[math.pow(x, 2) for x in (0.4, 0.8, 1.2)])
    raise ValueError(f"Unknown encoder type {args.enc_type}")


def build_decoder(args):
    layer = TransformerDecoderLayer(d_model=args.dec_dim, nhead=args.dec_nhead,
                                    dim_feedforward=args.dec_ffn_dim, dropout=args.dec_dropout)
    return TransformerDecoder(layer, num_layers=args.dec_nlayers, return_intermediate=True)


def load_text_embed(args):
    """reference model_3detr.py:417-419 (weights_only load: a plain tensor file)."""
    return torch.load(args.clip_embed_path, map_location="cpu", weights_only=True).float()


def build_3detr(args, dataset_config, text_embedding=None):
    if text_embedding is None:
        text_embedding = load_text_embed(args)
    model = Model3DETR(build_preencoder(args), build_encoder(args), build_decoder(args), dataset_config,
                       text_embedding, encoder_dim=args.enc_dim, decoder_dim=args.dec_dim,
                       mlp_dropout=args.mlp_dropout, num_queries=args.nqueries,
                       cls_logits_layout=getattr(args, "cls_logits_layout", "reference"))
    return model, BoxProcessor(dataset_config)
