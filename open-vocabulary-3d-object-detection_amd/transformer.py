"""Pre-norm DETR-style encoder / decoder (mirror of reference models/transformer.py).

Layout: sequence-first (L, B, C) tensors exactly as the reference, and the
attention modules keep ``nn.MultiheadAttention``'s parameter names
(``in_proj_weight``, ``in_proj_bias``, ``out_proj.{weight,bias}``) so reference
checkpoints load.  Differences that do not change results:
  * attention runs through the HIP flash-attention kernels (attention.py,
    csrc/attn.hip; bf16, no mask) or fused scaled-dot-product attention (fp32,
    masked encoder) and never materialises the head-averaged weights that
    ``nn.MultiheadAttention`` computes and the reference discards
    (need_weights=True by default, transformer.py:271-272, 365-372);
  * ``memory + pos`` is formed once and shared by the 8 decoder layers.
"""
from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from . import attention as flash
from . import resnorm as rn
from .gemm import in_projection, rows_linear
from .helpers import ACTIVATION_DICT, NORM_DICT, get_clones


class MultiheadAttention(nn.Module):
    """Seq-first multi-head attention with nn.MultiheadAttention's state-dict keys."""

    def __init__(self, embed_dim, num_heads, dropout=0.0):
        super().__init__()
        if embed_dim % num_heads:
            raise ValueError("embed_dim must be divisible by num_heads")
        self.embed_dim, self.num_heads, self.dropout = embed_dim, num_heads, dropout
        self.head_dim = embed_dim // num_heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * embed_dim))
        self.out_proj = nn.Linear(embed_dim, embed_dim)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)
        self.site = flash.new_site()   # dropout hash stream of this module (attention.py)

    def _heads(self, x, L, B):
        return x.view(L, B, self.num_heads, self.head_dim).permute(1, 2, 0, 3)

    def forward(self, query, key, value, attn_mask: Optional[Tensor] = None):
        L, B, E = query.shape
        S = key.shape[0]
        w, bias = self.in_proj_weight, self.in_proj_bias
        if query is key and key is value:
            srcs = [rows_linear(query, w, bias)]
            spec = ((0, 0), (0, E), (0, 2 * E))
        elif query is key:
            srcs = list(in_projection(w, bias, ((query, 0, 2 * E), (value, 2 * E, 3 * E))))
            spec = ((0, 0), (0, E), (1, 0))
        else:
            srcs = list(in_projection(w, bias, ((query, 0, E), (key, E, 2 * E), (value, 2 * E, 3 * E))))
            spec = ((0, 0), (1, 0), (2, 0))
        if srcs[0].dtype == torch.bfloat16 and flash.supported(srcs[0], E, self.num_heads,
                                                               attn_mask):
            # HIP flash attention straight on the projection rows (csrc/attn.hip)
            out = flash.attention_packed(srcs, spec, L, S, self.num_heads,
                                         dropout_p=self.dropout if self.training else 0.0,
                                         site=self.site)
            return rows_linear(out, self.out_proj.weight, self.out_proj.bias)
        q, k, v = (srcs[i][..., off:off + E] for i, off in spec)
        q, k, v = self._heads(q, L, B), self._heads(k, S, B), self._heads(v, S, B)
        mask = None
        if attn_mask is not None:
            # reference convention: True = NOT allowed, shape (B*H, L, S)
            mask = ~attn_mask.view(B, self.num_heads, L, S)
        out = F.scaled_dot_product_attention(q, k, v, attn_mask=mask,
                                             dropout_p=self.dropout if self.training else 0.0)
        out = out.permute(2, 0, 1, 3).reshape(L, B, E)
        return rows_linear(out, self.out_proj.weight, self.out_proj.bias)


class TransformerEncoderLayer(nn.Module):
    def __init__(self, d_model, nhead=4, dim_feedforward=128, dropout=0.1, dropout_attn=None,
                 activation="relu", normalize_before=True, norm_name="ln", use_ffn=True,
                 ffn_use_bias=True):
        super().__init__()
        if not normalize_before:
            raise NotImplementedError("the reference builds pre-norm layers only")
        self.self_attn = MultiheadAttention(d_model, nhead,
                                            dropout=dropout if dropout_attn is None else dropout_attn)
        self.use_ffn = use_ffn
        if use_ffn:
            self.linear1 = nn.Linear(d_model, dim_feedforward, bias=ffn_use_bias)
            self.dropout = nn.Dropout(dropout)
            self.linear2 = nn.Linear(dim_feedforward, d_model, bias=ffn_use_bias)
            self.norm2 = NORM_DICT[norm_name](d_model)
            self.dropout2 = nn.Dropout(dropout)
        self.norm1 = NORM_DICT[norm_name](d_model)
        self.dropout1 = nn.Dropout(dropout)
        self.activation = ACTIVATION_DICT[activation]()
        self.normalize_before = normalize_before
        self.nhead = nhead

    def forward(self, src, src_mask: Optional[Tensor] = None, src_key_padding_mask=None,
                pos: Optional[Tensor] = None, return_attn_weights=False):
        if src_key_padding_mask is not None or return_attn_weights:
            raise NotImplementedError
        x = self.norm1(src)
        qk = x if pos is None else x + pos
        src = src + self.dropout1(self.self_attn(qk, qk, x, attn_mask=src_mask))
        if self.use_ffn:
            x = self.norm2(src)
            h = self.dropout(self.activation(rows_linear(x, self.linear1.weight, self.linear1.bias)))
            src = src + self.dropout2(rows_linear(h, self.linear2.weight, self.linear2.bias))
        return src

    def forward_fused(self, pend, src_mask=None, pos=None):
        """bf16 training / eval step on a Pending residual (resnorm.py); -> Pending."""
        p1, p2 = (self.dropout1.p, self.dropout2.p) if self.training else (0.0, 0.0)
        site1, site2, site_ffn = rn.sites(self, 3)
        s, x, xp, _ = rn.resnorm(pend, self.norm1, pos=pos, want_a=True, want_ap=pos is not None)
        qk = xp if pos is not None else x
        y = self.self_attn(qk, qk, x, attn_mask=src_mask)
        if not self.use_ffn:
            return rn.Pending(s, y, p1, site1)
        s, x, _, _ = rn.resnorm(rn.Pending(s, y, p1, site1), self.norm2)
        h = rn.ffn_act(rows_linear(x, self.linear1.weight, self.linear1.bias), self.activation,
                       self.dropout, site_ffn)
        return rn.Pending(s, rows_linear(h, self.linear2.weight, self.linear2.bias), p2, site2)

    def fused_ok(self, x):
        return rn.supported(x, self.norm1, self.norm2 if self.use_ffn else None)


class TransformerDecoderLayer(nn.Module):
    def __init__(self, d_model, nhead=4, dim_feedforward=256, dropout=0.1, dropout_attn=None,
                 activation="relu", normalize_before=True, norm_fn_name="ln"):
        super().__init__()
        if not normalize_before:
            raise NotImplementedError("the reference builds pre-norm layers only")
        self.self_attn = MultiheadAttention(d_model, nhead, dropout=dropout)
        self.multihead_attn = MultiheadAttention(d_model, nhead, dropout=dropout)
        self.norm1 = NORM_DICT[norm_fn_name](d_model)
        self.norm2 = NORM_DICT[norm_fn_name](d_model)
        self.norm3 = NORM_DICT[norm_fn_name](d_model)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.dropout3 = nn.Dropout(dropout)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.activation = ACTIVATION_DICT[activation]()
        self.normalize_before = normalize_before

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, tgt_key_padding_mask=None,
                memory_key_padding_mask=None, pos=None, query_pos=None, return_attn_weights=False,
                memory_pos=None):
        if tgt_key_padding_mask is not None or memory_key_padding_mask is not None:
            raise NotImplementedError
        x = self.norm1(tgt)
        qk = x if query_pos is None else x + query_pos
        tgt = tgt + self.dropout1(self.self_attn(qk, qk, x, attn_mask=tgt_mask))
        x = self.norm2(tgt)
        q = x if query_pos is None else x + query_pos
        if memory_pos is None:
            memory_pos = memory if pos is None else memory + pos
        tgt = tgt + self.dropout2(self.multihead_attn(q, memory_pos, memory, attn_mask=memory_mask))
        x = self.norm3(tgt)
        h = self.dropout(self.activation(rows_linear(x, self.linear1.weight, self.linear1.bias)))
        tgt = tgt + self.dropout3(rows_linear(h, self.linear2.weight, self.linear2.bias))
        return tgt, None

    def forward_fused(self, s, x, xp, memory, memory_pos, query_pos=None, tgt_mask=None,
                      memory_mask=None):
        """bf16 step from norm1's outputs (x = norm1(tgt), xp = x + query_pos) -> Pending of
        the layer output (resnorm.py)."""
        p1, p2, p3 = ((self.dropout1.p, self.dropout2.p, self.dropout3.p) if self.training
                      else (0.0, 0.0, 0.0))
        site1, site2, site3, site_ffn = rn.sites(self, 4)
        qk = xp if query_pos is not None else x
        y = self.self_attn(qk, qk, x, attn_mask=tgt_mask)
        s, x2, q, _ = rn.resnorm(rn.Pending(s, y, p1, site1), self.norm2, pos=query_pos,
                                 want_a=query_pos is None, want_ap=query_pos is not None)
        y = self.multihead_attn(q if query_pos is not None else x2, memory_pos, memory,
                                attn_mask=memory_mask)
        s, x3, _, _ = rn.resnorm(rn.Pending(s, y, p2, site2), self.norm3)
        h = rn.ffn_act(rows_linear(x3, self.linear1.weight, self.linear1.bias), self.activation,
                       self.dropout, site_ffn)
        return rn.Pending(s, rows_linear(h, self.linear2.weight, self.linear2.bias), p3, site3)

    def fused_ok(self, x):
        return rn.supported(x, self.norm1, self.norm2, self.norm3)


class TransformerEncoder(nn.Module):
    def __init__(self, encoder_layer, num_layers, norm=None, weight_init_name="xavier_uniform"):
        super().__init__()
        self.layers = get_clones(encoder_layer, num_layers)
        self.num_layers = num_layers
        self.norm = norm
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def forward(self, src, mask=None, src_key_padding_mask=None, pos=None, xyz=None,
                transpose_swap=False):
        if transpose_swap:
            raise NotImplementedError
        masks = mask if isinstance(mask, list) else [mask] * len(self.layers)
        masks = [self._head_mask(m, layer) for layer, m in zip(self.layers, masks)]
        if self._fused_ok(src):
            pend = rn.Pending(src, None, 0.0, 0)
            for layer, m in zip(self.layers, masks):
                pend = layer.forward_fused(pend, src_mask=m, pos=pos)
            return xyz, self._finish_fused(pend), None
        out = src
        for layer, m in zip(self.layers, masks):
            out = layer(out, src_mask=m, pos=pos)
        if self.norm is not None:
            out = self.norm(out)
        return xyz, out, None

    @staticmethod
    def _head_mask(m, layer):
        if m is None:
            return None
        bsz, n, _ = m.shape
        return m.unsqueeze(1).expand(bsz, layer.nhead, n, n).reshape(bsz * layer.nhead, n, n)

    def _fused_ok(self, x):
        """HIP residual + LayerNorm launches (resnorm.py) under bf16 autocast"""
        return (all(hasattr(l, "fused_ok") and l.fused_ok(x) for l in self.layers)
                and (self.norm is None or rn.supported(x, self.norm)))

    def _finish_fused(self, pend):
        """the encoder output (fp32): last residual add (+ the encoder norm)"""
        s, _, _, xb = rn.resnorm(pend, norm_b=self.norm)
        return xb if self.norm is not None else s


class MaskedTransformerEncoder(TransformerEncoder):
    """Radius-masked encoder with interim SA downsampling after layer 0
    (reference transformer.py:144-209; mask = cdist(xyz) >= radius**2, quirk Q5)."""

    def __init__(self, encoder_layer, num_layers, masking_radius, interim_downsampling, norm=None,
                 weight_init_name="xavier_uniform"):
        super().__init__(encoder_layer, num_layers, norm=norm, weight_init_name=weight_init_name)
        if len(masking_radius) != num_layers:
            raise ValueError("one masking radius per layer")
        self.masking_radius = masking_radius
        self.interim_downsampling = interim_downsampling

    @torch.no_grad()
    def compute_mask(self, xyz, radius, dist=None):
        if dist is None or dist.shape[1] != xyz.shape[1]:
            dist = torch.cdist(xyz.float(), xyz.float(), p=2)
        return dist >= radius, dist

    def forward(self, src, mask=None, src_key_padding_mask=None, pos=None, xyz=None,
                transpose_swap=False):
        out = src
        xyz_dist = None
        xyz_inds = None
        fused = self._fused_ok(src)
        pend = rn.Pending(src, None, 0.0, 0)
        for idx, layer in enumerate(self.layers):
            m = None
            if self.masking_radius[idx] > 0:
                m, xyz_dist = self.compute_mask(xyz, self.masking_radius[idx], xyz_dist)
                m = self._head_mask(m, layer)
            if fused:
                pend = layer.forward_fused(pend, src_mask=m, pos=pos)
            else:
                out = layer(out, src_mask=m, pos=pos)
            if idx == 0 and self.interim_downsampling:
                if fused:
                    out = rn.resnorm(pend)[0]
                xyz, feats, xyz_inds = self.interim_downsampling(xyz, out.permute(1, 2, 0))
                out = feats.permute(2, 0, 1)
                pend = rn.Pending(out, None, 0.0, 0)
        if fused:
            return xyz, self._finish_fused(pend), xyz_inds
        if self.norm is not None:
            out = self.norm(out)
        return xyz, out, xyz_inds


class TransformerDecoder(nn.Module):
    def __init__(self, decoder_layer, num_layers, norm_fn_name="ln", return_intermediate=False,
                 weight_init_name="xavier_uniform"):
        super().__init__()
        self.layers = get_clones(decoder_layer, num_layers)
        self.num_layers = num_layers
        self.norm = NORM_DICT[norm_fn_name](self.layers[0].linear2.out_features) \
            if norm_fn_name is not None else None
        self.return_intermediate = return_intermediate
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, tgt_key_padding_mask=None,
                memory_key_padding_mask=None, pos=None, query_pos=None, transpose_swap=False,
                return_attn_weights=False):
        if transpose_swap or return_attn_weights:
            raise NotImplementedError
        memory_pos = memory if pos is None else memory + pos
        if all(hasattr(l, "fused_ok") and l.fused_ok(tgt) for l in self.layers) and \
                (self.norm is None or rn.supported(tgt, self.norm)):
            return self._forward_fused(tgt, memory, memory_pos, query_pos, tgt_mask, memory_mask)
        out = tgt
        inter = []
        for layer in self.layers:
            out, _ = layer(out, memory, tgt_mask=tgt_mask, memory_mask=memory_mask,
                           query_pos=query_pos, memory_pos=memory_pos)
            if self.return_intermediate:
                inter.append(self.norm(out))
        if self.norm is not None:
            out = self.norm(out)
            if self.return_intermediate:
                inter[-1] = out
        if self.return_intermediate:
            return torch.stack(inter), []
        return out, []

    def _forward_fused(self, tgt, memory, memory_pos, query_pos, tgt_mask, memory_mask):
        """bf16: one resnorm launch per sub-layer boundary; the decoder norm of layer i's
        output shares the launch with layer i+1's norm1 (same row statistics)."""
        # K / V projection inputs are cast to bf16 once for the 8 layers
        memory = memory.to(torch.bfloat16)
        memory_pos = memory_pos.to(torch.bfloat16)
        pend = rn.Pending(tgt, None, 0.0, 0)
        inter = []
        dec_norm = self.norm if self.return_intermediate else None
        for i, layer in enumerate(self.layers):
            s, x, xp, xd = rn.resnorm(pend, layer.norm1, pos=query_pos, want_a=True,
                                      want_ap=query_pos is not None,
                                      norm_b=dec_norm if i > 0 else None)
            if i > 0 and dec_norm is not None:
                inter.append(xd)
            pend = layer.forward_fused(s, x, xp, memory, memory_pos, query_pos, tgt_mask,
                                       memory_mask)
        s, _, _, xd = rn.resnorm(pend, norm_b=self.norm)
        out = xd if self.norm is not None else s
        if self.return_intermediate:
            if self.norm is None:
                raise NotImplementedError("return_intermediate without a decoder norm")
            inter.append(out)
            return torch.stack(inter), []
        return out, []
