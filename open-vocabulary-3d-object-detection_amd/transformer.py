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
import os
from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from . import _native
from . import attention as flash
from . import resnorm as rn
from . import gemm
from .gemm import cast_param, in_projection, rows_linear
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

    def _out(self, out, defer):
        """the output projection, or (defer) a resnorm.LinY the next resnorm launch computes"""
        if defer:
            return rn.LinY(out, self.out_proj.weight, self.out_proj.bias)
        return rows_linear(out, self.out_proj.weight, self.out_proj.bias)

    def forward(self, query, key, value, attn_mask: Optional[Tensor] = None, defer_out=False):
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
        packed = isinstance(attn_mask, flash.PackedMask)
        if srcs[0].dtype == torch.bfloat16 and flash.supported(srcs[0], E, self.num_heads,
                                                               attn_mask):
            # HIP flash attention straight on the projection rows (csrc/attn.hip)
            out = flash.attention_packed(srcs, spec, L, S, self.num_heads,
                                         dropout_p=self.dropout if self.training else 0.0,
                                         site=self.site, mask=attn_mask if packed else None)
            return self._out(out, defer_out)
        if packed:
            raise ValueError("a PackedMask needs the HIP attention path (bf16, head_dim 64)")
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


    def attend(self, srcs, spec, L, S, defer_out=False):
        """the flash path on already-projected rows (srcs / spec as attention.attention_packed:
        the in-projection ran elsewhere, e.g. inside the norm's launch, resnorm.resnorm_gemm)"""
        out = flash.attention_packed(srcs, spec, L, S, self.num_heads,
                                     dropout_p=self.dropout if self.training else 0.0,
                                     site=self.site)
        return self._out(out, defer_out)

    def forward_kv(self, query, kv, idx, defer_out=False, q=None):
        """Cross attention whose K / V projections of the memory were computed for all decoder
        layers at once (MemoryKV): kv = (K_all, V_all, dK_all, dV_all, token, token_grad),
        this layer's block = columns idx*E .. (idx+1)*E.  q: the query projection when it was
        already computed (then `query` only gives the shape)."""
        L, B, E = query.shape
        K_all, V_all, dK, dV, token, tok_grad = kv
        S = K_all.shape[0]
        if q is None:
            q = in_projection(self.in_proj_weight, self.in_proj_bias, ((query, 0, E),))[0]
        out = flash.attention_packed(
            [q, K_all, V_all], ((0, 0), (1, idx * E), (2, idx * E)), L, S, self.num_heads,
            dropout_p=self.dropout if self.training else 0.0, site=self.site,
            ext=((None, dK, dV), token, tok_grad))
        return self._out(out, defer_out)


class _MemoryKV(torch.autograd.Function):
    """K and V of the decoder's cross attention for all L layers in two GEMMs:
    K_all = (memory + pos) [Wk_0 .. Wk_{L-1}]^T + bk, V_all = memory [Wv_0 ..]^T + bv, each
    (S, B, L*E) bf16 (reference transformer.py:365-372 projects the same memory once per
    layer).  The layers' attention backward writes dK / dV column blocks into the shared
    buffers; the ``token`` output carries the dependency so this backward runs after all of
    them: d memory = dV_all Wv_all + dK_all Wk_all (one GEMM + one accumulating GEMM), and
    the K / V rows of every in_proj weight gradient (deferred with the others when
    gemm.DEFER_WGRAD, else returned)."""

    @staticmethod
    def forward(ctx, memory, pos, E, *params):
        ws, bs = params[0::2], params[1::2]
        S, B, C = memory.shape
        bf = torch.bfloat16
        if (pos is not None and memory.dtype in (torch.float32, bf) and pos.dtype == torch.float32
                and memory.is_contiguous() and pos.is_contiguous() and pos.shape == memory.shape
                and memory.numel() % 8 == 0):
            # bf16(memory + pos) summed in fp32 and rounded once (torch's GPU add into a bf16
            # output rounded the fp32 pos to bf16 first), and bf16(memory) for fp32 memory, in
            # one pass over the rows
            a_bf16 = memory.dtype == bf
            mem = memory.view(S * B, C) if a_bf16 else torch.empty((S * B, C), dtype=bf,
                                                                    device=memory.device)
            mpos = torch.empty((S * B, C), dtype=bf, device=memory.device)
            _native.call("ov3d_add_cast_bf16", memory, int(a_bf16), pos, memory.numel(), mpos,
                         None if a_bf16 else mem, like=memory)
        else:
            mem = memory.reshape(S * B, C).to(bf).contiguous()
            mpos = mem
            if pos is not None:   # the sum in the inputs' common type, rounded once on the store
                mpos = torch.empty((S * B, C), dtype=bf, device=memory.device)
                torch.add(memory, pos, out=mpos.view(S, B, C))
        # the K / V row blocks of every layer's bf16 in_proj copy, gathered in one launch
        n = len(ws) * E
        dev = memory.device
        Wk, Wv = (torch.empty((n, C), dtype=bf, device=dev) for _ in range(2))
        bk, bv = (torch.empty(n, dtype=bf, device=dev) for _ in range(2))
        srcs, dsts = [], []
        for l, (w, b) in enumerate(zip(ws, bs)):
            wc, bc = cast_param(w, bf), cast_param(b, bf)
            rows = slice(l * E, (l + 1) * E)
            srcs += [wc[E:2 * E], wc[2 * E:], bc[E:2 * E], bc[2 * E:]]
            dsts += [Wk[rows], Wv[rows], bk[rows], bv[rows]]
        _native.multi_copy(dsts, srcs)
        # both products in one launch of the 256 x 256 tile kernel (csrc/gemm256.hip; 256 x 256
        # tiles read 4 bytes of operands per output from L2 where the long row-block kernel's
        # 64 x 128 tiles read 12); the library GEMMs when it does not apply
        if gemm.gemm256_ok(mpos, Wk) and gemm.gemm256_ok(mem, Wv) and mpos.stride(0) == mem.stride(0):
            K_all, V_all = gemm.gemm256_pair(mpos, Wk, bk, mem, Wv, bv)
            K_all, V_all = K_all.view(S, B, n), V_all.view(S, B, n)
        else:
            K_all = torch.addmm(bk, mpos, Wk.t()).view(S, B, n)
            V_all = torch.addmm(bv, mem, Wv.t()).view(S, B, n)
        dK, dV = torch.empty_like(K_all), torch.empty_like(V_all)
        flash.defer_kv_grads(dK)   # the layers' dK / dV run batched in this op's backward
        token = torch.empty((), dtype=torch.float32, device=memory.device)
        tok_grad = _zero_scalar(memory.device)
        ctx.save_for_backward(mem, mpos, Wk, Wv)
        ctx.meta = (E, memory.dtype, pos is not None and pos.requires_grad, len(ws), S * B, C)
        ctx.bufs = (dK, dV)
        ctx.params = params
        ctx.mark_non_differentiable(K_all, V_all, dK, dV, tok_grad)
        ctx.set_materialize_grads(False)
        return K_all, V_all, dK, dV, token, tok_grad

    @staticmethod
    def backward(ctx, _k, _v, _dk, _dv, _tok, _tg):
        mem, mpos, Wk, Wv = ctx.saved_tensors
        E, mdt, pos_grad, L, R, C = ctx.meta
        flash.flush_kv_grads(ctx.bufs[0])   # the deferred dK / dV of every layer, one launch
        dK, dV = (t.view(R, L * E) for t in ctx.bufs)
        params = ctx.params
        with torch.autocast("cuda", enabled=False):
            if not pos_grad and gemm._tile_gemm_ok(dK, Wk, False) and gemm._tile_gemm_ok(dV, Wv, False):
                dmem = gemm.tile_gemm2(dK, Wk, dV, Wv)   # dK Wk + dV Wv in one launch
            else:
                dmk = dK @ Wk
                # in place when dmk is not also pos's gradient (no copy of dmk into a new output)
                dmem = dmk.addmm_(dV, Wv) if not pos_grad else dV @ Wv + dmk
            grads = [None] * len(params)
            for l in range(L):
                w, b = params[2 * l], params[2 * l + 1]
                for blk, (dy, x) in enumerate(((dK, mpos), (dV, mem))):
                    r0 = (1 + blk) * E
                    dyl = dy[:, l * E:(l + 1) * E]
                    if gemm.can_defer(x, w, b):
                        gemm.defer_weight_grad(dyl, x, w, b, rows=(r0, r0 + E))
                        continue
                    if grads[2 * l] is None:
                        grads[2 * l] = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
                        grads[2 * l + 1] = torch.zeros(b.shape, dtype=torch.float32, device=b.device)
                    gemm.fused_weight_grad(dyl, x, bias=True, out_w=grads[2 * l][r0:r0 + E],
                                           out_b=grads[2 * l + 1][r0:r0 + E])
        shape = ctx.bufs[0].shape[:2] + (C,)
        dpos = dmk.view(shape).to(mdt) if pos_grad else None
        return (dmem.view(shape).to(mdt), dpos, None, *grads)


_ZEROS = {}


def _zero_scalar(device):
    """a device 0.0 that nothing writes: allocated once (not zero-filled in every step)"""
    z = _ZEROS.get(device)
    if z is None:
        z = torch.zeros((), dtype=torch.float32, device=device)
        _ZEROS[device] = z
    return z


def memory_kv_ok(layers, memory):
    """the batched K / V path: bf16 autocast on the device, every cross attention a flash
    shape (head_dim 64, no mask) with its own in_proj weight / bias"""
    if not (memory.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    for l in layers:
        a = getattr(l, "multihead_attn", None)
        if not isinstance(a, MultiheadAttention) or a.embed_dim != a.num_heads * flash.HEAD_DIM \
                or a.in_proj_bias is None:
            return False
    return True


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
        y = self.self_attn(qk, qk, x, attn_mask=src_mask, defer_out=self.use_ffn)
        if not self.use_ffn:
            return rn.Pending(s, y, p1, site1)
        s, x, _, _ = rn.resnorm(rn.Pending(s, y, p1, site1), self.norm2)
        y = rn.ffn(x, self.linear1, self.linear2, self.activation, self.dropout, site_ffn)
        return rn.Pending(s, y, p2, site2)

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
                      memory_mask=None, kv=None, idx=0, pos_fan=None):
        """bf16 step from norm1's outputs (x = norm1(tgt), xp = x + query_pos) -> Pending of
        the layer output (resnorm.py)."""
        p1, p2, p3 = ((self.dropout1.p, self.dropout2.p, self.dropout3.p) if self.training
                      else (0.0, 0.0, 0.0))
        site1, site2, site3, site_ffn = rn.sites(self, 4)
        qk = xp if query_pos is not None else x
        y = self.self_attn(qk, qk, x, attn_mask=tgt_mask, defer_out=True)
        s, x2, q, _ = rn.resnorm(rn.Pending(s, y, p1, site1), self.norm2, pos=query_pos,
                                 want_a=query_pos is None, want_ap=query_pos is not None,
                                 pos_fan=pos_fan)
        qx = q if query_pos is not None else x2
        if kv is not None and memory_mask is None:
            y = self.multihead_attn.forward_kv(qx, kv, idx, defer_out=True)
        else:
            y = self.multihead_attn(qx, memory_pos, memory, attn_mask=memory_mask, defer_out=True)
        s, x3, _, _ = rn.resnorm(rn.Pending(s, y, p2, site2), self.norm3)
        y = rn.ffn(x3, self.linear1, self.linear2, self.activation, self.dropout, site_ffn)
        return rn.Pending(s, y, p3, site3)

    def fused_ok(self, x):
        return rn.supported(x, self.norm1, self.norm2, self.norm3)

    def ln_ok(self, tgt, query_pos, tgt_mask, memory_mask, kv):
        """forward_fused_ln applies: the fused boundary launches (csrc/lngemm.hip), flash
        shapes, batched memory K / V, the FFN's ReLU, bf16 row widths the kernels take"""
        sa, ca = self.self_attn, self.multihead_attn
        E = sa.embed_dim
        R = tgt.shape[0] * tgt.shape[1] if tgt.dim() == 3 else 0
        if not (rn.lngemm and kv is not None and tgt_mask is None and memory_mask is None
                and tgt.dim() == 3 and isinstance(self.activation, nn.ReLU)
                and sa.in_proj_bias is not None and ca.in_proj_bias is not None
                and self.linear1.bias is not None and self.linear2.bias is not None
                and flash.supported(tgt, E, sa.num_heads, None)):
            return False
        lib = _native.load()
        F = self.linear1.out_features
        return all(lib.ov3d_lngemm_supported(R, E, n) for n in (E, 2 * E, 3 * E, F)) and \
            self.linear2.out_features == E and self.linear1.in_features == E and \
            bool(lib.ov3d_lngemm_supported(R, E, self.linear2.in_features))

    def forward_fused_ln(self, pend, query_pos, kv, idx, pos_fan, norm_b=None, norm_b_fan=None,
                         xb_into=None):
        """bf16 step of the whole layer from the previous layer's Pending residual, every
        norm fused with the linear layer after it (norm1 -> in-projection, norm2 -> the cross
        attention's query projection, norm3 -> linear1 + ReLU + dropout: resnorm.resnorm_gemm)
        and linear2 left to the next boundary's launch (LinY).  norm_b: the decoder norm of
        the previous layer's output, computed by norm1's launch.  -> (Pending, xb)."""
        sa, ca = self.self_attn, self.multihead_attn
        E = sa.embed_dim
        p1, p2, p3, pf = ((self.dropout1.p, self.dropout2.p, self.dropout3.p, self.dropout.p)
                          if self.training else (0.0, 0.0, 0.0, 0.0))
        site1, site2, site3, site_ffn = rn.sites(self, 4)
        hp = query_pos is not None
        spec = ((1, 0, 2 * E), (0, 2 * E, 3 * E)) if hp else ((0, 0, 3 * E),)
        r = rn.resnorm_gemm(pend, self.norm1, sa.in_proj_weight, sa.in_proj_bias, spec,
                            pos=query_pos, norm_b=norm_b, pos_fan=pos_fan, norm_b_fan=norm_b_fan,
                            xb_into=xb_into)
        if r is None:
            return None
        s, xd, outs = r
        L = s.shape[0]
        aspec = ((0, 0), (0, E), (1, 0)) if hp else ((0, 0), (0, E), (0, 2 * E))
        y = sa.attend(outs, aspec, L, L, defer_out=True)
        s, _, (q,) = rn.resnorm_gemm(rn.Pending(s, y, p1, site1), self.norm2, ca.in_proj_weight,
                                     ca.in_proj_bias, ((1 if hp else 0, 0, E),), pos=query_pos,
                                     pos_fan=pos_fan)
        y = ca.forward_kv(s, kv, idx, defer_out=True, q=q.view(s.shape))
        F = self.linear1.out_features
        s, _, (h,) = rn.resnorm_gemm(rn.Pending(s, y, p2, site2), self.norm3, self.linear1.weight,
                                     self.linear1.bias, ((0, 0, F),), epi=(pf, site_ffn))
        return rn.Pending(s, rn.LinY(h, self.linear2.weight, self.linear2.bias, pf), p3, site3), xd


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


# the masked encoder's mask straight from the points (attention.pack_mask_points); 0: cdist's
# squared-distance GEMM + the kind-2 packing
POINT_MASK = os.environ.get("OV3D_POINT_MASK", "1") != "0"


def euclid_sq(x):
    """torch.cdist(x, x, p=2) for > 25 points (the matmul form, ATen _euclidean_dist) before its
    clamp_min(0).sqrt(): the same fp32 operations and GEMM, outside autocast as cdist runs."""
    with torch.autocast("cuda", enabled=False):
        x = x.float()
        xn = x.pow(2).sum(-1, keepdim=True)
        pad = torch.ones_like(xn)
        return torch.cat([x.mul(-2), xn, pad], -1).matmul(torch.cat([x, pad, xn], -1).mT)


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
        if dist is None or dist[0] != "dist" or dist[1].shape[1] != xyz.shape[1]:
            dist = ("dist", torch.cdist(xyz.float(), xyz.float(), p=2))
        return dist[1] >= radius, dist

    @torch.no_grad()
    def _packed_mask(self, xyz, radius, dist=None):
        """the same mask as compute_mask, packed for the HIP attention kernels straight from
        cdist's matmul-form squared distances, its clamp and sqrt fused into the packing (no
        (B, L, L) distance or (B*H, L, L) bool tensor)"""
        if POINT_MASK:   # the distances inside the packing launch (no GEMM, no L x L matrix)
            return flash.pack_mask_points(xyz, float(radius)), ("pts", None)
        if dist is None or dist[0] != "sq" or dist[1].shape[1] != xyz.shape[1]:
            dist = ("sq", euclid_sq(xyz))
        return flash.pack_mask(dist[1], float(radius), squared=True), dist

    @staticmethod
    def _packed_ok(layer, src):
        a = getattr(layer, "self_attn", None)
        return (isinstance(a, MultiheadAttention) and src.is_cuda and src.shape[0] % 32 == 0
                and a.embed_dim == a.num_heads * flash.HEAD_DIM and layer.nhead == a.num_heads)

    def forward(self, src, mask=None, src_key_padding_mask=None, pos=None, xyz=None,
                transpose_swap=False, interim_plan=None):
        """interim_plan: (inds, new_xyz, ball, (inverse offsets, rows)) of the interim SA
        computed ahead of time from the same points (Model3DETR.sampling_plan); identical
        results."""
        out = src
        xyz_dist = None
        xyz_inds = None
        fused = self._fused_ok(src)
        pend = rn.Pending(src, None, 0.0, 0)
        for idx, layer in enumerate(self.layers):
            m = None
            if self.masking_radius[idx] > 0:
                if fused and self._packed_ok(layer, out if idx else src):
                    m, xyz_dist = self._packed_mask(xyz, self.masking_radius[idx], xyz_dist)
                else:
                    m, xyz_dist = self.compute_mask(xyz, self.masking_radius[idx], xyz_dist)
                    m = self._head_mask(m, layer)
            if fused:
                pend = layer.forward_fused(pend, src_mask=m, pos=pos)
            else:
                out = layer(out, src_mask=m, pos=pos)
            if idx == 0 and self.interim_downsampling:
                if fused:
                    out = rn.resnorm(pend)[0]
                if interim_plan is not None:
                    inds, nxyz, ball, inv = interim_plan
                    xyz, feats, xyz_inds = self.interim_downsampling(
                        xyz, out.permute(1, 2, 0), inds=inds, new_xyz=nxyz, ball=ball, inverse=inv)
                else:
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
        if all(hasattr(l, "fused_ok") and l.fused_ok(tgt) for l in self.layers) and \
                (self.norm is None or rn.supported(tgt, self.norm)):
            return self._forward_fused(tgt, memory, pos, query_pos, tgt_mask, memory_mask)
        memory_pos = memory if pos is None else memory + pos
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

    def _forward_fused(self, tgt, memory, pos, query_pos, tgt_mask, memory_mask):
        """bf16: one resnorm launch per sub-layer boundary; the decoder norm of layer i's
        output shares the launch with layer i+1's norm1 (same row statistics)."""
        kv = None
        memory_pos = None
        if memory_mask is None and memory_kv_ok(self.layers, memory):
            # K / V of all layers' cross attention: two GEMMs over the memory (_MemoryKV)
            params = []
            for l in self.layers:
                params += [l.multihead_attn.in_proj_weight, l.multihead_attn.in_proj_bias]
            kv = _MemoryKV.apply(memory, pos, self.layers[0].multihead_attn.embed_dim, *params)
        else:
            memory_pos = memory if pos is None else memory + pos
            # K / V projection inputs are cast to bf16 once for the 8 layers
            memory = memory.to(torch.bfloat16)
            memory_pos = memory_pos.to(torch.bfloat16)
        hook = getattr(self, "after_memory_kv", None)
        if hook is not None:   # graphs.StepGraph: where the step's graph is split
            hook()
        pend = rn.Pending(tgt, None, 0.0, 0)
        inter = []
        dec_norm = self.norm if self.return_intermediate else None
        # the layer outputs (decoder norm) go straight into the heads' bf16 (L, B, Q, C) rows
        outs = None
        if dec_norm is not None and tgt.dim() == 3 and getattr(self, "rows_bf16", True):
            Q, B, C = tgt.shape
            outs = torch.empty((len(self.layers), B, Q, C), dtype=torch.bfloat16, device=tgt.device)
        # query_pos and the decoder norm are read by many launches: one gradient buffer each
        pos_fan, nb_fan = rn.FanIn(), rn.FanIn()
        for i, layer in enumerate(self.layers):
            kvi = None
            if kv is not None:   # the token gradient is returned once (by layer 0)
                kvi = kv[:5] + ((kv[5] if i == 0 else None),)
            xb_into = (outs, i - 1) if outs is not None and i > 0 else None
            r = None
            if layer.ln_ok(tgt, query_pos, tgt_mask, memory_mask, kvi):
                # every norm fused with the linear layer after it (csrc/lngemm.hip)
                r = layer.forward_fused_ln(pend, query_pos, kvi, i, pos_fan,
                                           norm_b=dec_norm if i > 0 else None, norm_b_fan=nb_fan,
                                           xb_into=xb_into)
            if r is not None:
                pend, xd = r
            else:
                s, x, xp, xd = rn.resnorm(pend, layer.norm1, pos=query_pos, want_a=True,
                                          want_ap=query_pos is not None,
                                          norm_b=dec_norm if i > 0 else None, pos_fan=pos_fan,
                                          norm_b_fan=nb_fan, xb_into=xb_into)
            if i > 0 and dec_norm is not None:
                inter.append(xd)
            if r is None:
                pend = layer.forward_fused(s, x, xp, memory, memory_pos, query_pos, tgt_mask,
                                           memory_mask, kv=kvi, idx=i, pos_fan=pos_fan)
        s, _, _, xd = rn.resnorm(pend, norm_b=self.norm, norm_b_fan=nb_fan,
                                 xb_into=(outs, len(self.layers) - 1) if outs is not None else None)
        out = xd if self.norm is not None else s
        if self.return_intermediate:
            if self.norm is None:
                raise NotImplementedError("return_intermediate without a decoder norm")
            inter.append(out)
            if outs is not None:
                return rn.Gather.apply(outs, *inter), []
            return torch.stack(inter), []
        return out, []
