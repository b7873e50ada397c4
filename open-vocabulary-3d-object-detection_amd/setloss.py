"""The set criterion's losses for all decoder layers as one HIP launch each way
(csrc/setloss.hip, ``ov3d_set_loss_fwd`` / ``ov3d_set_loss_bwd``).

Reference: criterion.py SetCriterion.loss_sem_cls (143-178), loss_angle (180-246),
loss_center (248-272), loss_giou (274-296), loss_size (298-337), loss_cardinality
(121-130) and the per-layer weighting + layer sum of forward (402-442).  The torch
expression of the same terms stays in criterion.py (``SetCriterion._losses_torch``) and
is the CPU / fp32 restatement the GPU tests compare against.

The forward returns the (L, 8) table of weighted dict values (rows: final layer, aux 0,
aux 1, ...; columns: ``COLUMNS``) and the total; loss_dict entries are views of the
table.  The backward writes the gradients of the head outputs the terms read (class
logits, angle logits / residuals, normalised centre / size, the GIoU matrix when the
GIoU term is weighted, the per-layer 2D alignment sums) in one launch.
"""
import ctypes
import math

import torch

from . import _native

COLUMNS = ("loss_sem_cls", "loss_angle_cls", "loss_angle_reg", "loss_center", "loss_size",
           "loss_giou", "loss_2dalignment", "loss_cardinality")
SEM, CENTER, SIZE, GIOU, ALIGN = 1, 2, 4, 8, 16
MAX_B = 256
_P = ctypes.c_void_p
_L = ctypes.c_longlong


class Desc(ctypes.Structure):
    """mirror of ov3d_set_loss_desc (include/ov3d.h)"""
    _fields_ = [("L", ctypes.c_int), ("B", ctypes.c_int), ("Q", ctypes.c_int), ("G", ctypes.c_int),
                ("T", ctypes.c_int), ("NB", ctypes.c_int), ("flags", ctypes.c_int),
                ("final_last", ctypes.c_int), ("match_ref_order", ctypes.c_int),
                ("logits", _P), ("ld_logits", _L), ("angle_logits", _P), ("ld_angle_logits", _L),
                ("angle_res", _P), ("ld_angle_res", _L), ("center", _P), ("ld_center", _L),
                ("size", _P), ("ld_size", _L), ("gious", _P), ("inds", _P), ("matched", _P),
                ("gt_sem", _P), ("gt_angle_cls", _P), ("gt_angle_res", _P), ("gt_center", _P),
                ("gt_size", _P), ("nactual", _P), ("cls_weights", _P), ("num_boxes", _P),
                ("align", _P), ("dict_w", ctypes.c_float * 8), ("total_w", ctypes.c_float * 8),
                ("total_order", ctypes.c_int * 8), ("n_total", ctypes.c_int),
                ("res_scale", ctypes.c_float), ("match_status", _P), ("n_status", ctypes.c_int)]


_checked = False
_tickets = {}


def _layout_check():
    global _checked
    if not _checked:
        n = _native.load().ov3d_set_loss_desc_size()
        if n != ctypes.sizeof(Desc):
            raise _native.NativeError(f"ov3d_set_loss_desc: library {n} B != ctypes {ctypes.sizeof(Desc)} B")
        _checked = True


def _ticket(dev):
    """one zero int per device; the forward kernel leaves it at zero again"""
    t = _tickets.get(dev)
    if t is None:
        t = torch.zeros(1, dtype=torch.int32, device=dev)
        _tickets[dev] = t
    return t


def rows(t):
    """(tensor, row stride) describing t as (prod(shape[:-1]), shape[-1]) rows with unit
    column stride; a copy only when t is not of that form (e.g. a transposed view)."""
    if t.dtype != torch.float32:
        t = t.float()
    n = t.shape[-1]
    if t.stride(-1) == 1 or n == 1:
        ld = t.stride(-2) if t.dim() > 1 and t.shape[-2] > 1 else n
        ok, exp = ld >= n, ld
        for d in range(t.dim() - 2, -1, -1):
            if t.shape[d] != 1 and t.stride(d) != exp:
                ok = False
                break
            exp *= t.shape[d]
        if ok:
            return t, ld
    return t.contiguous(), n


def supported(logits):
    return logits.is_cuda


def _res_scale(nb):
    """torch's (tensor / python float) multiplies by the fp32 reciprocal of the fp32 divisor"""
    return float(torch.tensor(1.0, dtype=torch.float32) / torch.tensor(math.pi / nb, dtype=torch.float32))


SPLIT_FWD = True   # ov3d_set_loss_fwd_split (tests compare it with the per-layer launch)


class _SetLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, logits, angle_logits, angle_res, center, size, gious, align, aux):
        desc, keep = meta
        dev = logits.device
        L = desc.L
        raw = torch.empty((L, 9), dtype=torch.float32, device=dev)
        table = torch.empty((L, 8), dtype=torch.float32, device=dev)
        total = torch.empty((), dtype=torch.float32, device=dev)
        n = _native.load().ov3d_set_loss_fwd_parts(L, desc.B, desc.Q) if SPLIT_FWD else 0
        if n > 0:   # a workgroup per (256 proposals, layer) instead of one per layer
            parts = torch.empty((n,), dtype=torch.float64, device=dev)
            _native.call("ov3d_set_loss_fwd_split", ctypes.addressof(desc), raw, _ticket(dev),
                         table, total, parts, like=logits)
        else:
            _native.call("ov3d_set_loss_fwd", ctypes.addressof(desc), raw, _ticket(dev), table,
                         total, like=logits)
        ctx.meta = meta
        ctx.shapes = tuple(t.shape if t is not None else None
                           for t in (logits, angle_logits, angle_res, center, size, gious, align))
        ctx.save_for_backward(raw)
        ctx.set_materialize_grads(False)
        return table, total

    @staticmethod
    def backward(ctx, d_table, d_total):
        desc, keep = ctx.meta
        (raw,) = ctx.saved_tensors
        dev = raw.device
        need = ctx.needs_input_grad
        shapes = ctx.shapes
        fl = desc.flags

        def out(i, cond=True):
            if not (need[i + 1] and cond and shapes[i] is not None):
                return None
            return torch.empty(shapes[i], dtype=torch.float32, device=dev)

        g = [out(0, fl & SEM), out(1), out(2), out(3, fl & CENTER), out(4, fl & SIZE),
             out(5, fl & GIOU), out(6, fl & ALIGN)]
        if any(x is not None for x in g):
            dt = d_table.float().contiguous() if d_table is not None else None
            dtot = d_total.float().reshape(1) if d_total is not None else None
            _native.call("ov3d_set_loss_bwd", ctypes.addressof(desc), raw, dt, dtot, *g, like=raw)
        return (None, *g, None)


def set_losses(L, B, Q, final_last, logits, angle_logits, angle_res, center, size, gious, align,
               inds, matched, targets, cls_weights, num_boxes, dict_w, total_w, total_order,
               match_ref_order=False, match_status=None):
    """-> table (L, 8) of weighted values (rows in dict order), total (0-d).
    match_status: the matcher's per-problem status (device): any nonzero -> total NaN.

    logits (L*B, Q, T) ..., gious (L*B, Q, G) or None, align (L,) or None, inds / matched
    (L*B, Q), dict_w / total_w: 8 floats per COLUMNS entry, total_order: column indices."""
    _layout_check()
    _native.check_device(logits, "set_losses logits")
    if B > MAX_B:
        raise ValueError(f"set_losses: at most {MAX_B} scenes per replica")
    dev = logits.device
    keep = []

    def dev_t(t, dtype):
        t = t.to(device=dev, dtype=dtype).contiguous()
        keep.append(t)
        return t

    lg, ld_lg = rows(logits)
    al, ld_al = rows(angle_logits)
    ar, ld_ar = rows(angle_res)
    ce, ld_ce = rows(center) if center is not None else (None, 3)
    sz, ld_sz = rows(size) if size is not None else (None, 3)
    keep += [lg, al, ar, ce, sz]
    gi = dev_t(gious, torch.float32) if gious is not None else None
    an = dev_t(align, torch.float32) if align is not None else None
    G = targets["gt_box_sem_cls_label"].shape[1]
    T, NB = logits.shape[-1], angle_logits.shape[-1]
    d = Desc()
    d.L, d.B, d.Q, d.G, d.T, d.NB = L, B, Q, G, T, NB
    d.flags = ((SEM if cls_weights is not None else 0) | (CENTER if center is not None else 0)
               | (SIZE if size is not None else 0) | (GIOU if gious is not None else 0)
               | (ALIGN if align is not None else 0))
    d.final_last = int(final_last)
    d.match_ref_order = int(match_ref_order)
    d.logits, d.ld_logits = lg.data_ptr(), ld_lg
    d.angle_logits, d.ld_angle_logits = al.data_ptr(), ld_al
    d.angle_res, d.ld_angle_res = ar.data_ptr(), ld_ar
    d.center, d.ld_center = (ce.data_ptr() if ce is not None else None), ld_ce
    d.size, d.ld_size = (sz.data_ptr() if sz is not None else None), ld_sz
    d.gious = gi.data_ptr() if gi is not None else None
    d.inds = dev_t(inds, torch.int64).data_ptr()
    d.matched = dev_t(matched, torch.float32).data_ptr()
    d.gt_sem = dev_t(targets["gt_box_sem_cls_label"], torch.int64).data_ptr()
    d.gt_angle_cls = dev_t(targets["gt_angle_class_label"], torch.int64).data_ptr()
    d.gt_angle_res = dev_t(targets["gt_angle_residual_label"], torch.float32).data_ptr()
    d.gt_center = dev_t(targets["gt_box_centers_normalized"], torch.float32).data_ptr()
    d.gt_size = dev_t(targets["gt_box_sizes_normalized"], torch.float32).data_ptr()
    d.nactual = dev_t(targets["nactual_gt"], torch.int64).data_ptr()
    d.cls_weights = dev_t(cls_weights, torch.float32).data_ptr() if cls_weights is not None else None
    d.num_boxes = dev_t(num_boxes.reshape(1), torch.float32).data_ptr()
    d.align = an.data_ptr() if an is not None else None
    for k in range(8):
        d.dict_w[k] = dict_w[k]
        d.total_w[k] = total_w[k]
    for j, k in enumerate(total_order):
        d.total_order[j] = k
    d.n_total = len(total_order)
    d.res_scale = _res_scale(NB)
    if match_status is not None:
        st = dev_t(match_status, torch.int32)
        d.match_status, d.n_status = st.data_ptr(), st.numel()
    return _SetLoss.apply((d, keep), logits, angle_logits, angle_res, center, size, gious, align,
                          None)


def target_counts(present, targets, L):
    """-> nactual (B,) int64, nactual repeated for the L layers (L*B,) int32, num_boxes (device
    scalar: max(total, 1), all-reduce-averaged across ranks), rotated flag (int32), the
    replica's total (int64) — criterion.py:346-352, 425 in ONE launch (ov3d_targets_prep)."""
    from .dist import all_reduce_average, get_world_size
    B, G = present.shape
    dev = present.device
    nact = torch.empty(B, dtype=torch.int64, device=dev)
    nrep = torch.empty(L * B, dtype=torch.int32, device=dev)
    total = torch.empty((), dtype=torch.int64, device=dev)
    rotated = torch.empty((), dtype=torch.int32, device=dev)
    single = get_world_size() == 1
    nb = torch.empty((), dtype=torch.float32, device=dev) if single else None
    _native.call("ov3d_targets_prep", B, G, L, present.float().contiguous(),
                 targets["gt_box_angles"].float().contiguous(), nact, nrep, total, nb, rotated,
                 like=present)
    if not single:
        nb = torch.clamp(all_reduce_average(total), min=1)
    return nact, nrep, nb, rotated, total


def matcher_cost(prob, obj, center, gious, targets, B, weights, final_last=False):
    """Matcher.cost (criterion.py:54-62) with the center cdist(p=1) of 357-360 for the L*B
    problems in one launch (ov3d_matcher_cost) -> (L*B, Q, G), in the reference's problem
    order (final layer first) when final_last."""
    pr, ldp = rows(prob)
    ob = obj.float().contiguous()
    ce = center.float().contiguous()
    gi = gious.detach().float().contiguous()
    gc = targets["gt_box_centers_normalized"].float().contiguous()
    gl = targets["gt_box_sem_cls_label"].to(torch.int64).contiguous()
    P, Q, G = gi.shape
    C = prob.shape[-1]
    cost = torch.empty((P, Q, G), dtype=torch.float32, device=prob.device)
    w_cls, w_obj, w_center, w_giou = (float(w) for w in weights)
    _native.call("ov3d_matcher_cost", P, B, Q, G, C, int(final_last), pr, ldp, ob, ce, gi, gc, gl,
                 w_cls, w_obj,
                 w_center, w_giou, cost, like=gi)
    return cost
