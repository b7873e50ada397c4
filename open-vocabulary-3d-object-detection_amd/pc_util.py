"""Point normalisation helpers on the hot path (mirror of reference
utils/pc_util.py:38-73: ``shift_scale_points``, ``scale_points``)."""
import torch


def shift_scale_points(pred_xyz, src_range, dst_range=None):
    """Map coords from [src_min, src_max] to [dst_min, dst_max] (default [0, 1]).

    pred_xyz (B,N,3) or (B,Q,K,3); src_range = [min (B,3), max (B,3)].
    Evaluated as ((x - smin) * ddiff) / sdiff + dmin, the reference's order.
    """
    smin, smax = src_range
    if dst_range is None:
        dmin = torch.zeros((smin.shape[0], 3), device=smin.device)
        dmax = torch.ones((smin.shape[0], 3), device=smin.device)
    else:
        dmin, dmax = dst_range
    if pred_xyz.ndim == 4:
        smin, smax, dmin, dmax = smin[:, None], smax[:, None], dmin[:, None], dmax[:, None]
    if smin.shape[0] != pred_xyz.shape[0] or smin.shape[-1] != pred_xyz.shape[-1]:
        raise ValueError("src_range does not match the points")
    sdiff = smax[:, None, :] - smin[:, None, :]
    ddiff = dmax[:, None, :] - dmin[:, None, :]
    return ((pred_xyz - smin[:, None, :]) * ddiff) / sdiff + dmin[:, None, :]


def scale_points(pred_xyz, mult_factor):
    if pred_xyz.ndim == 4:
        mult_factor = mult_factor[:, None]
    return pred_xyz * mult_factor[:, None, :]
