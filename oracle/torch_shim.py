"""TEST INFRASTRUCTURE ONLY — CPU stand-ins with the ``ov3d_amd.pointnet2_utils``
call surface, built on the C oracle, so the product's host logic (transformer,
heads, criterion) can be checked against the reference fixtures in the CPU
test suite.  Tests inject them explicitly (monkeypatch); the product never
imports this module.
"""
import torch

from . import oracle as _o
from . import pointnet2_ref as _ref


def furthest_point_sample(xyz, npoint):
    return _ref.furthest_point_sample(xyz, npoint)


def furthest_point_sample_gather(xyz, npoint):
    idx = _ref.furthest_point_sample(xyz.detach(), npoint)
    new_xyz = torch.gather(xyz.detach(), 1, idx.long()[..., None].expand(-1, -1, 3)).contiguous()
    return idx, new_xyz


gather_operation = _ref.gather_operation
ball_query = _ref.ball_query
grouping_operation = _ref.grouping_operation
QueryAndGroup = _ref.QueryAndGroup


def generalized_box3d_iou(corners1, corners2, nums_k2, rotated_boxes=True,
                          return_inter_vols_only=False, needs_grad=False, k2_bug=True):
    mode = _o.GIOU_MODE_TENSOR if needs_grad else _o.GIOU_MODE_CYTHON
    g = _o.giou3d(corners1.detach().cpu().numpy(), corners2.detach().cpu().numpy(),
                  nums_k2.cpu().numpy(), mode=mode, rotated=rotated_boxes, k2_bug=k2_bug)
    return torch.from_numpy(g).to(corners1.device)


def install(pkg):
    """Point the product modules' kernel entry points at the CPU oracle (tests only)."""
    import importlib
    import types
    for m in ("pointnet2_modules", "model_3detr", "criterion"):
        importlib.import_module(pkg.__name__ + "." + m)
    shim = types.SimpleNamespace(
        furthest_point_sample=furthest_point_sample,
        furthest_point_sample_gather=furthest_point_sample_gather,
        gather_operation=gather_operation, ball_query=ball_query,
        grouping_operation=grouping_operation, QueryAndGroup=QueryAndGroup)
    saved = [(pkg.pointnet2_modules, "pu", pkg.pointnet2_modules.pu),
             (pkg.model_3detr, "pu", pkg.model_3detr.pu),
             (pkg.criterion, "generalized_box3d_iou", pkg.criterion.generalized_box3d_iou)]
    pkg.pointnet2_modules.pu = shim
    pkg.model_3detr.pu = shim
    pkg.criterion.generalized_box3d_iou = generalized_box3d_iou
    return saved


def uninstall(saved):
    for mod, name, val in saved:
        setattr(mod, name, val)
