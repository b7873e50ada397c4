"""ov3d_amd — MI355X-native hot path of timsu1104/Open-vocabulary-3D-Object-Detection.

Drop-in modules (reference module -> here):
  third_party.pointnet2.pointnet2_utils   -> pointnet2_utils   (FPS, ball query, grouping on HIP)
  third_party.pointnet2.pointnet2_modules -> pointnet2_modules (PointnetSAModuleVotes)
  models (build_model, Model3DETR)        -> model_3detr, build_model
  criterion (build_criterion)             -> criterion
  utils.box_util.generalized_box3d_iou    -> box_util          (GIoU on HIP)
  utils.nms                               -> nms               (batched NMS on HIP)
  utils.dist                              -> dist              (RCCL over xGMI)
  models.model_regionclip (RegionCLIP)    -> regionclip        (ROIAlign on HIP, res5 + pool batched)
The HIP kernels live in lib/libov3d_hip.so (C ABI: include/ov3d.h); there is
no CPU fallback.
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401


def build_model(args, dataset_config, model_name=None, text_embedding=None):
    """reference models/__init__.py:10-14: "3detr" -> (Model3DETR, processor);
    "regionclip" (main.py:422) -> (RegionCLIP ROI-feature extractor, None)."""
    name = model_name or getattr(args, "model_name", "3detr")
    if name == "regionclip":
        from .regionclip import build_regionclip
        return build_regionclip(args, dataset_config)
    if name != "3detr":
        raise ValueError(f"unsupported model {name!r}")
    from .model_3detr import build_3detr
    return build_3detr(args, dataset_config, text_embedding=text_embedding)


def build_criterion(args, dataset_config):
    from .criterion import build_criterion as _b
    return _b(args, dataset_config)
