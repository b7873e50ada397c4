"""Dataset configs as the hot path consumes them (mirror of reference
datasets/sunrgbd.py:54-165 and datasets/scannet.py:36-169): class / angle-bin
counts, the 640-d CLIP embedding length, angle <-> (class, residual) coding and
box-parameter -> corner conversion.  Loaders, augmentation and file paths are
out of scope."""
import numpy as np
import torch

from .box_util import (flip_axis_to_camera_np, flip_axis_to_camera_tensor, get_3d_box_batch_np,
                       get_3d_box_batch_tensor)


class _Base:
    clip_embed_length = 640
    max_num_obj = 64

    def box_parametrization_to_corners(self, box_center_unnorm, box_size, box_angle):
        return get_3d_box_batch_tensor(box_size, box_angle,
                                       flip_axis_to_camera_tensor(box_center_unnorm))

    def box_parametrization_to_corners_np(self, box_center_unnorm, box_size, box_angle):
        return get_3d_box_batch_np(box_size, box_angle, flip_axis_to_camera_np(box_center_unnorm))


class SunrgbdDatasetConfig(_Base):
    def __init__(self):
        self.num_semcls = 20
        self.num_angle_bin = 12
        self.type2class = {n: i for i, n in enumerate(
            ["bathtub", "bed", "bookshelf", "box", "chair", "counter", "desk", "door", "dresser",
             "lamp", "night_stand", "pillow", "sink", "sofa", "table", "tv", "toilet"])}
        self.class2type = {v: k for k, v in self.type2class.items()}
        self.support_class = np.arange(10, 20)

    def angle2class(self, angle):
        """continuous angle -> (bin, residual); bin centres at k*2pi/N (sunrgbd.py:102-120)"""
        n = self.num_angle_bin
        angle = angle % (2 * np.pi)
        per = 2 * np.pi / float(n)
        shifted = (angle + per / 2) % (2 * np.pi)
        cls = int(shifted / per)
        return cls, shifted - (cls * per + per / 2)

    def class2angle_batch(self, pred_cls, residual, to_label_format=True):
        per = 2 * np.pi / float(self.num_angle_bin)
        angle = pred_cls * per + residual
        if to_label_format:
            mask = angle > np.pi
            angle[mask] = angle[mask] - 2 * np.pi
        return angle


class ScannetDatasetConfig(_Base):
    def __init__(self):
        self.num_semcls = 18
        self.num_angle_bin = 1
        names = ["cabinet", "bed", "chair", "sofa", "table", "door", "window", "bookshelf",
                 "picture", "counter", "desk", "curtain", "refrigerator", "shower curtain",
                 "toilet", "sink", "bathtub", "garbagebin"]
        self.type2class = {n: i for i, n in enumerate(names)}
        self.class2type = {v: k for k, v in self.type2class.items()}

    def angle2class(self, angle):
        raise ValueError("ScanNet does not have rotated bounding boxes.")

    def class2anglebatch_tensor(self, pred_cls, residual, to_label_format=True):
        return torch.zeros(pred_cls.shape[:2], dtype=torch.float32, device=pred_cls.device)


CONFIGS = {"sunrgbd": SunrgbdDatasetConfig, "scannet": ScannetDatasetConfig}
