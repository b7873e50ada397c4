"""SUN RGB-D training / evaluation batches built on the device.

Drop-in for datasets/sunrgbd.py:168 ``SunrgbdDetectionDataset`` (same constructor
arguments): the raw scans are loaded once (np.load of ``{scan}_pc.npz`` /
``{scan}_bbox.npy`` as the reference does, sunrgbd.py:256-262) and kept resident in HBM;
``get_batch(indices)`` returns the collated batch dict of the reference's
``__getitem__`` (sunrgbd.py:256-462) as device tensors, built by the HIP kernels of
csrc/sunaug.hip (support-class filter, flip / rotation / scale, RandomCuboid, label
build, random_sampling, normalisations).

Random draws: the reference's numpy calls, in the reference's order, on ``rng`` (the
global ``np.random`` by default, as the reference's workers use), so the same seed gives
the reference's batch bit for bit:
  per scene   random() (flip), random() (rotation), random() (scale),
              RandomCuboid: up to 100 x [rand(3), choice(n) when check_aspect passes],
              random_sampling: choice(n_crop, num_points, replace=n_crop < num_points).
RandomCuboid's accept / reject needs the augmented points, so attempts are drawn
speculatively on the host in growing chunks (8, 32, 100), each chunk evaluated on the
device in one launch, and the generator is replayed to the state after the accepted
attempt: one device->host read per scene and chunk (with ``rngs`` = one generator per
scene: per batch and chunk).

Scope: use_color / use_height are rejected as in practice by the reference (use_color
fails in scale_points' broadcast at sunrgbd.py:407-410; use_height is never passed by
build_dataset).  use_pbox: the pseudo boxes are appended after the support-class filter of the
GT boxes, unfiltered (sunrgbd.py:266-271).  use_image: image (B, MAX_NUM_PIXEL*3) float32
zero-padded, image_height / image_width, calib_Rtilt / calib_K (sunrgbd.py:275-285, 456-461);
the images are kept resident as read (uint8 from a JPEG decoder).  use_2d_feature: feature_2d
(sunrgbd.py:272-273, 454-455).
"""
import os

import numpy as np
import torch

from . import _native as nat

MAX_ATTEMPTS = 100   # random_cuboid.py:43
MAX_NUM_PIXEL = 530 * 730   # sunrgbd.py:47
RAW_DATA_PATH = "/share/suzhengyuan/code/ScanRefer-3DVG/votenet/sunrgbd/sunrgbd_trainval"  # :42


def read_image_cv2(path):
    """the reference's image read (sunrgbd.py:281: np.array(cv2.imread(path)), BGR uint8)"""
    try:
        import cv2
    except ImportError as e:   # not in this image; pass image_reader= to the dataset
        raise ImportError("use_image needs cv2 (absent here): pass image_reader=") from e
    return np.array(cv2.imread(path))


def read_calib(path):
    """sunrgbd.py:277-279: two lines of 9 floats, column-major 3x3 (Rtilt, K)"""
    with open(path) as f:
        lines = f.readlines()
    rt = np.reshape(np.array([float(x) for x in lines[0].rstrip().split(" ")]), (3, 3), "F")
    k = np.reshape(np.array([float(x) for x in lines[1].rstrip().split(" ")]), (3, 3), "F")
    return rt, k


class SceneStore:
    """Raw scans resident in device memory: points (S, n_max, 3) of the scans' dtype and
    boxes (S, k_max, 8) float64, with per-scan counts."""

    def __init__(self, scans, device, extras=None):
        pcs, boxes = [s[0] for s in scans], [s[1] for s in scans]
        # boxes past the first ngt are use_pbox pseudo boxes (never support-filtered)
        self.ngt = np.array([s[2] if len(s) > 2 else s[1].shape[0] for s in scans], np.int32)
        dt = pcs[0].dtype
        if any(p.dtype != dt for p in pcs) or dt not in (np.float32, np.float64):
            raise TypeError("scans must share one float32 / float64 point dtype")
        self.pc_f64 = int(dt == np.float64)
        self.n = np.array([p.shape[0] for p in pcs], np.int32)
        self.k = np.array([b.shape[0] for b in boxes], np.int32)
        self.n_max = int(self.n.max())
        self.k_max = max(int(self.k.max()), 1)
        S = len(pcs)
        pts = np.zeros((S, self.n_max, 3), dt)
        bx = np.zeros((S, self.k_max, 8), np.float64)
        for i, (p, b) in enumerate(zip(pcs, boxes)):
            pts[i, : p.shape[0]] = p[:, 0:3]
            bx[i, : b.shape[0]] = b
        self.device = torch.device(device)
        self.points = torch.as_tensor(pts).to(self.device)
        self.boxes = torch.as_tensor(bx).to(self.device)
        self.n_dev = torch.as_tensor(self.n).to(self.device)
        self.k_dev = torch.as_tensor(self.k).to(self.device)
        self.ngt_dev = torch.as_tensor(self.ngt).to(self.device)
        self.extras = {}
        if extras:
            self._stack_extras(extras)

    def _stack_extras(self, extras):
        """per-scan dicts of image (H, W, 3) / calib_Rtilt / calib_K / feature_2d ->
        resident tensors: images flattened and zero-padded to MAX_NUM_PIXEL * 3 in their
        read dtype (the float32 conversion happens per batch, exactly as full_img_1d's).

        Memory: S x MAX_NUM_PIXEL x 3 elements on the device (1.16 MB per uint8 image: the
        5285 SUN v1 training scans are 6.1 GB of the 288 GB HBM).  Each image is copied
        straight into its row of the preallocated device tensor, so the host never holds
        more than one padded image beside the decoded ones."""
        dev = self.device
        if "image" in extras[0]:
            imgs = [np.asarray(e["image"]) for e in extras]
            dt = imgs[0].dtype if all(i.dtype == imgs[0].dtype for i in imgs) else np.float32
            flat = torch.zeros((len(imgs), MAX_NUM_PIXEL * 3), dtype=torch.from_numpy(
                np.zeros(0, dt)).dtype, device=dev)
            for i, im in enumerate(imgs):
                if im.size > MAX_NUM_PIXEL * 3:
                    raise ValueError("image larger than MAX_NUM_PIXEL (sunrgbd.py:284-285)")
                flat[i, : im.size].copy_(torch.from_numpy(
                    np.ascontiguousarray(im.reshape(-1), dtype=dt)))
            self.extras["image"] = flat
            self.extras["image_height"] = torch.as_tensor(np.array([i.shape[0] for i in imgs], np.int64)).to(dev)
            self.extras["image_width"] = torch.as_tensor(np.array([i.shape[1] for i in imgs], np.int64)).to(dev)
            for k in ("calib_Rtilt", "calib_K"):
                self.extras[k] = torch.as_tensor(np.stack([np.asarray(e[k], np.float64)
                                                           for e in extras])).to(dev)
        if "feature_2d" in extras[0]:
            self.extras["feature_2d"] = torch.as_tensor(np.stack([e["feature_2d"] for e in extras])).to(dev)


class SunrgbdDetectionDataset:
    """datasets/sunrgbd.py:168-254 constructor; scans resident on `device`.

    `scans` (list of (pc, bboxes) arrays) replaces reading ``root_dir`` (synthetic data,
    tests).  Batches: ``get_batch(indices, rng=np.random)``."""

    def __init__(self, dataset_config, split_set="train", root_dir=None, meta_data_dir=None,
                 pseudo_box_dir=None, feature_2d_dir=None, num_points=20000, use_color=False,
                 use_image=False, use_height=False, use_v1=True, augment=False,
                 use_random_cuboid=True, random_cuboid_min_points=30000, use_pbox=False,
                 use_2d_feature=False, device="cuda", scans=None, extras=None,
                 raw_data_path=RAW_DATA_PATH, image_reader=read_image_cv2):
        assert num_points <= 50000
        assert split_set in ["train", "val", "trainval"]
        if use_color:
            raise NotImplementedError("use_color: the reference fails in scale_points "
                                      "(sunrgbd.py:407-410, (64,3) x (1,6) broadcast)")
        if use_height:
            raise NotImplementedError("use_height is never enabled by build_dataset")
        self.dataset_config = dataset_config
        self.num_points = num_points
        self.augment = augment
        self.use_image = use_image
        self.use_random_cuboid = use_random_cuboid
        self.min_points = random_cuboid_min_points
        self.aspect, self.min_crop, self.max_crop = 0.75, 0.75, 1.0   # sunrgbd.py:234-239
        self.max_num_obj = 64
        self.train = split_set == "train"
        self.use_2d_feature = use_2d_feature
        if scans is None:
            scans, self.scan_names = self._read(root_dir, split_set, use_pbox, pseudo_box_dir)
            if use_image or use_2d_feature:
                extras = [self._read_extras(n, use_image, use_2d_feature, raw_data_path,
                                            feature_2d_dir, image_reader) for n in self.scan_names]
        else:
            self.scan_names = [f"{i:06d}" for i in range(len(scans))]
        if (use_image or use_2d_feature) and not extras:
            raise ValueError("use_image / use_2d_feature: no images / features (extras=)")
        self.store = SceneStore(scans, device, extras)
        sup = np.asarray(dataset_config.support_class, np.float64) if self.train else np.zeros(0)
        self._support = torch.as_tensor(sup).to(self.store.device)

    @staticmethod
    def _read(root_dir, split_set, use_pbox, pseudo_box_dir):
        """the reference's file reads (sunrgbd.py:205-229, 256-267); allow_pickle stays off"""
        subs = ["train", "val"] if split_set == "trainval" else [split_set]
        paths = []
        for sub in subs:
            d = root_dir + "_%s" % sub
            paths += [os.path.join(d, x) for x in
                      sorted(set(os.path.basename(f)[0:6] for f in os.listdir(d)))]
        paths.sort()
        scans = []
        for p in paths:
            pc = np.load(p + "_pc.npz")["pc"]
            bb = np.load(p + "_bbox.npy")
            ngt = bb.shape[0]
            if use_pbox:
                bb = np.concatenate([bb, np.load(os.path.join(pseudo_box_dir, os.path.basename(p))
                                                 + "_bbox.npy")], 0)
            scans.append((pc[:, 0:3], bb, ngt))
        return scans, [os.path.basename(p) for p in paths]

    @staticmethod
    def _read_extras(name, use_image, use_2d_feature, raw_data_path, feature_2d_dir, reader):
        """sunrgbd.py:272-285 for one scan"""
        e = {}
        if use_2d_feature:
            e["feature_2d"] = np.load(os.path.join(feature_2d_dir, name) + ".npy")
        if use_image:
            e["calib_Rtilt"], e["calib_K"] = read_calib(os.path.join(raw_data_path, "calib", name + ".txt"))
            e["image"] = reader(os.path.join(raw_data_path, "image", name + ".jpg"))
        return e

    def __len__(self):
        return len(self.scan_names)

    # ---- the random plan (host, reference order) ----
    def _draw_aug(self, rng):
        flip = rng.random() > 0.5
        rot_angle = (rng.random() * np.pi / 3) - np.pi / 6
        scale = rng.random() * 0.3 + 0.85
        return [float(flip), rot_angle, float(np.cos(rot_angle)), float(np.sin(rot_angle)),
                scale, 0.0, 0.0, 0.0]

    def _draw_attempts(self, rng, n, att, t0, t1):
        """attempts t0..t1-1 of RandomCuboid's loop into att (rows of [crop xyz, centre]);
        the draws are the reference's: rand(3), then choice(n) (== randint(0, n)) only
        when check_aspect passes (random_cuboid.py:45-53)"""
        amin, lo, span = self.aspect, self.min_crop, self.max_crop - self.min_crop
        for t in range(t0, t1):
            crop = lo + rng.rand(3) * span
            c0, c1, c2 = float(crop[0]), float(crop[1]), float(crop[2])
            att[t, :3] = crop
            if (min(c0, c1) / max(c0, c1) >= amin or min(c0, c2) / max(c0, c2) >= amin
                    or min(c1, c2) / max(c1, c2) >= amin):
                att[t, 3] = rng.randint(0, n)
            else:
                att[t, 3] = -1.0

    def _replay_attempts(self, rng, n, upto):
        """advance rng exactly over attempts 0..upto (the accepted one included)"""
        scratch = np.empty((upto + 1, 4))
        self._draw_attempts(rng, n, scratch, 0, upto + 1)

    def get_batch(self, indices, rng=None, rngs=None):
        """Collated reference batch for scans `indices` (device tensors).

        rng: one numpy RandomState-like generator drawn scene after scene (the reference's
        per-worker np.random); rngs: one generator per scene instead (one sync per batch)."""
        st = self.store
        dev = st.device
        B = len(indices)
        if rngs is None:
            rngs = [rng if rng is not None else np.random] * B
            shared = True
        else:
            shared = False
            assert len(rngs) == B
        idx = torch.as_tensor(np.asarray(indices, np.int32)).to(dev)
        npts = st.n_dev[idx.long()].contiguous()
        nbox = st.k_dev[idx.long()].contiguous()
        ngt = st.ngt_dev[idx.long()].contiguous()
        n_host = st.n[np.asarray(indices)]
        T = torch.float64 if st.pc_f64 else torch.float32
        nparts = nat.load().ov3d_sun_range_parts(st.n_max)
        pts = torch.empty((B, st.n_max, 3), dtype=T, device=dev)
        rpart = torch.empty((B, nparts, 6), dtype=T, device=dev)
        boxes = torch.zeros((B, st.k_max, 8), dtype=torch.float64, device=dev)
        nbox_aug = torch.empty(B, dtype=torch.int32, device=dev)
        A = MAX_ATTEMPTS
        cuboid = self.augment and self.use_random_cuboid
        counts = torch.empty((B, A), dtype=torch.int32, device=dev)
        accept = torch.empty((B, A), dtype=torch.int32, device=dev)
        crop_mm = torch.empty((B, A, 6), dtype=T, device=dev)
        sel = torch.empty((B, 2), dtype=torch.int32, device=dev)
        params = np.zeros((B, 8))
        attempts = np.full((B, A, 4), -1.0)     # undrawn rows: centre -1 (never accepted)
        choices = np.zeros((B, self.num_points), np.int64)

        def launch_aug(lo, hi):
            p = torch.as_tensor(params[lo:hi]).to(dev)
            nat.call("ov3d_sun_aug_points", st.points, st.pc_f64, st.n_max, 3, idx[lo:hi],
                     npts[lo:hi], hi - lo, st.n_max, p, int(self.augment), pts[lo:hi],
                     rpart[lo:hi], like=pts)
            nat.call("ov3d_sun_aug_boxes", st.boxes, st.k_max, idx[lo:hi], nbox[lo:hi],
                     ngt[lo:hi], hi - lo, st.k_max, p, int(self.augment), self._support,
                     int(self._support.numel()), boxes[lo:hi], nbox_aug[lo:hi], like=pts)
            return p

        def launch_cuboid(lo, hi):
            att = torch.as_tensor(attempts[lo:hi]).to(dev)
            nat.call("ov3d_sun_cuboid_eval", pts[lo:hi], st.pc_f64, st.n_max, npts[lo:hi],
                     rpart[lo:hi], att, hi - lo, A, self.min_points, boxes[lo:hi], nbox_aug[lo:hi],
                     st.k_max, counts[lo:hi], crop_mm[lo:hi], accept[lo:hi], sel[lo:hi], like=pts)
            return att, sel[lo:hi].cpu().numpy()

        def run_cuboid(lo, hi):
            """RandomCuboid for scenes lo..hi-1: attempts are drawn in growing chunks (most
            scans accept one of the first few) and evaluated on the device; a scene whose
            drawn attempts all fail draws the next chunk from where its generator stands.
            Returns the device attempts and sel (t*, n_crop) with every rng positioned
            after the accepted attempt (or after all 100: the fallback)."""
            drawn = np.zeros(hi - lo, np.int64)
            done = np.zeros(hi - lo, bool)
            s_all = np.zeros((hi - lo, 2), np.int32)
            chunk = 8
            while True:
                for b in range(lo, hi):
                    if not done[b - lo]:
                        t0 = int(drawn[b - lo])
                        t1 = min(A, t0 + chunk)
                        self._draw_attempts(rngs[b], int(n_host[b]), attempts[b], t0, t1)
                        drawn[b - lo] = t1
                att, s = launch_cuboid(lo, hi)
                for b in range(lo, hi):
                    if done[b - lo]:
                        continue
                    if s[b - lo, 0] >= 0:
                        rngs[b].set_state(state0[b])
                        self._replay_attempts(rngs[b], int(n_host[b]), int(s[b - lo, 0]))
                        done[b - lo] = True
                    elif drawn[b - lo] >= A:
                        done[b - lo] = True
                    s_all[b - lo] = s[b - lo]
                if done.all():
                    return att, s_all
                chunk = min(A, chunk * 4)

        state0 = [None] * B
        att_dev = []
        spans = [(b, b + 1) for b in range(B)] if shared else [(0, B)]
        for lo, hi in spans:
            for b in range(lo, hi):
                r = rngs[b]
                if self.augment:
                    params[b] = self._draw_aug(r)
                    if cuboid:
                        state0[b] = r.get_state()
            launch_aug(lo, hi)
            if cuboid:
                a, s = run_cuboid(lo, hi)
                att_dev.append(a)
            else:
                s = np.zeros((hi - lo, 2), np.int32)
            for b in range(lo, hi):
                n_crop = int(s[b - lo, 1]) if cuboid else int(n_host[b])
                choices[b] = rngs[b].choice(n_crop, self.num_points,
                                            replace=n_crop < self.num_points)
        att_all = (torch.cat(att_dev) if att_dev else
                   torch.full((B, A, 4), -1.0, dtype=torch.float64, device=dev))
        if not cuboid:
            sel.copy_(torch.stack([torch.full_like(npts, -1), npts], 1))
        ch = torch.as_tensor(choices).to(dev)
        N = self.num_points
        crop_idx = torch.empty((B, st.n_max), dtype=torch.int32, device=dev)
        out_pc = torch.empty((B, N, 3), dtype=torch.float32, device=dev)
        nd = nat.load().ov3d_sun_range_parts(N)
        dpart = torch.empty((B, nd, 6), dtype=T, device=dev)
        nat.call("ov3d_sun_crop_sample", pts, st.pc_f64, st.n_max, npts, rpart, att_all, B, A, sel,
                 ch, N, crop_idx, out_pc, dpart, like=pts)
        G = self.max_num_obj
        f32 = dict(dtype=torch.float32, device=dev)
        out = {
            "point_clouds": out_pc,
            "gt_box_corners": torch.empty((B, G, 8, 3), **f32),
            "gt_box_centers": torch.empty((B, G, 3), **f32),
            "gt_box_centers_normalized": torch.empty((B, G, 3), **f32),
            "gt_box_sem_cls_label": torch.empty((B, G), dtype=torch.int64, device=dev),
            "gt_box_present": torch.empty((B, G), **f32),
            "scan_idx": idx.long(),
            "gt_box_sizes": torch.empty((B, G, 3), **f32),
            "gt_box_sizes_normalized": torch.empty((B, G, 3), **f32),
            "gt_box_angles": torch.empty((B, G), **f32),
            "gt_angle_class_label": torch.empty((B, G), dtype=torch.int64, device=dev),
            "gt_angle_residual_label": torch.empty((B, G), **f32),
            "point_cloud_dims_min": torch.empty((B, 3), dtype=T, device=dev),
            "point_cloud_dims_max": torch.empty((B, 3), dtype=T, device=dev),
        }
        args = nat.SunLabelsArgs(
            B=B, max_num_obj=G, k_max=st.k_max, num_angle_bin=self.dataset_config.num_angle_bin,
            num_attempts=A, n_dims_part=nd, boxes=boxes.data_ptr(), nbox=nbox_aug.data_ptr(),
            sel=sel.data_ptr() if cuboid else None, crop_mm=crop_mm.data_ptr(),
            dims_part=dpart.data_ptr(), dims_min=out["point_cloud_dims_min"].data_ptr(),
            dims_max=out["point_cloud_dims_max"].data_ptr(),
            corners=out["gt_box_corners"].data_ptr(), centers=out["gt_box_centers"].data_ptr(),
            centers_normalized=out["gt_box_centers_normalized"].data_ptr(),
            sem_cls=out["gt_box_sem_cls_label"].data_ptr(), present=out["gt_box_present"].data_ptr(),
            sizes=out["gt_box_sizes"].data_ptr(), sizes_normalized=out["gt_box_sizes_normalized"].data_ptr(),
            angles=out["gt_box_angles"].data_ptr(), angle_cls=out["gt_angle_class_label"].data_ptr(),
            angle_res=out["gt_angle_residual_label"].data_ptr())
        nat.call("ov3d_sun_labels", nat.byref(args), st.pc_f64, like=pts)
        li = idx.long()
        for k, v in st.extras.items():
            out[k] = v[li].float() if k == "image" else v[li]
        return out

    def __getitem__(self, idx):
        """one scene through the device path, as the reference's numpy dict"""
        return {k: v[0].cpu().numpy() for k, v in self.get_batch([idx]).items()}
