"""ctypes binding of ``lib/libov3d_hip.so`` (the C ABI declared in include/ov3d.h).

This is the only door from Python to the hot-path kernels.  There is no CPU
fallback: if the library is missing, or a tensor is not on a ROCm device, the
call raises.  Pointers are ``tensor.data_ptr()``; the stream is torch's current
HIP stream on the tensor's device, so every op is stream-ordered with the
surrounding torch work and capturable into a hipGraph.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libov3d_hip.so")

OV3D_GIOU_CYTHON = 0
OV3D_GIOU_TENSOR = 1

_lib = None

# name -> argtypes ("p" pointer, "i" int, "l" long long, "f" float, "d" double)
_SIGS = {
    "ov3d_fps": "piiipppp",
    "ov3d_fps_pair_status": "piiipp",
    "ov3d_ball_query": "ppiiifipp",
    "ov3d_ball_query_cells": "ppiiifipplp",
    "ov3d_group_fwd": "ppplllpiiiiifipp",
    "ov3d_group_bwd": "ppiiiiilllpp",
    "ov3d_gather_fwd": "ppiiiipp",
    "ov3d_gather_bwd": "ppiiiipp",
    "ov3d_giou3d": "pppiiiiipipp",
    "ov3d_giou3d_bwd_aligned": "pppiiippp",
    "ov3d_giou3d_bwd": "pppiiiipppp",
    "ov3d_hungarian": "ppiiipppp",
    "ov3d_sa_l1_fwd": "ppiippip",
    "ov3d_sa_l1_fwd_cin": "pipiippip",
    "ov3d_sa_layer_fwd": "ppppiiipppip",
    "ov3d_sa_layer_fwd_x0": "pppppiiippip",
    "ov3d_sa_layer_pool_fwd": "ppppiiiipppppppip",
    "ov3d_sa_layer_dy": "ppppiiiippppppip",
    "ov3d_reduce_partials": "piipp",
    "ov3d_reduce_partials_f32": "piipp",
    "ov3d_colsum_f32": "piipp",
    "ov3d_bn_finalize": "pdippffpppppppp",
    "ov3d_sa_pool_fwd": "ppppppiiipppp",
    "ov3d_sa_pool_bwd": "ppppppiiippip",
    "ov3d_bn_bwd_finalize": "pdippppppppp",
    "ov3d_bn_relu_bwd": "ippppppppppiippipp",
    "ov3d_bn_relu_bwd_cin": "ippppppppppiiippipp",
    "ov3d_nms3d": "ppiiidiipp",
    "ov3d_nms_boxes_from_corners": "pppiipp",
    "ov3d_clip_preprocess": "plppiiifffffffipp",
    "ov3d_roi_align_fwd": "piiiiipiiifiiipp",
    "ov3d_roi_align_pool2_fwd": "piiiiipiiifiiippp",
    "ov3d_im2col3x3": "piiiiiiipp",
    "ov3d_bias_residual_act": "pilippip",
    "ov3d_avgpool2_nhwc": "piiiiipp",
    "ov3d_attnpool_tokens": "piiiippp",
    "ov3d_attnpool_mean": "piiippp",
    "ov3d_attnpool_fused": "pppplliiiipp",
    "ov3d_attn_fwd": "pppllliiiiffpiplpppip",
    "ov3d_attn_bwd": "ppplllplplpiiiiffppplplplpip",
    "ov3d_attn_bwd_dkdv_batch": "piiiiiffp",
    "ov3d_attn_fwd_masked": "pppllliiiiffpiplpppipp",
    "ov3d_attn_fwd_pregen": "pppllliiiiffpiplpppipp",
    "ov3d_attn_dropgen": "iiiifpipp",
    "ov3d_attn_bwd_masked": "ppplllplplpiiiiffppplplplpipp",
    "ov3d_attn_mask_pack": "pifiiipp",
    "ov3d_nbr_max_fwd": "pliippp",
    "ov3d_set_loss_fwd_split": "ppppppp",
    "ov3d_group_inverse": "piiiippppp",
    "ov3d_group_bwd_csr": "pppiiilllpp",
    "ov3d_group_bwd_csr_bf16": "plppiiilllpp",
    "ov3d_group_rows_bf16": "ppplllpiiiiifiipp",
    "ov3d_nbr_max_bwd": "ppliipp",
    "ov3d_nbr_max_bnrelu_fwd": "pliippppp",
    "ov3d_rows_bn_bwd_pooled": "ippiplippppppppipp",
    "ov3d_wgrad": "plpliiiplpppip",
    "ov3d_wgrad_bn": "plpliiippplpppip",
    "ov3d_wgrad_group": "pipp",
    "ov3d_rows_bn_stats": "pillilipip",
    "ov3d_rows_bn_apply": "pillilippfpipllip",
    "ov3d_rows_bn_bwd": "ipllipillilipppppppfpipipllip",
    "ov3d_set_loss_fwd": "pppppp",
    "ov3d_matcher_cost": "iiiiiiplpppppffffpp",
    "ov3d_targets_prep": "iiipppppppp",
    "ov3d_set_loss_bwd": "pppppppppppp",
    "ov3d_adamw_step": "pppipfpddfpifpp",
    "ov3d_adamw_set_grads": "pipp",
    "ov3d_multi_copy": "ipppp",
    "ov3d_add_cast_bf16": "piplppp",
    "ov3d_seed_next": "ppp",
    "ov3d_fourier_pe": "piipppiiipp",
    "ov3d_box_param_fwd": "liiiiplpppppppppppppppp",
    "ov3d_box_param_bwd": "liiiplppppppppppppplp",
    "ov3d_relu_dropout_fwd": "plifpipp",
    "ov3d_relu_dropout_bwd": "pplfpp",
    "ov3d_resnorm_fwd": "lipipifpipppippfppppppilllp",
    "ov3d_resnorm_bwd": "lipppppppilllppfpippipipippppip",
    "ov3d_rows_gemm": "iiiplplipplp",
    "ov3d_bn_stats_finalize": "piidppffpppppppp",
    "ov3d_colsum_group": "pipiip",
    "ov3d_sa_dy_fused": "ppppiiiipppppppppppip",
    "ov3d_sa_dy2_fused": "pppppppppppppppiiipppip",
    "ov3d_bn_bwd_stats_finalize": "piidppppppppp",
    "ov3d_rows_gemm_act": "iiiplplipifpiplplp",
    "ov3d_rows_gemm_group": "iipip",
    "ov3d_tile_gemm": "iiiplplipplp",
    "ov3d_tile_gemm_act": "iiiplplipifpiplplp",
    "ov3d_tile_gemm2": "iiiplpliplpliplp",
    "ov3d_tile_gemm_batched": "iiiipllpllipllp",
    "ov3d_sun_aug_points": "pilippiipippp",
    "ov3d_sun_aug_boxes": "plpppiipipippp",
    "ov3d_sun_cuboid_eval": "piipppiiippippppp",
    "ov3d_sun_crop_sample": "piipppiippipppp",
    "ov3d_sun_labels": "pip",
    "ov3d_box_points_count": "pllipiipp",
    "ov3d_box3d_iou_eval": "ppppiiipp",
    "ov3d_ap_match": "ppppiiiidpp",
    "ov3d_ap_curve": "plppiplppp",
    "ov3d_project_box2d": "pppliipppppp",
    "ov3d_heads_out_fwd": "plippipiippippppppipp",
    "ov3d_heads_out_bwd": "pppiiiipiippppppplp",
    "ov3d_gemm256": "plplpiplpliiiip",
    "ov3d_conv3x3_gemm256": "piiiiplpiplpliip",
    "ov3d_gemm256_pair": "pplpplppippliiip",
    "ov3d_gemm256_batched": "pllpllpliplliiiiip",
    "ov3d_lngemm_fwd": "ipipfpipppippfppppppilllipifpip",
    "ov3d_rows256": "pliiplpllpp",
    "ov3d_rows256_bn": "plppplplpllpp",
    "ov3d_lngemm_bwd": "ipppppppilllppfpipppipipliifplplp",
}
EXPORTS = tuple(_SIGS) + ("ov3d_version", "ov3d_sa_layer_supported", "ov3d_attn_fwd_workspace",
                          "ov3d_attn_dropbits_words", "ov3d_attn_maskbits_words", "ov3d_fps_workspace", "ov3d_attn_small_bwd", "ov3d_set_loss_fwd_parts",
                          "ov3d_wgrad_workspace", "ov3d_wgrad_tiles", "ov3d_wgrad_group_tiles",
                          "ov3d_set_loss_desc_size",
                          "ov3d_resnorm_supported", "ov3d_resnorm_bwd_parts",
                          "ov3d_adamw_chunk", "ov3d_wgrad_group_workspace",
                          "ov3d_rows_gemm_supported", "ov3d_sa_dy_fused_supported",
                          "ov3d_tile_gemm_supported", "ov3d_sun_range_parts", "ov3d_heads_out_max_text",
                          "ov3d_heads_out_workspace", "ov3d_stamps_arm", "ov3d_stamps_count",
                          "ov3d_stamps_get", "ov3d_wall_clock_khz",
                          "ov3d_attnpool_fused_supported", "ov3d_lngemm_supported",
                          "ov3d_lngemm_bwd_parts", "ov3d_lngemm_stamps_arm", "ov3d_stream_create",
                          "ov3d_ball_query_ws_bytes", "ov3d_rows256_supported")

_CT = {"p": ctypes.c_void_p, "i": ctypes.c_int, "l": ctypes.c_longlong, "f": ctypes.c_float,
       "d": ctypes.c_double}


class NativeError(RuntimeError):
    pass


def load():
    """Load libov3d_hip.so (raises if it was not built: run __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"{LIB_PATH} not found: the HIP extension is required (no CPU fallback); "
                "build it with `make -C open-vocabulary-3d-object-detection_amd/csrc`")
        lib = ctypes.CDLL(LIB_PATH)
        for name, sig in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = [_CT[c] for c in sig]
            fn.restype = ctypes.c_int
        lib.ov3d_sa_layer_supported.argtypes = [ctypes.c_int, ctypes.c_int]
        lib.ov3d_sa_layer_supported.restype = ctypes.c_int
        lib.ov3d_attn_fwd_workspace.argtypes = [ctypes.c_int] * 5
        lib.ov3d_attn_fwd_workspace.restype = ctypes.c_longlong
        lib.ov3d_attn_dropbits_words.argtypes = [ctypes.c_int] * 4
        lib.ov3d_attn_dropbits_words.restype = ctypes.c_longlong
        lib.ov3d_set_loss_fwd_parts.argtypes = [ctypes.c_int] * 3
        lib.ov3d_set_loss_fwd_parts.restype = ctypes.c_longlong
        lib.ov3d_fps_workspace.argtypes = [ctypes.c_int] * 2
        lib.ov3d_fps_workspace.restype = ctypes.c_longlong
        lib.ov3d_stamps_arm.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong]
        lib.ov3d_stamps_arm.restype = ctypes.c_int
        lib.ov3d_stamps_count.argtypes = []
        lib.ov3d_stamps_count.restype = ctypes.c_int
        lib.ov3d_stamps_get.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4
        lib.ov3d_stamps_get.restype = ctypes.c_int
        lib.ov3d_wall_clock_khz.argtypes = []
        lib.ov3d_wall_clock_khz.restype = ctypes.c_longlong
        lib.ov3d_attn_small_bwd.argtypes = [ctypes.c_int]
        lib.ov3d_attn_small_bwd.restype = ctypes.c_int
        lib.ov3d_attn_maskbits_words.argtypes = [ctypes.c_int] * 3
        lib.ov3d_attn_maskbits_words.restype = ctypes.c_longlong
        lib.ov3d_wgrad_workspace.argtypes = [ctypes.c_int] * 4
        lib.ov3d_wgrad_workspace.restype = ctypes.c_longlong
        lib.ov3d_wgrad_tiles.argtypes = [ctypes.c_int] * 2
        lib.ov3d_wgrad_tiles.restype = ctypes.c_int
        lib.ov3d_wgrad_group_tiles.argtypes = [ctypes.c_int] * 2
        lib.ov3d_wgrad_group_tiles.restype = ctypes.c_int
        lib.ov3d_set_loss_desc_size.argtypes = []
        lib.ov3d_set_loss_desc_size.restype = ctypes.c_longlong
        lib.ov3d_resnorm_supported.argtypes = [ctypes.c_int]
        lib.ov3d_resnorm_supported.restype = ctypes.c_int
        lib.ov3d_resnorm_bwd_parts.argtypes = [ctypes.c_longlong, ctypes.c_int]
        lib.ov3d_resnorm_bwd_parts.restype = ctypes.c_int
        lib.ov3d_adamw_chunk.argtypes = []
        lib.ov3d_adamw_chunk.restype = ctypes.c_int
        lib.ov3d_wgrad_group_workspace.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.ov3d_wgrad_group_workspace.restype = ctypes.c_longlong
        lib.ov3d_sa_dy_fused_supported.argtypes = [ctypes.c_int] * 2
        lib.ov3d_sa_dy_fused_supported.restype = ctypes.c_int
        lib.ov3d_rows_gemm_supported.argtypes = [ctypes.c_int] * 3
        lib.ov3d_rows256_supported.argtypes = [ctypes.c_longlong, ctypes.c_int, ctypes.c_int]
        lib.ov3d_rows256_supported.restype = ctypes.c_int
        lib.ov3d_rows_gemm_supported.restype = ctypes.c_int
        lib.ov3d_tile_gemm_supported.argtypes = [ctypes.c_int] * 3
        lib.ov3d_tile_gemm_supported.restype = ctypes.c_int
        lib.ov3d_sun_range_parts.argtypes = [ctypes.c_int]
        lib.ov3d_sun_range_parts.restype = ctypes.c_int
        lib.ov3d_heads_out_max_text.argtypes = []
        lib.ov3d_heads_out_max_text.restype = ctypes.c_int
        lib.ov3d_attnpool_fused_supported.argtypes = [ctypes.c_int] * 3
        lib.ov3d_attnpool_fused_supported.restype = ctypes.c_int
        lib.ov3d_lngemm_supported.argtypes = [ctypes.c_int] * 3
        lib.ov3d_lngemm_supported.restype = ctypes.c_int
        lib.ov3d_lngemm_bwd_parts.argtypes = [ctypes.c_int]
        lib.ov3d_lngemm_bwd_parts.restype = ctypes.c_int
        lib.ov3d_lngemm_stamps_arm.argtypes = [ctypes.c_void_p]
        lib.ov3d_lngemm_stamps_arm.restype = ctypes.c_int
        lib.ov3d_heads_out_workspace.argtypes = [ctypes.c_int] * 2
        lib.ov3d_heads_out_workspace.restype = ctypes.c_longlong
        lib.ov3d_stream_create.argtypes = [ctypes.c_void_p]
        lib.ov3d_ball_query_ws_bytes.argtypes = [ctypes.c_int] * 2
        lib.ov3d_ball_query_ws_bytes.restype = ctypes.c_longlong
        lib.ov3d_stream_create.restype = ctypes.c_int
        lib.ov3d_version.argtypes = []
        lib.ov3d_version.restype = ctypes.c_char_p
        _lib = lib
    return _lib


def version():
    return load().ov3d_version().decode()


def stream_create(device):
    """-> torch.cuda.ExternalStream over a new HIP stream of the caller's own (ov3d_stream_create):
    unlike torch.cuda.Stream() it never comes from (or returns to) PyTorch's recycled pool.  The
    stream lives for the process."""
    with torch.cuda.device(device):
        h = ctypes.c_void_p()
        rc = load().ov3d_stream_create(ctypes.byref(h))
        if rc != 0 or not h.value:
            raise NativeError(f"ov3d_stream_create failed with status {rc}")
        return torch.cuda.ExternalStream(h.value, device=device)


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def check_device(t, name):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if t.device.type != "cuda":
        raise NativeError(f"{name}: ov3d kernels run on the ROCm device only (got {t.device})")
    return t


def check(t, name, dtype=None, ndim=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if t.device.type != "cuda":
        raise NativeError(f"{name}: ov3d kernels run on the ROCm device only (got {t.device})")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim}-d tensor, got shape {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    return t


# Optional per-launch timing (bench.py): HIP events recorded on the launch stream.
_TIMING = {}


def timing_enable(names):
    _TIMING.clear()
    for n in names:
        _TIMING[n] = []


def timing_collect():
    """-> {name: [{"ms": float, "shape": (int args...)}]}; synchronises the events."""
    out = {}
    for n, recs in _TIMING.items():
        out[n] = []
        for ev0, ev1, shape in recs:
            ev1.synchronize()
            out[n].append({"ms": ev0.elapsed_time(ev1), "shape": shape})
    _TIMING.clear()
    return out


# Optional launch census (tests): the set of entry points called while enabled.
_CALLED = None


STAMP_KINDS = ("fwd", "dq", "dkdv", "gemm256")


def stamps_arm(buf, min_work=1 << 20):
    """arm the attention kernels' in-kernel launch stamps into the int64 device tensor buf (None
    disarms; the launch table stays readable).  Launches captured into a graph while armed keep
    stamping on every replay."""
    lib = load()
    if buf is None:
        lib.ov3d_stamps_arm(None, 0, 0)
    else:
        lib.ov3d_stamps_arm(buf.data_ptr(), buf.numel(), int(min_work))


def stamps_read(buf):
    """-> [(kind, launch duration ms, Lq * Lk)] for every recorded launch whose slots hold
    stamps: max(exit) - min(entry) over its waves (wall clock, ov3d_wall_clock_khz)."""
    lib = load()
    khz = lib.ov3d_wall_clock_khz()
    host = buf.cpu()
    out = []
    for i in range(lib.ov3d_stamps_count()):
        kind, off, waves, work = ctypes.c_int(), ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_longlong()
        lib.ov3d_stamps_get(i, ctypes.byref(kind), ctypes.byref(off), ctypes.byref(waves), ctypes.byref(work))
        st = host[off.value: off.value + 2 * waves.value].view(-1, 2)
        if bool((st == 0).any()):
            continue
        out.append((STAMP_KINDS[kind.value], (st[:, 1].max() - st[:, 0].min()).item() / khz, work.value))
    return out


def census_start():
    global _CALLED
    _CALLED = {}


def census_stop():
    """-> {entry point: number of calls} since census_start()"""
    global _CALLED
    out, _CALLED = _CALLED or {}, None
    return out


def note(name):
    """count a launch made without call() (census)"""
    if _CALLED is not None:
        _CALLED[name] = _CALLED.get(name, 0) + 1


def call(name, *args, like):
    """Invoke `name` with args (+ the current stream of `like`); raise on nonzero status."""
    fn = getattr(load(), name)
    note(name)
    conv = []
    for a in args:
        if isinstance(a, torch.Tensor) or a is None:
            conv.append(_ptr(a))
        else:
            conv.append(a)
    rec = _TIMING.get(name)
    if rec is not None:
        stream = torch.cuda.current_stream(like.device)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
    rc = fn(*conv, _stream(like))
    if rec is not None:
        ev1.record(stream)
        rec.append((ev0, ev1, tuple(a for a in args if isinstance(a, int))[:3]))
    if rc != 0:
        raise NativeError(f"{name} failed with status {rc}")


class SunLabelsArgs(ctypes.Structure):
    """ov3d_sun_labels_args (include/ov3d.h)"""
    _fields_ = [(n, ctypes.c_int) for n in ("B", "max_num_obj", "k_max", "num_angle_bin",
                                             "num_attempts", "n_dims_part")] + \
               [(n, ctypes.c_void_p) for n in ("boxes", "nbox", "sel", "crop_mm", "dims_part",
                                                "dims_min", "dims_max", "corners", "centers",
                                                "centers_normalized", "sem_cls", "present", "sizes",
                                                "sizes_normalized", "angles", "angle_cls",
                                                "angle_res")]


def byref(struct):
    """address of a ctypes structure, for a "p" argument (the caller keeps it alive)"""
    return ctypes.c_void_p(ctypes.addressof(struct))


def multi_copy(dsts, srcs):
    """copy every src tensor into the same-size dst tensor (contiguous, device) in one launch"""
    n = len(dsts)
    if n == 0:
        return
    for d, s in zip(dsts, srcs):
        if d.nbytes != s.nbytes or not (d.is_contiguous() and s.is_contiguous()) or d.dtype != s.dtype:
            raise ValueError("multi_copy: contiguous same-dtype, same-size tensors only")
        check_device(d, "multi_copy dst")
        check_device(s, "multi_copy src")
    sp = (ctypes.c_void_p * n)(*[s.data_ptr() for s in srcs])
    dp = (ctypes.c_void_p * n)(*[d.data_ptr() for d in dsts])
    nb = (ctypes.c_longlong * n)(*[d.nbytes for d in dsts])
    call("ov3d_multi_copy", n, ctypes.addressof(sp), ctypes.addressof(dp), ctypes.addressof(nb),
         like=dsts[0])
