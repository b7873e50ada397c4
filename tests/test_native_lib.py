"""The C-ABI library: loads, exports every entry point include/ov3d.h declares,
and the product refuses CPU tensors (no silent fallback).  No compute here."""
import ctypes
import os
import re

import pytest
import torch

from helpers import ROOT, ov3d


def header_symbols():
    src = open(os.path.join(ROOT, "include", "ov3d.h")).read()
    return sorted(set(re.findall(r"^(?:int|long long|const char\*)\s+(ov3d_\w+)\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    from ov3d_amd import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 11
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_native.EXPORTS)


def test_ctypes_signatures_match_header_arity():
    """_native._SIGS (argument kinds incl. the trailing stream) vs the header prototypes."""
    from ov3d_amd import _native
    src = open(os.path.join(ROOT, "include", "ov3d.h")).read()
    protos = dict(re.findall(r"^int\s+(ov3d_\w+)\(([^)]*)\);", src, flags=re.M))
    for name, sig in _native._SIGS.items():
        params = [a.strip() for a in protos[name].split(",")]
        assert len(params) == len(sig), (name, len(params), len(sig))
        for a, k in zip(params, sig):
            if "*" in a:
                assert k == "p", (name, a)
            elif a.startswith("double"):
                assert k == "d", (name, a)
            elif a.startswith("float"):
                assert k == "f", (name, a)
            elif a.startswith("long long"):
                assert k == "l", (name, a)
            else:
                assert k == "i", (name, a)


def test_version_string():
    from ov3d_amd import _native
    assert "gfx950" in _native.version()


def test_no_cpu_fallback():
    from ov3d_amd import _native, pointnet2_utils
    with pytest.raises(_native.NativeError):
        pointnet2_utils.furthest_point_sample(torch.zeros(1, 16, 3), 4)
    from ov3d_amd.box_util import generalized_box3d_iou
    with pytest.raises(_native.NativeError):
        generalized_box3d_iou(torch.zeros(1, 2, 8, 3), torch.zeros(1, 2, 8, 3), torch.tensor([2]))


def test_missing_library_fails_loudly(monkeypatch):
    from ov3d_amd import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libov3d_hip.so")
    with pytest.raises(_native.NativeError):
        _native.load()


def test_package_exports_drop_in_modules():
    import importlib
    for m in ("pointnet2_utils", "pointnet2_modules", "model_3detr", "criterion", "box_util", "nms",
              "dist", "transformer", "helpers", "position_embedding"):
        importlib.import_module("ov3d_amd." + m)
    assert callable(ov3d.build_model) and callable(ov3d.build_criterion)


def test_round4_entries_reject_bad_arguments():
    """The RegionCLIP close / pool / token entries and the squared-distance mask
    kind validate before touching the device (host-side checks; no GPU needed)."""
    from ov3d_amd import _native
    lib = _native.load()
    fake = ctypes.c_void_p(16)   # never dereferenced: every call below fails validation first
    assert lib.ov3d_bias_residual_act(None, 2, 4, 8, None, None, 1, None) == -1
    assert lib.ov3d_bias_residual_act(fake, 2, 4, 7, fake, fake, 1, None) == -1      # cols % 8
    assert lib.ov3d_avgpool2_nhwc(None, 2, 1, 4, 4, 8, None, None) == -1
    assert lib.ov3d_avgpool2_nhwc(fake, 3, 1, 4, 4, 8, fake, None) == -1            # elem bytes
    assert lib.ov3d_attnpool_tokens(None, 2, 1, 81, 64, None, None, None) == -1
    assert lib.ov3d_attn_mask_pack(fake, 3, 1.0, 1, 32, 64, fake, None) == -1        # kind 3


def test_round5_entries_reject_bad_arguments():
    """ov3d_gemm256 / ov3d_conv3x3_gemm256 validate shapes, strides and alignment before any
    launch; ov3d_sa_dy_fused keeps its argument checks (its > 2 GiB inputs route to the 64-bit
    kernel instead of failing).  Host-side checks only."""
    from ov3d_amd import _native
    lib = _native.load()
    p = ctypes.c_void_p(256)      # 16-byte aligned, never dereferenced
    odd = ctypes.c_void_p(264)    # 8-byte aligned only
    ok = dict(A=p, lda=128, B=p, ldb=128, bias=None, bf=0, R=None, ldr=0, C=p, ldc=64, M=100,
              N=64, K=128, relu=0)

    def g(**kw):
        a = dict(ok, **kw)
        return lib.ov3d_gemm256(a["A"], a["lda"], a["B"], a["ldb"], a["bias"], a["bf"], a["R"],
                                a["ldr"], a["C"], a["ldc"], a["M"], a["N"], a["K"], a["relu"], None)
    assert g(A=None) == -1
    assert g(K=100) == -1             # K % 8
    assert g(N=60, ldc=64) == -1      # N % 8
    assert g(lda=100) == -1           # lda < K
    assert g(ldb=136 + 4) == -1       # ldb % 8
    assert g(C=odd) == -1             # 16-byte alignment
    assert g(R=p, ldr=32) == -1       # ldr < N
    assert g(M=0) == -1
    assert lib.ov3d_conv3x3_gemm256(p, 2, 9, 9, 96, p, 864, None, 0, None, 0, p, 64, 64, 1,
                                    None) == -1   # Cin % 64
    assert lib.ov3d_conv3x3_gemm256(p, 2, 9, 9, 64, p, 512, None, 0, None, 0, p, 64, 64, 1,
                                    None) == -1   # ldb < 9 Cin
    assert lib.ov3d_conv3x3_gemm256(None, 2, 9, 9, 64, p, 576, None, 0, None, 0, p, 64, 64, 1,
                                    None) == -1
    assert lib.ov3d_sa_dy_fused(None, None, None, None, 1 << 23, 128, 256, 64, None, None, None,
                                None, None, None, None, None, None, None, None, 1, None) == -1
    # the fused attention pool: shape limits, strides and alignment
    assert lib.ov3d_attnpool_fused_supported(81, 2560, 40) == 1
    assert lib.ov3d_attnpool_fused_supported(96, 2560, 40) == 0      # ntok + 1 > 96
    assert lib.ov3d_attnpool_fused_supported(81, 2560, 49) == 0      # H > 48
    assert lib.ov3d_attnpool_fused_supported(81, 2500, 40) == 0      # C % 64
    assert lib.ov3d_attnpool_fused(p, p, p, p, 40 * 2560, 2560, 4, 81, 2560, 49, p, None) == -1
    assert lib.ov3d_attnpool_fused(p, p, p, p, 40 * 2560, 2564, 4, 81, 2560, 40, p, None) == -1
    assert lib.ov3d_attnpool_fused(p, p, p, odd, 40 * 2560, 2560, 4, 81, 2560, 40, p, None) == -1
    assert lib.ov3d_attnpool_mean(p, 4, 81, 2564, p, p, None) == -1          # C % 8
    assert lib.ov3d_attnpool_mean(None, 4, 81, 2560, p, p, None) == -1
