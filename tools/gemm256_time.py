"""Per-call time of the 256 x 256 tile GEMM / implicit-GEMM 3x3 convolution (csrc/gemm256.hip)
against the library path it replaces (hipBLASLt through torch; im2col + hipBLASLt for the 3x3
convolutions), same random operands, back-to-back launches bracketed by HIP events; TFLOP/s and
max |diff| against each other.  python tools/gemm256_time.py [--reps 10] [--json out.json]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402

# (name, M, N, K, bias, residual, relu)
GEMMS = [("square 8192^3", 8192, 8192, 8192, False, False, False),
         ("res5 b1 conv1 18x18 (1024 ROIs)", 1024 * 324, 640, 1280, True, False, True),
         ("res5 b1 downsample 9x9 (4096 ROIs)", 4096 * 81, 2560, 1280, True, False, False),
         ("res5 conv3+close 9x9 (4096 ROIs)", 4096 * 81, 2560, 640, True, True, True),
         ("res5 conv1 9x9 (4096 ROIs)", 4096 * 81, 640, 2560, True, False, True),
         ("decoder memory K/V (8 layers)", 16384, 2048, 256, True, False, False)]
# (name, n, H, W, C, Cout)
CONVS = [("res5 b1 conv2 18x18 (1024 ROIs)", 1024, 18, 18, 640, 640),
         ("res5 conv2 9x9 (4096 ROIs)", 4096, 9, 9, 640, 640)]


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        torch.cuda._sleep(int(2e6))
    except Exception:
        pass
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="substring filter on the shape names")
    ap.add_argument("--no-lib", action="store_true", help="time gemm256 only")
    a = ap.parse_args()
    ov3d_import.load()
    from ov3d_amd import _native, gemm
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    rows = []
    for name, M, N, K, hb, hr, relu in GEMMS:
        if a.only and a.only not in name:
            continue
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev, generator=g).to(torch.bfloat16) if hb else None
        r = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16) if hr else None
        own = lambda: gemm.gemm256(x, w, bias=b, residual=r, relu=relu)

        def lib():
            y = torch.nn.functional.linear(x, w, b)
            if r is not None:
                y += r
            return y.relu_() if relu else y
        t_own = timed(own, a.reps)
        t_lib = float('nan') if a.no_lib else timed(lib, a.reps)
        d = float('nan') if a.no_lib else (own().float() - lib().float()).abs().max().item()
        fl = 2.0 * M * N * K
        rows.append({"shape": name, "M": M, "N": N, "K": K, "ms_gemm256": round(t_own, 4),
                     "ms_library": round(t_lib, 4), "tflops_gemm256": round(fl / t_own / 1e9, 1),
                     "tflops_library": round(fl / t_lib / 1e9, 1), "max_abs_diff": d})
        print(rows[-1], flush=True)
        del x, w, r
        torch.cuda.empty_cache()
    if not a.only or a.only in "decoder memory K/V pair":
        M, N, K = 16384, 2048, 256
        x1, x2 = (torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16) for _ in range(2))
        w1, w2 = ((torch.randn(N, K, device=dev, generator=g) / 16).to(torch.bfloat16) for _ in range(2))
        b1, b2 = (torch.randn(N, device=dev, generator=g).to(torch.bfloat16) for _ in range(2))
        own = lambda: gemm.gemm256_pair(x1, w1, b1, x2, w2, b2)
        lib = lambda: (torch.addmm(b1, x1, w1.t()), torch.addmm(b2, x2, w2.t()))
        t_own = timed(own, a.reps)
        t_lib = float('nan') if a.no_lib else timed(lib, a.reps)
        fl = 4.0 * M * N * K
        rows.append({"shape": "decoder memory K/V pair (one launch vs two addmm)", "M": M, "N": N,
                     "K": K, "ms_gemm256": round(t_own, 4), "ms_library": round(t_lib, 4),
                     "tflops_gemm256": round(fl / t_own / 1e9, 1),
                     "tflops_library": round(fl / t_lib / 1e9, 1)})
        print(rows[-1], flush=True)
    for name, n, H, W, C, cout in CONVS:
        if a.only and a.only not in name:
            continue
        x = torch.randn(n, H, W, C, device=dev, generator=g).to(torch.bfloat16)
        wm = (torch.randn(cout, 9 * C, device=dev, generator=g) / (9 * C) ** 0.5).to(torch.bfloat16)
        b = torch.randn(cout, device=dev, generator=g).to(torch.bfloat16)
        M = n * H * W
        own = lambda: gemm.conv3x3_gemm256(x, wm, bias=b, relu=True)
        cols = torch.empty((M, 9 * C), dtype=torch.bfloat16, device=dev)

        def lib():
            _native.call("ov3d_im2col3x3", x, 2, n, H, W, C, 1, 9 * C, cols, like=x)
            return torch._addmm_activation(b, cols, wm.t())
        t_own = timed(own, a.reps)
        t_lib = float('nan') if a.no_lib else timed(lib, a.reps)
        d = float('nan') if a.no_lib else (own().reshape(M, cout).float() - lib().float()).abs().max().item()
        fl = 2.0 * M * cout * 9 * C
        rows.append({"shape": name, "M": M, "N": cout, "K": 9 * C, "ms_gemm256": round(t_own, 4),
                     "ms_library": round(t_lib, 4), "library": "ov3d_im2col3x3 + hipBLASLt",
                     "tflops_gemm256": round(fl / t_own / 1e9, 1),
                     "tflops_library": round(fl / t_lib / 1e9, 1), "max_abs_diff": d})
        print(rows[-1], flush=True)
        del x, cols
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
