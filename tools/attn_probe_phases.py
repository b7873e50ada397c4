"""Phase stamps of the flash-attention forward (attn_fwd_kernel) on the encoder shape.

    python tools/attn_probe_phases.py build   # (CPU) tools/probe/libov3d_attnprobe.so, attn.hip with -DOV3D_ATTN_PROBE
    python tools/attn_probe_phases.py run     # (GPU) per-phase s_memtime cycles per 64-key tile, p = 0 and 0.1
    python tools/attn_probe_phases.py run dec # the same for the decoder cross attention (128 x 2048 keys,
                                              # split-K): "prologue" = kernel entry to the first tile

Phases per tile and wave: 0 loop top (the barrier's exit to the next tile), 1 K LDS reads + QK^T
MFMAs issued + V operand reads + next-tile global loads issued, 2 row max (waits for the
score MFMAs), 3 exp / row sum / dropout / bf16 pack, 4 PV MFMAs issued, 5 next tile's LDS
store, 6 barrier.
"""
import ctypes
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "open-vocabulary-3d-object-detection_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "attnprobe")   # travels to the GPU box (tools/probe is gpurun-ignored)
LIB = os.path.join(OUT, "libov3d_attnprobe.so")
PHASES = ["top", "qk_issue", "rowmax", "softmax", "pv_issue", "lds_store", "barrier", "prologue"]


def build():
    os.makedirs(OUT, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
             "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"]
    obj = os.path.join(OUT, "attn_probe.o")
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-DOV3D_ATTN_PROBE", "-c",
                    os.path.join(CSRC, "attn.hip"), "-o", obj], check=True)
    others = [o for o in glob.glob(os.path.join(CSRC, "*.o")) if not o.endswith("attn.o")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", LIB, obj, *others],
                   check=True)
    print("built", LIB)


def run():
    import torch
    sys.path.insert(0, ROOT)
    import ov3d_import
    ov3d_import.load()
    from ov3d_amd import _native
    _native.LIB_PATH = LIB
    lib = _native.load()
    from ov3d_amd import attention as A
    lib.ov3d_attn_probe_set.argtypes = [ctypes.c_void_p]
    B, H, L = 8, 4, 2048
    Lq = 128 if (len(sys.argv) > 2 and sys.argv[2] == "dec") else L
    E = H * 64
    q = torch.randn(Lq, B, E, device="cuda", dtype=torch.bfloat16)
    kv = torch.randn(L, B, 2 * E, device="cuda", dtype=torch.bfloat16)
    spec = ((0, 0), (1, 0), (1, E))
    nsplit = A._split(Lq, L, B * H)
    nwg = (Lq // 128) * B * H * nsplit
    res = {}
    for p in (0.0, 0.1):
        for _ in range(3):
            A.attention_packed([q, kv], spec, Lq, L, H, p, site=1)
        torch.cuda.synchronize()
        dbg = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device="cuda")
        lib.ov3d_attn_probe_set(dbg.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        A.attention_packed([q, kv], spec, Lq, L, H, p, site=1)
        e1.record()
        torch.cuda.synchronize()
        lib.ov3d_attn_probe_set(None)
        d = dbg.view(nwg, 4, 8).double().cpu()
        tiles = L // 64 // nsplit
        per = (d.mean((0, 1)) / tiles).tolist()
        per[7] *= tiles   # the prologue: once per wave, not per tile
        tot = d.sum(2)
        us = e0.elapsed_time(e1) * 1e3
        res[f"p={p}"] = {"cycles_per_tile": dict(zip(PHASES, [round(x) for x in per])),
                         "total_per_tile": round(sum(per)),
                         "wave_total_cycles_mean": round(float(tot.mean())),
                         "wave_total_cycles_max": round(float(tot.max())),
                         "kernel_us": round(us, 1),
                         "implied_clock_GHz_from_max_wave": round(float(tot.max()) / us / 1e3, 3)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
