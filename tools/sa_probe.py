"""Phase stamps of the SA layer-3 backward kernel (sa_dy9_kernel) on the GPU.

    python tools/sa_probe.py build     # (CPU) tools/probe/libov3d_saprobe.so, sa_bwd.hip with -DOV3D_SA_PROBE
    python tools/sa_probe.py run       # (GPU) one eager SUN training step, per-phase cycles per tile
    python tools/sa_probe.py run fwd   # (GPU) the same for the layer-3 forward (sa_layer_kernel)

Phases (per tile, per wave, s_memtime cycles): 1 prologue z -> LDS, 2 barrier, 3 y3 MFMA +
dy3 epilogue, 4 barrier, 5 dz MFMA + store + stats, 6 dW MFMA, 7 barrier.
"""
import ctypes
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "open-vocabulary-3d-object-detection_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "saprobe")   # travels to the GPU box (tools/probe does not)
LIB = os.path.join(OUT, "libov3d_saprobe.so")
PHASES = ["loop", "prologue", "barrier1", "y3+dy3", "barrier2", "dz+stats", "dW", "barrier3"]


def build():
    os.makedirs(OUT, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off"]
    objs = []
    for src in ("sa_bwd", "sa_mlp"):
        objs.append(os.path.join(OUT, src + "_probe.o"))
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-DOV3D_SA_PROBE", "-c",
                        os.path.join(CSRC, src + ".hip"), "-o", objs[-1]], check=True)
    others = [o for o in glob.glob(os.path.join(CSRC, "*.o"))
              if not o.endswith(("sa_bwd.o", "sa_mlp.o"))]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", LIB, *objs, *others,
                    "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib"],
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
    import bench
    from ov3d_amd import synthetic, sa_fused
    dev = torch.device("cuda", 0)
    args = bench.default_args()
    model, crit, opt = bench.build(args, dev)
    batch = synthetic.make_batch(8, seed=1, device=dev)
    for _ in range(2):
        bench.train_step(model, crit, opt, batch, args, torch.bfloat16)
    torch.cuda.synchronize()
    fwd = len(sys.argv) > 2 and sys.argv[2] == "fwd"   # the layer-3 forward (sa_layer_kernel POOL)
    nwg = sa_fused.NPARTS_LAYER if fwd else sa_fused.NWG_DY_FUSED
    waves = 4 if fwd else 8
    dbg = torch.zeros(nwg * waves * 8, dtype=torch.int64, device=dev)
    setter = lib.ov3d_sal_probe_set if fwd else lib.ov3d_sa_probe_set
    setter.argtypes = [ctypes.c_void_p]
    setter(dbg.data_ptr())
    bench.train_step(model, crit, opt, batch, args, torch.bfloat16)
    torch.cuda.synchronize()
    setter(None)
    d = dbg.view(nwg, waves, 8).double().cpu()
    tiles = (8 * 2048 * 64 // 64) / nwg
    per = (d.mean((0, 1)) / tiles).tolist()
    names = ["loop", "prologue", "barrier1", "MFMA", "barrier2", "epilogue", "-", "-"] if fwd else PHASES
    res = {"tiles_per_wg": tiles, "cycles_per_tile_by_phase": dict(zip(names, [round(x) for x in per])),
           "total_cycles_per_tile": round(sum(per)),
           "by_wave_total": [round(x) for x in (d.sum(2).mean(0) / tiles).tolist()]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
