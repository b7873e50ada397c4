"""FPS diagnostics on the GPU: per-phase cycle stamps and A/B timing of build variants.

    python tools/fps_probe.py build          # (CPU container) compile the probe / variant libraries
    python tools/fps_probe.py run            # (GPU box) time + stamp, print a JSON summary

Variants are fps.hip compiled with different -D flags into tools/probe/*.so (git-ignored,
travels with gpurun).  Every variant's indices are compared bit for bit with the product
library's before its time is reported.  The stamp build (-DOV3D_FPS_PROBE) records, per
wave, s_memtime totals for: the update phase of iterations that updated / skipped, the
publish + barrier wait, and the post-barrier reduction (cdna_hip_programming.md §7).
"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "open-vocabulary-3d-object-detection_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "fpsprobe")   # travels to the GPU box (tools/probe is gpurun-ignored)
NONIEEE = ["-mno-amdgpu-ieee", "-fno-honor-nans"]   # the product's fps.o flags (csrc/Makefile)
FPS = os.path.join(CSRC, "fps.hip")
BASE = os.path.join(OUT, "fps_base.hip")      # a saved earlier fps.hip to A/B against (optional)
VARIANTS = {                                   # name -> (source, extra flags)
    "stamps": (FPS, ["-DOV3D_FPS_PROBE", *NONIEEE]),
    "base": (BASE, [*NONIEEE]),
    "cur": (FPS, [*NONIEEE]),
}


def build():
    os.makedirs(OUT, exist_ok=True)
    for name, (src, flags) in VARIANTS.items():
        if not os.path.exists(src):
            continue
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
               "-ffp-contract=off", "-shared", f"-I{CSRC}", *flags, src,
               "-o", os.path.join(OUT, f"libfps_{name}.so")]
        subprocess.run(cmd, check=True)
        print("built", name)


def run():
    import torch
    sys.path.insert(0, ROOT)
    import ov3d_import
    ov3d_import.load()
    from ov3d_amd import _native as nat, synthetic

    dev = torch.device("cuda", 0)
    res = {}
    for (B, N, M) in ((8, 20000, 2048), (8, 2048, 128)):
        if N == 20000:
            xyz = synthetic.make_batch(B, seed=5, num_points=N, device=dev)["point_clouds"][..., :3].contiguous()
        else:
            big = synthetic.make_batch(B, seed=5, num_points=20000, device=dev)["point_clouds"][..., :3].contiguous()
            from ov3d_amd import pointnet2_utils as pu
            _, xyz = pu.furthest_point_sample_gather(big, N)
            xyz = xyz.contiguous()
        ref = torch.empty(B, M, dtype=torch.int32, device=dev)
        nat.call("ov3d_fps", xyz, B, N, M, ref, None, None, like=xyz)
        torch.cuda.synchronize()
        key = f"B{B}_N{N}_M{M}"
        res[key] = {}
        s = torch.cuda.current_stream().cuda_stream
        for name in VARIANTS:
            if not os.path.exists(os.path.join(OUT, f"libfps_{name}.so")):
                continue
            lib = ctypes.CDLL(os.path.join(OUT, f"libfps_{name}.so"))
            f = lib.ov3d_fps
            f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            dbg = None
            if name.endswith("stamps"):
                dbg = torch.zeros(B * 16 * 12, dtype=torch.int64, device=dev)
                lib.ov3d_fps_probe_set.argtypes = [ctypes.c_void_p]
                lib.ov3d_fps_probe_set(dbg.data_ptr())
            idx = torch.empty_like(ref)
            for _ in range(3):
                assert f(xyz.data_ptr(), B, N, M, idx.data_ptr(), None, None, s) == 0
            torch.cuda.synchronize()
            same = bool(torch.equal(idx, ref))
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            reps = 20 if N > 5000 else 100
            ev[0].record()
            for _ in range(reps):
                f(xyz.data_ptr(), B, N, M, idx.data_ptr(), None, None, s)
            ev[1].record()
            torch.cuda.synchronize()
            us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
            r = {"us": round(us, 1), "us_per_iter": round(us / (M - 1), 4), "bitexact": same}
            if dbg is not None:
                d = dbg.view(B, 16, 12).double().cpu()
                upd, cupd, nupd, cnupd, bar, post, cyc, rt, loop, pwm, pslot, pxyz = [d[..., i] for i in range(12)]
                it = (upd + nupd)[0, 0].item()
                r.update({
                    "clock_ghz": round((cyc / rt * 0.1).median().item(), 3),
                    "update_frac": round((upd.sum() / (upd + nupd).sum()).item(), 3),
                    "cyc_per_iter": round((cyc / it).median().item(), 1),
                    "cyc_update_when_updating": round((cupd.sum() / upd.sum().clamp(min=1)).item(), 1),
                    "cyc_update_when_skipping": round((cnupd.sum() / nupd.sum().clamp(min=1)).item(), 1),
                    "cyc_publish_barrier": round((bar / it).median().item(), 1),
                    "cyc_publish_barrier_min_wave": round((bar / it).min(1).values.median().item(), 1),
                    "cyc_post": round((post / it).median().item(), 1),
                    "cyc_update_loop_when_updating": round((loop.sum() / upd.sum().clamp(min=1)).item(), 1),
                    "cyc_to_wave_max_when_updating": round((pwm.sum() / upd.sum().clamp(min=1)).item(), 1),
                    "cyc_wave_max_to_slot": round((pslot.sum() / upd.sum().clamp(min=1)).item(), 1),
                    "cyc_slot_to_coords": round((pxyz.sum() / upd.sum().clamp(min=1)).item(), 1),
                    "barrier_wait_by_wave": [round(x, 1) for x in (bar / it).median(0).values.tolist()],
                    "update_frac_by_wave": [round(x, 3) for x in (upd / it).median(0).values.tolist()],
                })
            res[key][name] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
