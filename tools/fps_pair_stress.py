"""Repeat the two-workgroup FPS (20480 < N <= 40960) on fixed inputs and compare every run
with the oracle's indices (the cross-workgroup exchange is the thing under test: a race shows
as an occasional mismatch).  Per mismatching scene it prints the two halves' XCC ids and the
exchange path they chose (read back from the kernel's hand-shake words).
python tools/fps_pair_stress.py [reps]   (OV3D_FPS_XCH=mem: force the memory path)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    ov3d_import.load()
    from oracle import oracle as O
    from ov3d_amd import _native as nat
    lib = nat.load()
    alt = None
    if len(sys.argv) > 2:   # another build's ov3d_fps (diagnostic: an earlier version of fps.hip)
        import ctypes
        alt = ctypes.CDLL(sys.argv[2]).ov3d_fps
        alt.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        alt.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    bad = 0
    for B, N, M in ((3, 30000, 700), (8, 40000, 2048), (2, 40000, 1024), (5, 25000, 300), (8, 30000, 700)):
        g = np.random.default_rng(B * N + M)
        xyz = g.uniform(-3, 3, (B, N, 3)).astype(np.float32)
        ref = O.fps(xyz, M)
        x = torch.from_numpy(xyz).to(dev)
        ws = torch.zeros(max(lib.ov3d_fps_workspace(B, N), 1), dtype=torch.float32, device=dev)
        nbad = 0
        modes = {}
        for _ in range(reps):
            idx = torch.empty((B, M), dtype=torch.int32, device=dev)
            if alt is not None:
                assert alt(x.data_ptr(), B, N, M, idx.data_ptr(), None, ws.data_ptr(),
                           nat._stream(x)) == 0
            else:
                nat.call("ov3d_fps", x, B, N, M, idx, None, ws, like=x)
            torch.cuda.synchronize()
            hs = ws.view(torch.int32)[B * 64:B * 128].view(B, 2, 32).cpu().numpy()
            got = idx.cpu().numpy()
            for b in range(B):
                key = (int(hs[b, 0, 0]), int(hs[b, 1, 0]), int(hs[b, 0, 4]), int(hs[b, 1, 4]))
                ok = np.array_equal(got[b], ref[b])
                if not ok:
                    first = int(np.nonzero(got[b] != ref[b])[0][0])
                    print(f"  scene {b}: first wrong sample {first} of {M} (got {got[b][first]}, "
                          f"want {ref[b][first]}), lost flags {hs[b, 0, 8]} {hs[b, 1, 8]}", flush=True)
                m = modes.setdefault(key, [0, 0])
                m[0] += 1
                m[1] += 0 if ok else 1
                nbad += 0 if ok else 1
        bad += nbad
        print(f"B={B} N={N} M={M}: {reps} runs, {nbad} bad scenes; "
              f"(xcc0, xcc1, mem0, mem1) -> [scenes, bad]: {modes}", flush=True)
    print("mismatching scenes:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
