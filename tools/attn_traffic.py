"""profiles/r04_attn_pmc.json from a tools/gpu_pmc.sh summary: HBM bytes per launch of the encoder
self-attention forward (FETCH_SIZE doubled for gfx950, MI355X_MICROARCH.md; + WRITE_SIZE).
python tools/attn_traffic.py gpurun_out/pmc/summary.json profiles/r04_attn_pmc.json"""
import json
import sys

KEY = "attn_fwd_kernel<true, false, false> grid=131072"


def main(src, dst):
    d = json.load(open(src))[KEY]
    f, w = d["FETCH_SIZE"]["mean"], d["WRITE_SIZE"]["mean"]
    out = {"kernel": KEY,
           "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, tools/gpu_pmc.sh) of the "
                   "encoder self-attention forward (B 8, H 4, L 2048, dropout 0.1) in an eager bench "
                   "step; FETCH_SIZE doubled for gfx950 (MI355X_MICROARCH.md). Algorithmic bytes: Q, K, "
                   "V 3 x 8 MiB read, O 8 MiB + drop words 32 MiB + lse written.",
           "fetch_size_kb_raw": f, "write_size_kb": w,
           "fwd_traffic_bytes_per_launch": int((2 * f + w) * 1024),
           "source": src}
    json.dump(out, open(dst, "w"), indent=1)
    print(out["fwd_traffic_bytes_per_launch"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
