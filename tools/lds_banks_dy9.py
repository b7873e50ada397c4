"""Bank-conflict census of sa_dy9's LDS accesses (csrc/sa_bwd.hip), from the lane groups and
bank rules of MI355X_MICROARCH.md §LDS: ds_read_b64 / ds_read_b64_tr_b16 serve lanes 0-31 and
32-63 per cycle over 64 banks, ds_read_b128 four fixed groups of 16 lanes over 64 banks,
ds_write_b64 four groups of 16 lanes and ds_write_b128 eight groups of 8 over 32 banks (2-byte
writes taken as b32 writes of their dword: lanes writing halves of one dword do not conflict).  Prints the
extra LDS cycles each access pattern costs per tile (0 = conflict-free) and checks that the
swizzled dy3^T image (dsw) maps every (channel, row) to its own element."""


def zsw(r):
    return ((r & 3) << 2) | ((r >> 2) & 3)


def zimg(r, k):               # element of (row r, column k) in the swizzled As / W3s images
    return r * 128 + 8 * ((k >> 3) ^ zsw(r)) + (k & 7)


def dsw(n):
    return (((n >> 1) & 1) << 3) | (((n >> 3) & 1) << 2) | (((n >> 2) & 1) << 1) | ((n ^ (n >> 4)) & 1)


LDR, LDY = 64, 160            # DsT line (bf16), Ys row stride (bf16)


def dst(n, row):              # element of (channel n, tile row) in the swizzled DsT image
    return n * LDR + 4 * ((row >> 2) ^ dsw(n)) + (row & 3)


def extra(groups, byte_addr, dwords, nbanks):
    cyc = 0
    for g in groups:
        banks = {}
        for lane in g:
            for d in range(dwords):
                dw = byte_addr[lane] // 4 + d
                banks.setdefault(dw % nbanks, set()).add(dw)
        cyc += max(len(v) for v in banks.values()) - 1
    return cyc


HALVES = [range(32), range(32, 64)]
QUARTERS = [range(q, q + 16) for q in range(0, 64, 16)]
B128 = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)],
        [*range(32, 36), *range(44, 48), *range(52, 60)], [*range(36, 44), *range(48, 52), *range(60, 64)]]
EIGHTS = [range(q, q + 8) for q in range(0, 64, 8)]


def tr16_lane(lane, c0, s, hi):   # col_operand's (row k0, column d0) of a lane
    g, i = lane >> 4, lane & 15
    return 16 * s + 4 * (g >> 1) + (i >> 2) + 8 * hi, c0 + 16 * (g & 1) + 4 * (i & 3)


def main():
    res = {}
    t = 0   # dz A operand: lines n = k0 (channels), rows d0 of row block rbz
    for rbz in (0, 1):
        for s in range(16):
            for hi in (0, 1):
                a = {}
                for lane in range(64):
                    n, row = tr16_lane(lane, 32 * rbz, s, hi)
                    a[lane] = 2 * dst(n, row)
                t += extra(HALVES, a, 2, 64)
    res["dz tr16 reads of DsT"] = t
    t = 0   # dW3 A operand: line ny = 32w + r32, pieces 4s + h (+2)
    for w in range(8):
        for s in range(4):
            for hi in (0, 1):
                a = {lane: 2 * dst(32 * w + (lane & 31), 16 * s + 4 * (lane >> 5) + 8 * hi) for lane in range(64)}
                t += extra(HALVES, a, 2, 64)
    res["dW3 b64 reads of DsT"] = t
    t = 0   # y3 epilogue: line ny, rows rb*32 + 8q + 4h .. +3
    for w in range(8):
        for rb in (0, 1):
            for q in range(4):
                a = {lane: 2 * dst(32 * w + (lane & 31), 32 * rb + 8 * q + 4 * (lane >> 5)) for lane in range(64)}
                t += extra(QUARTERS, a, 2, 32)
    res["y3 b64 writes of DsT"] = t
    t = 0   # statistics: Ys rows read transposed, columns kbz + r32
    for kbz in (0, 32, 64, 96):
        for s in range(4):
            for hi in (0, 1):
                a = {}
                for lane in range(64):
                    k0, d0 = tr16_lane(lane, kbz, s, hi)
                    a[lane] = 2 * (k0 * LDY + d0)
                t += extra(HALVES, a, 2, 64)
    res["Ys tr16 reads"] = t
    t = 0   # y3 A / B operands: ds_read_b128 of rows (As: rb*32 + r32; W3s: 32w + r32), k 16s + 8h
    for base in range(0, 256, 32):
        for s in range(8):
            a = {lane: 2 * zimg(base + (lane & 31), 16 * s + 8 * (lane >> 5)) for lane in range(64)}
            t += extra(B128, a, 4, 64)
    res["y3 b128 reads of As/W3s"] = t
    t = 0   # dW3 B operand (As, columns 32b..) and dz B operand (W3s, columns kbz..): tr16
    for rows0 in range(0, 256, 16):
        for c0 in (0, 32, 64, 96):
            for hi in (0, 1):
                a = {}
                for lane in range(64):
                    r, k = tr16_lane(lane, c0, 0, hi)
                    a[lane] = 2 * zimg(rows0 + r, k)
                t += extra(HALVES, a, 2, 64)
    res["tr16 reads of As/W3s"] = t
    t = 0   # prologue ds_write_b128: thread ch -> row ch/16, k 8(ch%16) (8 lanes per group, mod 32)
    for c in range(2):
        for w in range(8):
            a = {}
            for lane in range(64):
                ch = w * 64 + lane + 512 * c
                a[lane] = 2 * zimg(ch // 16, 8 * (ch % 16))
            t += extra(EIGHTS, a, 4, 32)
    res["As b128 writes"] = t
    t = 0   # Dz: 2-byte writes of (row rbz*32 + 4h + ..., channel kbz + r32); b128 reads of rows
    for w in range(8):
        for i in range(16):
            a = {lane: 2 * ((32 * (w >> 2) + 4 * (lane >> 5) + (i & 3) + 8 * (i >> 2)) * 128 + 32 * (w & 3) + (lane & 31))
                 for lane in range(64)}
            t += extra(HALVES, {k: v - v % 4 for k, v in a.items()}, 1, 32)
    for c in range(2):
        for w in range(8):
            a = {lane: 2 * 8 * (w * 64 + lane + 512 * c) for lane in range(64)}
            t += extra(B128, a, 4, 64)
    res["Dz writes + reads"] = t
    assert sorted(zimg(r, k) for r in range(64) for k in range(128)) == list(range(64 * 128))
    seen = {dst(n, r) for n in range(256) for r in range(64)}
    assert len(seen) == 256 * 64 and min(seen) == 0 and max(seen) == 256 * 64 - 1
    for k, v in res.items():
        print(f"{k:24s} extra cycles per tile: {v}")
    return res


def asw(r):
    return ((r >> 1) & 1) << 2


def dy2_census(swizzled=True):
    """sa_dy2_fused (K = 64 layer-1 channels, N = 128 layer-2 channels, 4 waves): extra LDS cycles
    per tile of each access pattern; swizzled=False: the round-5 padded rows (72 / 136 bf16)."""
    K, N = 64, 128
    if swizzled:
        def ds(r, n): return r * N + 8 * ((n >> 3) ^ zsw(r)) + (n & 7)
        def az(r, k): return r * K + 8 * ((k >> 3) ^ asw(r)) + (k & 7)
        def ys(r, k): return r * (K + 68) + k
    else:
        def ds(r, n): return r * (N + 8) + n
        def az(r, k): return r * (K + 8) + k
        def ys(r, k): return r * (K + 8) + k
    res = {}
    t = 0   # prologue writes: As / Ds ds_write_b128 (8-lane groups, 32 banks), Ys 2 x ds_write_b64
    for w in range(4):
        for c in range(2):
            a = {l: 2 * az((w * 64 + l + 256 * c) // 8, 8 * ((w * 64 + l + 256 * c) % 8)) for l in range(64)}
            t += extra(EIGHTS, a, 4, 32)
            for half in (0, 4):
                a = {l: 2 * ys((w * 64 + l + 256 * c) // 8, 8 * ((w * 64 + l + 256 * c) % 8) + half)
                     for l in range(64)}
                t += extra(QUARTERS, a, 2, 32)
        for c in range(4):
            a = {l: 2 * ds((w * 64 + l + 256 * c) // 16, 8 * ((w * 64 + l + 256 * c) % 16)) for l in range(64)}
            t += extra(EIGHTS, a, 4, 32)
    res["prologue writes"] = t
    t = 0   # dz1 B operand: Ds rows rb*32 + r32, n = 16s + 8h (ds_read_b128)
    for w in range(4):
        rb = w >> 1
        for s in range(8):
            a = {l: 2 * ds(rb * 32 + (l & 31), 16 * s + 8 * (l >> 5)) for l in range(64)}
            t += extra(B128, a, 4, 64)
    res["dz1 b128 reads of Ds"] = t
    t = 0   # layer-1 statistics: Ys row rb*32 + r32, channels kbase + 8g + 4h (ds_read_b64)
    for w in range(4):
        kbase, rb = (w & 1) * 32, w >> 1
        for g in range(4):
            a = {l: 2 * ys(rb * 32 + (l & 31), kbase + 8 * g + 4 * (l >> 5)) for l in range(64)}
            t += extra(HALVES, a, 2, 64)
    res["Ys b64 reads"] = t
    t = 0   # dW2: A = Ds transposed (columns 32w..), B = As transposed (columns 32b..), tr16
    for w in range(4):
        for s in range(4):
            for hi in (0, 1):
                a = {}
                for l in range(64):
                    r, n = tr16_lane(l, 32 * w, s, hi)
                    a[l] = 2 * ds(r, n)
                t += extra(HALVES, a, 2, 64)
                for b in (0, 1):
                    a = {}
                    for l in range(64):
                        r, k = tr16_lane(l, 32 * b, s, hi)
                        a[l] = 2 * az(r, k)
                    t += extra(HALVES, a, 2, 64)
    res["dW2 tr16 reads of Ds / As"] = t
    if swizzled:
        assert sorted(ds(r, n) for r in range(64) for n in range(N)) == list(range(64 * N))
        assert sorted(az(r, k) for r in range(64) for k in range(K)) == list(range(64 * K))
    return res


def isw(r):
    return (((r >> 1) & 1) << 2) | ((r >> 2) & 3)


def attn_census(swizzled=True):
    """csrc/attn.hip K / V / Q / dO tile images (64 rows x 64 bf16): extra LDS cycles per tile and
    wave of the row reads (ds_read_b128, rows 32t + r, columns 16s + 8h), the transposed reads of
    v_operand (ds_read_b64_tr_b16) and the tile stores (ds_write_b128, 8 lanes a row);
    swizzled=False: the round-5 padded 72-element rows."""
    if swizzled:
        def f(r, c): return r * 64 + 8 * ((c >> 3) ^ isw(r)) + (c & 7)
    else:
        def f(r, c): return r * 72 + c
    res = {"row reads": 0, "transposed reads": 0, "stores": 0}
    for t in (0, 1):
        for s in range(4):
            a = {l: 2 * f(32 * t + (l & 31), 16 * s + 8 * (l >> 5)) for l in range(64)}
            res["row reads"] += extra(B128, a, 4, 64)
    for dt in (0, 1):
        for t in (0, 1):
            for s in (0, 1):
                for hi in (0, 1):
                    a = {}
                    for l in range(64):
                        g, i = l >> 4, l & 15
                        a[l] = 2 * f(32 * t + 16 * s + 4 * (g >> 1) + (i >> 2) + 8 * hi,
                                     32 * dt + 16 * (g & 1) + 4 * (i & 3))
                    res["transposed reads"] += extra(HALVES, a, 2, 64)
    for c in (0, 1):
        for w in range(4):
            a = {l: 2 * f((w * 64 + l + 256 * c) >> 3, 8 * ((w * 64 + l + 256 * c) & 7)) for l in range(64)}
            res["stores"] += extra(EIGHTS, a, 4, 32)
    if swizzled:
        assert sorted(f(r, c) for r in range(64) for c in range(64)) == list(range(64 * 64))
    return res


def rows256_census(swizzled=True):
    """csrc/rows256.hip X tile image (128 rows x 256 bf16, 512-byte rows, 16-byte chunk c of row r
    at c ^ (r & 15)): extra LDS cycles per tile and wave of the fragment reads (ds_read_b128:
    lane l reads row 16 rb + (l & 15), logical chunk 4 ks + (l >> 4)); the image is written by
    LDS-DMA (lane-linear 1 KB pieces, no bank rule).  swizzled=False: plain rows."""
    def f(r, c):   # byte address of logical 16-byte chunk c of row r
        return r * 512 + 16 * ((c ^ (r & 15)) if swizzled else c)
    cyc = 0
    for rb in range(8):
        for ks in range(8):
            a = {l: f(16 * rb + (l & 15), 4 * ks + (l >> 4)) for l in range(64)}
            cyc += extra(B128, a, 4, 64)
    if swizzled:
        assert sorted(f(r, c) // 16 for r in range(128) for c in range(32)) == list(range(128 * 32))
    return cyc


if __name__ == "__main__":
    main()
    for sw in (False, True):
        for k, v in attn_census(sw).items():
            print(f"attn {'swizzled' if sw else 'padded  '} {k:18s} extra cycles per tile and wave: {v}")
    for sw in (False, True):
        print(f"rows256 {'swizzled' if sw else 'plain   '} fragment reads extra cycles per tile and wave: "
              f"{rows256_census(sw)}")
    for sw in (False, True):
        for k, v in dy2_census(sw).items():
            print(f"sa_dy2 {'swizzled' if sw else 'padded  '} {k:28s} extra cycles per tile: {v}")
