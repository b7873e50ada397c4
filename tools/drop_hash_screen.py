"""Statistical screen of attention-dropout hash candidates (numpy, uint32 arithmetic as the
kernels do it).  A hash maps (query q, key pair j) of one (seed, site, b*H+h) to 32 bits; its
low / high 16-bit halves decide the even / odd key: keep iff (half ^ 0x8000) >= round(p*2^16).

Screens, per candidate and p in {0.1, 0.3}:
  rate     drop rate vs p (z-score)
  chi2     byte histograms of both halves' high and low bytes (255 dof)
  pair     correlation of the even / odd decisions of one pair
  nbr      correlation of decisions d apart along the keys (1, 2, 4, 64) and the queries (1, 32)
  rect     4-wise statistic E[(d11-p)(d12-p)(d21-p)(d22-p)] over random query pairs x key
           pairs (rectangles), as a z-score: the structure a per-query x per-key factorised
           input (A_q ^ B_j) could leave behind
python tools/drop_hash_screen.py [--queries 4096] [--pairs 1024] [--heads 4]
"""
import argparse

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def u32(x):
    return (np.asarray(x, np.uint64) & M32).astype(np.uint64)


def mix32(x):
    x = u32(x)
    x ^= x >> np.uint64(16)
    x = u32(x * np.uint64(0x7feb352d))
    x ^= x >> np.uint64(15)
    x = u32(x * np.uint64(0x846ca68b))
    x ^= x >> np.uint64(16)
    return x


def umul24(x, c):
    return u32((u32(x) & np.uint64(0xFFFFFF)) * np.uint64(c & 0xFFFFFF))


def mix24(x):
    x = u32(x)
    x ^= x >> np.uint64(16)
    x = umul24(x, 0x7feb35) ^ (x >> np.uint64(24))
    x ^= x >> np.uint64(15)
    x = umul24(x, 0x846ca7) ^ (x >> np.uint64(24))
    x ^= x >> np.uint64(16)
    return x


K_PAIR = 0x27D4EB2F


def head_mix(seed, site, bh):
    s = np.uint64(seed)
    return mix32(u32(s) ^ mix32(u32((s >> np.uint64(32)) + np.uint64(site * 0x9E3779B9))) ^ u32(bh * 0x85EBCA6B))


def query_base(hm, q):
    return mix32(hm ^ u32(np.asarray(q, np.uint64) * np.uint64(0xC2B2AE35)))


def key_base(hm, j):
    """per (head, key pair) random word (the loader threads' mix32)"""
    return mix32(mix32(hm ^ np.uint64(0x68E31DA4)) + u32(np.asarray(j, np.uint64) * np.uint64(0x9E3779B9)))


def cand_current(hm, q, j):
    # round-3 kernels: mix24(query base + (2h + pair) * kPairMul), pair index j = key >> 1
    return mix24(query_base(hm, q)[:, None] + u32(j[None, :] * np.uint64(K_PAIR)))


def cand_xor_mix24(hm, q, j):
    return mix24(query_base(hm, q)[:, None] ^ key_base(hm, j)[None, :])


def cand_xor_mul(hm, q, j):
    x = query_base(hm, q)[:, None] ^ key_base(hm, j)[None, :]
    y = umul24(x, 0x7feb35)
    return y ^ (y >> np.uint64(16))


def cand_xor_fold_mul(hm, q, j):
    x = query_base(hm, q)[:, None] ^ key_base(hm, j)[None, :]
    x = x ^ (x >> np.uint64(16))
    y = umul24(x, 0x7feb35)
    return y ^ (y >> np.uint64(16))


def cand_xor_fold_mul_top(hm, q, j):
    # fold, multiply, fold the product's top byte back as mix24's first round does
    x = query_base(hm, q)[:, None] ^ key_base(hm, j)[None, :]
    x = x ^ (x >> np.uint64(16))
    y = umul24(x, 0x7feb35) ^ (x >> np.uint64(24))
    return y ^ (y >> np.uint64(15))


def _mix_b1(x):
    x = u32(x)
    x ^= x >> np.uint64(16)
    x = umul24(x, 0x7feb35)
    x ^= x >> np.uint64(16)
    x = umul24(x, 0x846ca7)
    return x ^ (x >> np.uint64(16))


def _mix_b2(x):
    x = u32(x)
    x ^= x >> np.uint64(16)
    x = umul24(x, 0x7feb35) ^ (x >> np.uint64(24))
    x ^= x >> np.uint64(16)
    x = umul24(x, 0x846ca7)
    return x ^ (x >> np.uint64(16))


def _mix_b4(x):
    x = u32(x)
    x ^= x >> np.uint64(16)
    x = umul24(x, 0x7feb35) ^ (x >> np.uint64(24))
    x ^= x >> np.uint64(16)
    x = umul24(x, 0x846ca7) ^ (x >> np.uint64(24))
    return x ^ (x >> np.uint64(16))


def cand_b4(hm, q, j):
    return _mix_b4(query_base(hm, q)[:, None] + u32(j[None, :] * np.uint64(K_PAIR)))


def cand_b1(hm, q, j):
    return _mix_b1(query_base(hm, q)[:, None] + u32(j[None, :] * np.uint64(K_PAIR)))


def cand_b2(hm, q, j):
    return _mix_b2(query_base(hm, q)[:, None] + u32(j[None, :] * np.uint64(K_PAIR)))


CANDS = {"current": cand_current, "b1": cand_b1, "b2": cand_b2, "b4": cand_b4, "xor_mix24": cand_xor_mix24, "xor_mul": cand_xor_mul,
         "xor_fold_mul": cand_xor_fold_mul, "xor_fold_mul_top": cand_xor_fold_mul_top}


def drops(h, p):
    t = np.uint64(int(round(p * 65536)))
    lo = (h & np.uint64(0xFFFF)) ^ np.uint64(0x8000)
    hi = (h >> np.uint64(16)) ^ np.uint64(0x8000)
    d = np.empty(h.shape[:-1] + (2 * h.shape[-1],), np.int8)
    d[..., 0::2] = lo < t
    d[..., 1::2] = hi < t
    return d


def corr(a, b):
    a = a.astype(np.float64).ravel()
    b = b.astype(np.float64).ravel()
    a -= a.mean()
    b -= b.mean()
    r = (a * b).mean() / np.sqrt((a * a).mean() * (b * b).mean())
    return r * np.sqrt(a.size)   # z-score under independence


def chi2_bytes(v):
    c = np.bincount(v.ravel().astype(np.int64), minlength=256).astype(np.float64)
    e = c.sum() / 256
    return ((c - e) ** 2 / e).sum()


def screen(name, fn, Q, J, heads, rng):
    out = {"rate": [], "chi2": [], "pair": [], "nbr": {}, "rect": []}
    for hh in range(heads):
        hm = head_mix(0x1234_5678_9ABC + 17 * hh, 3 + hh, 5 * hh + 1)
        h = fn(hm, np.arange(Q, dtype=np.uint64), np.arange(J, dtype=np.uint64))
        for sh, mask in ((0, 0xFF), (8, 0xFF), (16, 0xFF), (24, 0xFF)):
            out["chi2"].append(chi2_bytes((h >> np.uint64(sh)) & np.uint64(mask)))
        for p in (0.1, 0.3):
            d = drops(h, p)
            n = d.size
            out["rate"].append((d.mean() - p) / np.sqrt(p * (1 - p) / n))
            out["pair"].append(corr(d[:, 0::2], d[:, 1::2]))
            for k in (1, 2, 4, 64):
                out["nbr"].setdefault(f"k{k}", []).append(corr(d[:, :-k], d[:, k:]))
            for qd in (1, 32):
                out["nbr"].setdefault(f"q{qd}", []).append(corr(d[:-qd], d[qd:]))
            # rectangles: random query pairs x random key pairs
            R = 2_000_000
            q1, q2 = rng.integers(0, Q, R), rng.integers(0, Q, R)
            k1, k2 = rng.integers(0, 2 * J, R), rng.integers(0, 2 * J, R)
            ok = (q1 != q2) & (k1 != k2)
            q1, q2, k1, k2 = q1[ok], q2[ok], k1[ok], k2[ok]
            z = ((d[q1, k1] - p) * (d[q1, k2] - p) * (d[q2, k1] - p) * (d[q2, k2] - p)).astype(np.float64)
            out["rect"].append(z.mean() / (z.std() / np.sqrt(z.size)))
    worst = lambda xs: max(abs(x) for x in xs)
    nb = " ".join(f"{k}={worst(v):.1f}" for k, v in out["nbr"].items())
    print(f"{name:18s} rate|z|<={worst(out['rate']):.1f}  chi2 {min(out['chi2']):.0f}-{max(out['chi2']):.0f}"
          f"  pair|z|<={worst(out['pair']):.1f}  nbr|z| {nb}  rect|z|<={worst(out['rect']):.1f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=4096)
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--heads", type=int, default=4)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    for name, fn in CANDS.items():
        if a.only and name not in a.only.split(","):
            continue
        screen(name, fn, a.queries, a.pairs, a.heads, rng)


if __name__ == "__main__":
    main()
