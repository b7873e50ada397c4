"""Golden vectors for the Hungarian matcher: scipy.optimize.linear_sum_assignment
(the solver the reference calls at criterion.py:79) on batched (P, Q, G) float32
costs, sliced to the first nactual[p] columns exactly like the reference.

    python tests/golden/make_lsap_golden.py   ->  tests/golden/lsap.npz

Cases: matcher-like real costs, small-integer costs (dense ties), constant
costs, nactual >= Q (wide problems, not transposed by scipy), nactual = 0."""
import os

import numpy as np
from scipy.optimize import linear_sum_assignment

HERE = os.path.dirname(os.path.abspath(__file__))


def solve(cost, nact):
    P, Q, _ = cost.shape
    inds = np.zeros((P, Q), np.int64)
    mask = np.zeros((P, Q), np.float32)
    for p in range(P):
        if nact[p] > 0:
            r, c = linear_sum_assignment(cost[p, :, :nact[p]])
            inds[p, r] = c
            mask[p, r] = 1
    return inds, mask


def main():
    rng = np.random.default_rng(2024)
    out = {}
    cases = {
        # 8 decoder layers x B=8, Q=128, G=64 slots, 1..10 GT (SUN-like)
        "real": (rng.standard_normal((64, 128, 64)) * 3, rng.integers(0, 11, 64)),
        "ties": (rng.integers(0, 3, (32, 128, 64)), rng.integers(1, 40, 32)),
        "const": (np.ones((4, 64, 64)), np.array([1, 7, 64, 33])),
        "wide": (rng.standard_normal((16, 32, 64)), rng.integers(20, 65, 16)),
        "wide_ties": (rng.integers(0, 2, (16, 32, 64)), rng.integers(20, 65, 16)),
        "scannet": (rng.standard_normal((8, 256, 64)) * 2, rng.integers(0, 65, 8)),
    }
    for name, (c, n) in cases.items():
        c = c.astype(np.float32)
        n = n.astype(np.int32)
        c *= np.arange(c.shape[2])[None, None, :] < n[:, None, None]   # unused slots -> 0

        inds, mask = solve(c, n)
        out[f"{name}_cost"], out[f"{name}_nact"] = c, n
        out[f"{name}_inds"], out[f"{name}_mask"] = inds, mask
    np.savez_compressed(os.path.join(HERE, "lsap.npz"), **out)


if __name__ == "__main__":
    main()
