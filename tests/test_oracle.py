"""Pin the CPU oracle (oracle/ov3d_oracle.c) against the reference's own outputs
(golden fixtures made by tests/golden/make_golden.py from /root/reference) and,
for the un-vendored pointnet2 kernels, against a literal Python emulation of the
upstream CUDA kernels' control flow."""
import math

import numpy as np
import pytest

from helpers import fixture
from oracle import oracle as O


# ------------------------------------------------------------------ GIoU
@pytest.mark.parametrize("tag", ["rot", "aligned"])
@pytest.mark.parametrize("rflag", ["r", "a"])
def test_giou_cython_path_matches_reference(tag, rflag):
    fx = fixture("giou.npz")
    got = O.giou3d(fx[f"{tag}_c1"], fx[f"{tag}_c2"], fx[f"{tag}_nums"], mode=O.GIOU_MODE_CYTHON,
                   rotated=(rflag == "r"), k2_bug=True)
    ref = fx[f"{tag}_{rflag}_cython"]
    # a few ulp: torch-CPU sqrt is not correctly rounded in rare near-tie cases
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-6)


@pytest.mark.parametrize("tag", ["rot", "aligned"])
@pytest.mark.parametrize("rflag", ["r", "a"])
def test_giou_tensor_path_matches_reference(tag, rflag):
    fx = fixture("giou.npz")
    got = O.giou3d(fx[f"{tag}_c1"], fx[f"{tag}_c2"], fx[f"{tag}_nums"], mode=O.GIOU_MODE_TENSOR,
                   rotated=(rflag == "r"))
    np.testing.assert_allclose(got, fx[f"{tag}_{rflag}_tensor"], rtol=0, atol=2e-6)


def test_giou_k2_bug_is_the_only_mode_difference():
    """Q1: Cython and TorchScript paths agree for k2 < 4 and differ only beyond it."""
    fx = fixture("giou.npz")
    cy, ts = fx["rot_r_cython"], fx["rot_r_tensor"]
    np.testing.assert_allclose(cy[:, :, :4], ts[:, :, :4], atol=2e-6)
    assert np.abs(cy[:, :, 4:] - ts[:, :, 4:]).max() > 0.05
    nobug = O.giou3d(fx["rot_c1"], fx["rot_c2"], fx["rot_nums"], mode=O.GIOU_MODE_CYTHON,
                     rotated=True, k2_bug=False)
    np.testing.assert_allclose(nobug, ts, atol=2e-6)


# ------------------------------------------------------------------- NMS
@pytest.mark.parametrize("i", [0, 1, 2])
@pytest.mark.parametrize("old", [0, 1])
def test_nms_matches_reference(i, old):
    fx = fixture("nms.npz")
    boxes = fx[f"boxes{i}"]
    picks, keep = O.nms3d(boxes, 0.25, old_type=bool(old), samecls=True)
    assert picks == fx[f"samecls{i}_{old}"].tolist()
    assert keep.sum() == len(picks)
    picks, _ = O.nms3d(boxes[:, :7], 0.25, old_type=bool(old), samecls=False)
    assert picks == fx[f"any{i}_{old}"].tolist()


def _nms_stable_reference(boxes, thr):
    """utils/nms.py:120-162 with np.argsort(kind='stable') (the documented tie rule)."""
    x1, y1, z1, x2, y2, z2, score, cls = boxes.T
    area = (x2 - x1) * (y2 - y1) * (z2 - z1)
    I = np.argsort(score, kind="stable")
    pick = []
    while I.size:
        last = I.size
        i = I[-1]
        pick.append(int(i))
        r = I[: last - 1]
        l = np.maximum(0, np.minimum(x2[i], x2[r]) - np.maximum(x1[i], x1[r]))
        w = np.maximum(0, np.minimum(y2[i], y2[r]) - np.maximum(y1[i], y1[r]))
        h = np.maximum(0, np.minimum(z2[i], z2[r]) - np.maximum(z1[i], z1[r]))
        inter = l * w * h
        o = inter / (area[i] + area[r] - inter) * (cls[i] == cls[r])
        I = np.delete(I, np.concatenate(([last - 1], np.where(o > thr)[0])))
    return pick


def test_nms_tie_rule_is_stable_argsort():
    rs = np.random.RandomState(3)
    K = 64
    lo = rs.uniform(-1, 1, (K, 3))
    boxes = np.concatenate([lo, lo + rs.uniform(0.3, 1.0, (K, 3)),
                            rs.randint(0, 5, (K, 1)) / 4.0, rs.randint(0, 2, (K, 1))], 1)
    picks, _ = O.nms3d(boxes, 0.25)
    assert picks == _nms_stable_reference(boxes, 0.25)


# ------------------------------------------------------------------- FPS
def _upstream_fps(xyz, M):
    """Literal emulation of the upstream furthest_point_sampling_kernel: block = largest
    power of two <= N (cap 512), thread t scans k = t, t+bs, ... keeping the first max,
    then the halving tree reduction that keeps the lower slot on ties.  Integer-valued
    coordinates keep every distance exact, so fma/no-fma does not matter here."""
    N = len(xyz)
    bs = 1
    while bs * 2 <= N and bs < 512:
        bs *= 2
    p = xyz.astype(np.float64)
    temp = np.full(N, 1e10)
    skip = (p * p).sum(1) <= 1e-3
    old, out = 0, [0]
    for _ in range(1, M):
        d = ((p - p[old]) ** 2).sum(1)
        vals = np.full(bs, -1.0)
        inds = np.zeros(bs, dtype=np.int64)
        for t in range(bs):
            best, besti = -1.0, 0
            for k in range(t, N, bs):
                if skip[k]:
                    continue
                d2 = min(d[k], temp[k])
                temp[k] = d2
                if d2 > best:
                    best, besti = d2, k
            vals[t], inds[t] = best, besti
        s = bs // 2
        while s >= 1:
            for t in range(s):
                v1, v2 = vals[t], vals[t + s]
                i1, i2 = inds[t], inds[t + s]
                vals[t] = max(v1, v2)
                inds[t] = i2 if v2 > v1 else i1
            s //= 2
        old = int(inds[0])
        out.append(old)
    return np.array(out, dtype=np.int32)


@pytest.mark.parametrize("N,M", [(600, 40), (300, 30), (37, 12), (1, 3), (5, 9)])
def test_fps_tie_rule_matches_upstream_tree_reduction(N, M):
    rs = np.random.RandomState(N)
    xyz = rs.randint(-3, 4, size=(N, 3)).astype(np.float32)   # many exact ties + origin points
    xyz[rs.choice(N, size=max(1, N // 10), replace=False)] = 0.0
    got = O.fps(xyz[None], M)[0]
    np.testing.assert_array_equal(got, _upstream_fps(xyz, M))


def test_fps_basic_properties():
    rs = np.random.RandomState(0)
    xyz = rs.uniform(-2, 2, (3, 1000, 3)).astype(np.float32)
    idx = O.fps(xyz, 64)
    assert (idx[:, 0] == 0).all()
    for b in range(3):
        assert len(set(idx[b].tolist())) == 64
        # furthest property: each new point is at max min-distance from the chosen set
        chosen = xyz[b, idx[b, :10]]
        d = ((xyz[b][:, None] - chosen[None]) ** 2).sum(-1).min(1)
        nxt = xyz[b, idx[b, 10]]
        dn = ((chosen - nxt) ** 2).sum(-1).min()
        assert dn >= d.max() * (1 - 1e-5)


def test_fps_rank_orders_ties_like_the_tree():
    # thread t = k mod 512 wins ties in bit-reversed order: 0 < 256 < 128 < 384 < 64 ...
    ranks = [O.fps_rank(k, 100000) for k in (0, 256, 128, 384, 64, 320, 1)]
    assert ranks == sorted(ranks) and len(set(ranks)) == len(ranks)
    # same thread, next stride: k = 512 is thread 0's second point, before thread 256's first
    assert O.fps_rank(0, 100000) < O.fps_rank(512, 100000) < O.fps_rank(256, 100000)


# ------------------------------------------------------------ ball query
def test_ball_query_matches_brute_force():
    rs = np.random.RandomState(1)
    xyz = rs.uniform(0, 1, (2, 500, 3)).astype(np.float32)
    cen = xyz[:, :40].copy()
    cen[1, 5] = 50.0  # no neighbour -> all zeros
    idx = O.ball_query(xyz, cen, 0.15, 16)
    for b in range(2):
        for j in range(40):
            d2 = ((xyz[b].astype(np.float64) - cen[b, j]) ** 2).sum(1)
            hits = np.nonzero(d2 < np.float32(0.15) ** 2)[0][:16]
            exp = np.zeros(16, np.int64)
            if len(hits):
                exp[:] = hits[0]
                exp[: len(hits)] = hits
            np.testing.assert_array_equal(idx[b, j], exp)


def test_group_gathers_columns():
    rs = np.random.RandomState(2)
    f = rs.randn(2, 5, 30).astype(np.float32)
    idx = rs.randint(0, 30, (2, 7, 4)).astype(np.int32)
    out = O.group(f, idx)
    for b in range(2):
        np.testing.assert_array_equal(out[b], f[b][:, idx[b]])


def test_math_constants():
    assert math.isclose(float(np.float32(0.2) * np.float32(0.2)), 0.04000000357627869, rel_tol=1e-7)


# ------------------------------------------------------------------ Hungarian
LSAP_CASES = ["real", "ties", "const", "wide", "wide_ties", "scannet"]


def _lsap_batch(cost, nact):
    P, Q, _ = cost.shape
    inds = np.zeros((P, Q), np.int64)
    mask = np.zeros((P, Q), np.float32)
    for p in range(P):
        if nact[p] > 0:
            g = O.lsap(cost[p, :, :nact[p]])
            inds[p, g >= 0] = g[g >= 0]
            mask[p, g >= 0] = 1
    return inds, mask


@pytest.mark.parametrize("case", LSAP_CASES)
def test_lsap_matches_scipy_golden(case):
    """oracle LSAP == scipy.optimize.linear_sum_assignment (criterion.py:79) incl. ties."""
    fx = fixture("lsap.npz")
    inds, mask = _lsap_batch(fx[f"{case}_cost"], fx[f"{case}_nact"])
    np.testing.assert_array_equal(mask, fx[f"{case}_mask"])
    np.testing.assert_array_equal(inds, fx[f"{case}_inds"])


def test_lsap_matches_scipy_random_shapes():
    scipy_opt = pytest.importorskip("scipy.optimize")
    rng = np.random.default_rng(5)
    for it in range(600):
        nq, ng = int(rng.integers(1, 60)), int(rng.integers(1, 60))
        c = (rng.integers(0, 3, (nq, ng)) if it % 2 else rng.standard_normal((nq, ng))).astype(np.float32)
        r, col = scipy_opt.linear_sum_assignment(c)
        ref = np.full(nq, -1)
        ref[r] = col
        np.testing.assert_array_equal(O.lsap(c), ref)


def test_lsap_rejects_invalid_entries():
    c = np.zeros((3, 2), np.float32)
    c[1, 1] = np.nan
    with pytest.raises(ValueError):
        O.lsap(c)


def test_bench_ball_query_scanned_count_matches_the_reference_scan():
    """bench.py's ball-query byte count (the points the reference scan actually
    reads) from the oracle's indices equals a direct simulation of the Appendix A.2 scan
    (stop after the S-th strict d^2 < r^2 hit, else N), incl. centroids with no / few hits"""
    import torch
    import bench
    rng = np.random.default_rng(4)
    B, N, M, S, r = 2, 700, 40, 8, 0.2
    xyz = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    new = xyz[:, rng.choice(N, M, replace=False)].copy()
    new[0, 0] = (5.0, 5.0, 5.0)         # no neighbour: scans all N
    new[1, 1] = xyz[1, -1] + 0.01         # few neighbours near the end
    idx = O.ball_query(xyz, new, r, S)
    want = 0
    r2 = np.float32(r) * np.float32(r)
    for b in range(B):
        for m in range(M):
            d = xyz[b] - new[b, m]
            d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
            hits = np.nonzero(d2 < r2)[0]
            want += hits[S - 1] + 1 if len(hits) >= S else N
    assert bench.ball_query_scanned(torch.from_numpy(idx), N) == want
