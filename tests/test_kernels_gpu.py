"""HIP kernels (libov3d_hip.so, called through the C ABI via the product
wrappers) against the CPU oracle: bit-exact for indices / integer outputs /
the no-contraction float kernels, and against the reference fixtures."""
import numpy as np
import pytest
import torch

from helpers import fixture, ov3d
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def scene_batch(B, N, seed, uniform=False):
    from ov3d_amd import synthetic
    return synthetic.make_batch(B, seed=seed, num_points=N, uniform_volume=uniform)["point_clouds"]


# ------------------------------------------------------------------- FPS
@pytest.mark.parametrize("B,N,M", [(8, 20000, 2048), (8, 2048, 128), (2, 40000, 1024),
                                   (3, 2048, 1024), (2, 1000, 64), (4, 300, 17), (2, 37, 37),
                                   (1, 1, 4), (2, 20480, 8), (2, 20481, 8), (1, 40960, 512),
                                   (1, 40961, 64), (8, 40000, 2048), (3, 30000, 700),
                                   (2, 20482, 2048)])
def test_fps_bit_exact(cuda, B, N, M):
    from ov3d_amd import pointnet2_utils as pu
    xyz = scene_batch(B, N, seed=N + M) if N >= 64 else torch.rand(B, N, 3)
    ref = O.fps(xyz.numpy(), M)
    xg = xyz.to(cuda)
    idx = pu.furthest_point_sample(xg, M)
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
    idx2, new_xyz = pu.furthest_point_sample_gather(xg, M)
    np.testing.assert_array_equal(idx2.cpu().numpy(), ref)
    np.testing.assert_array_equal(new_xyz.cpu().numpy(),
                                  np.take_along_axis(xyz.numpy(), ref[..., None].astype(np.int64), 1))


@pytest.mark.parametrize("B,N,M", [(3, 30000, 700), (8, 40000, 512), (5, 25000, 300)])
def test_fps_two_workgroup_halves_repeated(cuda, B, N, M):
    """The two-workgroup kernel (20480 < N <= 40960) repeated on one input: both halves must
    own complementary point sets in EVERY run.  Round 3 found the halves each sorting the scene
    with LDS atomics, whose order inside a Morton cell differs between workgroups: now and then
    a boundary-cell point belonged to neither half (scene 2 of this (3, 30000, 700) input lost
    sample 209 in 8 of 40 runs; tools/fps_pair_stress.py).  Half 0 now publishes its order."""
    from ov3d_amd import pointnet2_utils as pu
    g = np.random.default_rng(B * N + M)
    xyz = g.uniform(-3, 3, (B, N, 3)).astype(np.float32)
    ref = O.fps(xyz, M)
    xg = torch.from_numpy(xyz).to(cuda)
    for _ in range(12):
        idx = pu.furthest_point_sample(xg, M)
        np.testing.assert_array_equal(idx.cpu().numpy(), ref)


def test_fps_two_workgroup_lost_partner_is_an_error(cuda, monkeypatch):
    """A partner workgroup that never answers (OV3D_FPS_PAIR_SILENT=1: half 1 returns at once;
    a small OV3D_FPS_PAIR_SPIN so half 0 gives up in milliseconds): the indices are wrong, so
    the reference API raises, the fused gather returns NaN coordinates (a captured step's loss
    turns NaN) and ov3d_fps_pair_status reports every scene.  Without the hook: all zeros."""
    from ov3d_amd import pointnet2_utils as pu
    B, N, M = 2, 30000, 64
    xg = torch.from_numpy(np.random.default_rng(5).uniform(-3, 3, (B, N, 3)).astype(np.float32)).to(cuda)
    ref = O.fps(xg.cpu().numpy(), M)
    monkeypatch.setenv("OV3D_FPS_PAIR_SPIN", "2000")
    monkeypatch.setenv("OV3D_FPS_PAIR_SILENT", "1")
    with pytest.raises(pu.FPSPairLost):
        pu.furthest_point_sample(xg, M)
    _, nx = pu.furthest_point_sample_gather(xg, M)
    assert torch.isnan(nx).all()
    with pytest.raises(pu.FPSPairLost):
        pu.furthest_point_sample_gather(xg, M, check=True)
    monkeypatch.delenv("OV3D_FPS_PAIR_SILENT")
    monkeypatch.delenv("OV3D_FPS_PAIR_SPIN")
    idx, nx = pu.furthest_point_sample_gather(xg, M, check=True)
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
    assert torch.isfinite(nx).all()
    ws = pu._fps_workspace(B, N, cuda)
    from ov3d_amd import _native as nat
    out = torch.empty((B, M), dtype=torch.int32, device=cuda)
    nat.call("ov3d_fps", xg, B, N, M, out, None, ws, like=xg)
    assert pu.fps_pair_status(ws, B, N, M).cpu().tolist() == [0] * B


def test_fps_two_workgroup_range_beyond_coresidency(cuda):
    """B above CUs / 2 at 20480 < N <= 40960: the 2B workgroups of the pair kernel cannot all be
    resident (one per CU), so ov3d_fps takes the one-workgroup two-cluster kernel; indices equal
    the oracle's, status all zero (the pair kernel used to be chosen regardless)."""
    from ov3d_amd import pointnet2_utils as pu
    cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    B, N, M = cus // 2 + 8, 24000, 32
    xyz = np.random.default_rng(9).uniform(-3, 3, (B, N, 3)).astype(np.float32)
    ref = O.fps(xyz, M)
    idx, nx = pu.furthest_point_sample_gather(torch.from_numpy(xyz).to(cuda), M, check=True)
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)


@pytest.mark.parametrize("N", [700, 5000, 30000])
def test_fps_ties_and_skipped_points(cuda, N):
    """integer grid -> exact distance ties; origin points -> the |p|^2 <= 1e-3 skip."""
    from ov3d_amd import pointnet2_utils as pu
    rs = np.random.RandomState(N)
    xyz = rs.randint(-4, 5, size=(2, N, 3)).astype(np.float32)
    xyz[:, rs.choice(N, N // 8, replace=False)] = 0.0
    xyz[:, 7] = 1e-2  # |p|^2 = 3e-4 <= 1e-3 -> never selected
    ref = O.fps(xyz, 200)
    got = pu.furthest_point_sample(torch.from_numpy(xyz).to(cuda), 200).cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    assert not (got[:, 1:] == 7).any()


# ------------------------------------------------------------ ball query
@pytest.mark.parametrize("B,N,M,r,S,uniform", [(8, 20000, 2048, 0.2, 64, False),
                                               (8, 20000, 2048, 0.2, 64, True),
                                               (4, 2048, 1024, 0.4, 32, False),
                                               (2, 1001, 100, 0.3, 16, False),
                                               (3, 1000, 99, 0.3, 16, False),   # one per wave
                                               (8, 40000, 1024, 0.4, 32, True),
                                               (8, 40000, 2048, 0.2, 64, False),  # C4 pre-encoder
                                               (2, 500, 64, 0.05, 8, True)])
def test_ball_query_bit_exact(cuda, B, N, M, r, S, uniform):
    from ov3d_amd import pointnet2_utils as pu
    xyz = scene_batch(B, N, seed=3 * N + M, uniform=uniform)
    xn = xyz.numpy()
    cen = xn[:, np.random.RandomState(1).choice(N, M, replace=False)].copy()
    cen[:, 0] += 100.0  # one centroid with no neighbour at all
    ref = O.ball_query(xn, cen, r, S)
    got = pu.ball_query(r, S, xyz.to(cuda), torch.from_numpy(cen).to(cuda)).cpu().numpy()
    np.testing.assert_array_equal(got, ref)


def _bq_case(name, rs):
    """(xyz (B,N,3), centroids (B,M,3), r, S) for the cell-index edge cases"""
    B, N, M = 3, 9000, 257   # N >= 8192: the cell path (kBQCellsMinN)
    xyz = rs.uniform(-2.0, 2.0, (B, N, 3)).astype(np.float32)
    r, S = 0.2, 64
    if name == "dense_cluster":      # > 1024 hits in one centroid's runs: the scan fallback
        xyz[:, :3000] = rs.uniform(0.0, 0.05, (B, 3000, 3))
    elif name == "mid_density":      # 65 .. 1024 hits: bisection for the S-th smallest index
        xyz = rs.uniform(0.0, 1.0, (B, N, 3)).astype(np.float32)
    elif name == "wide_extent":      # one scene 400 m wide: cells far larger than r
        xyz[1, :10] *= 100.0
    elif name == "nonfinite":        # NaN / inf points never hit; NaN centroid: no hit
        xyz[:, 5] = np.nan
        xyz[:, 6] = np.inf
        xyz[:, 7, 1] = -np.inf
    elif name == "huge_radius":      # every point a candidate
        r = 50.0
    elif name == "zero_radius":
        r = 0.0
    elif name == "negative_radius":  # the reference squares it
        r = -0.3
    elif name == "one_point_scene":  # zero extent
        xyz[:] = 0.5
    elif name == "S_above_64":       # the index-order scan
        S = 100
    elif name == "S_1":
        S = 1
    elif name == "boundary":         # lattice of spacing r: neighbours at d2 ~ r^2 (rounding edge)
        xyz = (rs.randint(-5, 6, (B, N, 3)) * np.float32(0.2)).astype(np.float32)
    cen = xyz[:, rs.choice(N, M, replace=False)].copy()
    cen[:, 0] += 100.0               # no neighbour at all
    cen[:, 1] = xyz[:, 0] + np.float32(abs(r) * 0.999)   # just inside / outside the sphere
    cen[:, 2] = np.nan if name == "nonfinite" else cen[:, 2]
    cen[:, 3] = -100.0               # far outside the grid on the low side
    return xyz, cen, r, S


@pytest.mark.parametrize("name", ["dense_cluster", "mid_density", "wide_extent", "nonfinite",
                                  "huge_radius", "zero_radius", "negative_radius",
                                  "one_point_scene", "S_above_64", "S_1", "boundary"])
def test_ball_query_cells_edge_cases(cuda, name):
    """ov3d_ball_query_cells (the product's ball query: a per-scene cell index, 27 cells per
    centroid, the S smallest hit indices) equals the index-order scan of the oracle on the
    inputs that stress it: more hits than the wave keeps (scan fallback), the bisection path,
    cells far wider than r, non-finite points and centroids, radii 0 / negative / larger than the
    scene, a zero-extent scene, S > 64, points on cell boundaries"""
    from ov3d_amd import pointnet2_utils as pu
    xyz, cen, r, S = _bq_case(name, np.random.RandomState(7))
    ref = O.ball_query(xyz, cen, r, S)
    got = pu.ball_query(r, S, torch.from_numpy(xyz).to(cuda), torch.from_numpy(cen).to(cuda))
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_ball_query_cells_equals_scan_at_full_size(cuda):
    """size-independent check at N = 65535 (the largest the 16-bit cell counters take) and the
    fallback above it: cells == the scan entry point ov3d_ball_query"""
    from ov3d_amd import _native as nat, pointnet2_utils as pu
    for N in (65535, 65536):
        xyz = scene_batch(2, N, seed=N)
        xg = xyz.to(cuda)
        cen = xg[:, ::N // 1024][:, :1024].contiguous()
        got = pu.ball_query(0.2, 64, xg, cen)
        scan = torch.empty_like(got)
        nat.call("ov3d_ball_query", xg, cen, 2, N, 1024, 0.2, 64, scan, like=xg)
        assert torch.equal(got, scan)


# -------------------------------------------------------------- grouping
@pytest.mark.parametrize("C", [0, 3, 256])
@pytest.mark.parametrize("gather_bwd", [True, False])
def test_group_fwd_bwd(cuda, C, gather_bwd, monkeypatch):
    from ov3d_amd import pointnet2_utils as pu
    monkeypatch.setattr(pu, "GATHER_BWD", gather_bwd)   # inverse-index backward vs atomics
    B, N, M, S, r = 2, 2048, 256, 32, 0.4
    xyz = scene_batch(B, N, seed=11)
    new_xyz = xyz[:, :M].clone()
    feats = torch.randn(B, C, N) if C else None
    grouper = pu.QueryAndGroup(r, S, use_xyz=True, ret_grouped_xyz=True, normalize_xyz=True)
    fg = feats.to(cuda).requires_grad_(True) if C else None
    out, gxyz = grouper(xyz.to(cuda), new_xyz.to(cuda), fg)
    idx = O.ball_query(xyz.numpy(), new_xyz.numpy(), r, S)
    exp_xyz = (O.group(xyz.transpose(1, 2).contiguous().numpy(), idx) - new_xyz.transpose(1, 2).numpy()[..., None]) / np.float32(r)
    np.testing.assert_array_equal(out[:, :3].detach().cpu().numpy(), exp_xyz.astype(np.float32))
    if C:
        np.testing.assert_array_equal(out[:, 3:].detach().cpu().numpy(), O.group(feats.numpy(), idx))
        g = torch.randn_like(out)
        out.backward(g)
        ref = torch.zeros(B, C, N, dtype=torch.float64)
        gi = torch.from_numpy(idx).long().view(B, 1, M * S).expand(B, C, M * S)
        ref.scatter_add_(2, gi, g[:, 3:].double().cpu().reshape(B, C, M * S))
        np.testing.assert_allclose(fg.grad.cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)


def test_group_inverse_index(cuda):
    """ov3d_group_inverse: every row appears exactly once, in the list of the point it reads,
    each list ascending (the fill's atomics order is undone: the gather-form backward's fp32
    sums are then identical in every run) -- i.e. exactly a stable argsort by point"""
    from ov3d_amd import pointnet2_utils as pu
    B, N, M, S = 3, 500, 128, 16
    idx = torch.randint(0, N, (B, M, S), device=cuda, dtype=torch.int32)
    idx[1] = 7          # one point read by every row of a scene: a 2048-entry list
    idx[2, :20] = 9     # a ~330-entry list (the wave rank sort's LDS path)
    off, rows = pu.group_inverse(idx, N)
    off, rows, idx = off.cpu().numpy(), rows.cpu().numpy(), idx.cpu().numpy().reshape(-1)
    assert off[0] == 0 and off[-1] == B * M * S and np.all(np.diff(off) >= 0)
    assert np.array_equal(np.sort(rows), np.arange(B * M * S))
    for bn in range(B * N):
        r = rows[off[bn]:off[bn + 1]]
        assert np.all(idx[r] == bn % N) and np.all(r // (M * S) == bn // N)
    key = np.repeat(np.arange(B), M * S) * N + idx
    np.testing.assert_array_equal(rows, np.argsort(key, kind="stable"))
    off2, rows2 = pu.group_inverse(torch.from_numpy(idx.reshape(B, M, S)).to(cuda), N)
    np.testing.assert_array_equal(rows2.cpu().numpy(), rows)


def test_gather_fwd_bwd(cuda):
    from ov3d_amd import pointnet2_utils as pu
    f = torch.randn(2, 5, 300, device=cuda, requires_grad=True)
    idx = torch.randint(0, 300, (2, 40), device=cuda, dtype=torch.int32)
    out = pu.gather_operation(f, idx)
    ref = torch.gather(f.detach(), 2, idx.long()[:, None].expand(2, 5, 40))
    assert torch.equal(out.detach(), ref)
    g = torch.randn_like(out)
    out.backward(g)
    exp = torch.zeros(2, 5, 300, device=cuda).scatter_add_(2, idx.long()[:, None].expand(2, 5, 40), g)
    torch.testing.assert_close(f.grad, exp)


def test_gather_matches_cpu_twin_bit_exact(cuda):
    """ov3d_gather_fwd / _bwd against the boundary's CPU twins (ov3d_gather_fwd_cpu / _bwd_cpu):
    bit-exact on FPS-style distinct indices (no summation-order freedom in the backward)"""
    from ov3d_amd import pointnet2_utils as pu
    g = torch.Generator(device="cpu").manual_seed(12)
    B, C, N, M = 3, 7, 5000, 512
    f = torch.randn((B, C, N), generator=g)
    idx = torch.stack([torch.randperm(N, generator=g)[:M] for _ in range(B)]).int()
    gout = torch.randn((B, C, M), generator=g)
    fd = f.to(cuda).requires_grad_()
    out = pu.gather_operation(fd, idx.to(cuda))
    out.backward(gout.to(cuda))
    assert np.array_equal(out.detach().cpu().numpy(), O.gather(f.numpy(), idx.numpy()))
    assert np.array_equal(fd.grad.cpu().numpy(), O.gather_bwd(gout.numpy(), idx.numpy(), N))


# ------------------------------------------------------------------ GIoU
@pytest.mark.parametrize("tag", ["rot", "aligned"])
@pytest.mark.parametrize("rflag", [True, False])
@pytest.mark.parametrize("mode", [0, 1])
def test_giou_vs_oracle_and_reference(cuda, tag, rflag, mode):
    from ov3d_amd.box_util import giou3d_raw
    fx = fixture("giou.npz")
    c1, c2, nums = fx[f"{tag}_c1"], fx[f"{tag}_c2"], fx[f"{tag}_nums"]
    got = giou3d_raw(torch.from_numpy(c1).to(cuda), torch.from_numpy(c2).to(cuda),
                     torch.from_numpy(nums).to(cuda), mode, rflag).cpu().numpy()
    np.testing.assert_array_equal(got, O.giou3d(c1, c2, nums, mode=mode, rotated=rflag))
    ref = fx[f"{tag}_{'r' if rflag else 'a'}_{'cython' if mode == 0 else 'tensor'}"]
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-6)


def test_giou_large_batch_vs_oracle(cuda):
    """BASELINE shapes: 8 decoder layers x B=8, 128 predictions x 64 GT slots."""
    from ov3d_amd.box_util import generalized_box3d_iou
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    cfg = SunrgbdDatasetConfig()
    g = torch.Generator().manual_seed(0)
    P, Q, G = 64, 128, 64
    def boxes(n):
        c = torch.rand(P, n, 3, generator=g) * torch.tensor([4.0, 4.0, 2.0]) - torch.tensor([2.0, -1.0, 0.5])
        s = torch.rand(P, n, 3, generator=g) * 1.7 + 0.3
        a = torch.rand(P, n, generator=g) * 6.28 - 3.14
        return cfg.box_parametrization_to_corners(c, s, a)
    c1, c2 = boxes(Q), boxes(G)
    nums = torch.randint(1, 11, (P,), generator=g)
    got = generalized_box3d_iou(c1.to(cuda), c2.to(cuda), nums.to(cuda)).cpu().numpy()
    np.testing.assert_array_equal(got, O.giou3d(c1.numpy(), c2.numpy(), nums.numpy()))


def test_giou_backward_matches_reference_autograd(cuda):
    from ov3d_amd.box_util import generalized_box3d_iou
    fx = fixture("giou.npz")
    c1 = torch.from_numpy(fx["grad_c1"]).to(cuda).requires_grad_(True)
    g = generalized_box3d_iou(c1, torch.from_numpy(fx["grad_c2"]).to(cuda),
                              torch.from_numpy(fx["grad_nums"]).to(cuda), rotated_boxes=False,
                              needs_grad=True)
    np.testing.assert_allclose(g.detach().cpu().numpy(), fx["grad_giou"], atol=2e-6)
    (g * torch.from_numpy(fx["grad_G"]).to(cuda)).sum().backward()
    np.testing.assert_allclose(c1.grad.cpu().numpy(), fx["grad_dc1"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("flag", ["host", "device"])
def test_rotated_giou_backward_matches_reference_autograd(cuda, flag):
    """d(sum(G * giou))/dcorners1 through the rotated Sutherland-Hodgman clip (the reference's
    TorchScript autograd, box_util.py:387-440, 579-600), rotated given on the host or as the
    criterion's device flag"""
    from ov3d_amd.box_util import generalized_box3d_iou
    fx = fixture("giou.npz")
    c1 = torch.from_numpy(fx["rgrad_c1"]).to(cuda).requires_grad_(True)
    rot = True if flag == "host" else torch.ones((), dtype=torch.int32, device=cuda)
    g = generalized_box3d_iou(c1, torch.from_numpy(fx["rgrad_c2"]).to(cuda),
                              torch.from_numpy(fx["rgrad_nums"]).to(cuda), rotated_boxes=rot,
                              needs_grad=True)
    np.testing.assert_allclose(g.detach().cpu().numpy(), fx["rgrad_giou"], atol=2e-6)
    (g * torch.from_numpy(fx["rgrad_G"]).to(cuda)).sum().backward()
    ref = fx["rgrad_dc1"]
    assert np.abs(ref).max() > 0.1             # the clip's gradient is exercised
    np.testing.assert_allclose(c1.grad.cpu().numpy(), ref, rtol=1e-4, atol=2e-5)


# ------------------------------------------------------------------- NMS
@pytest.mark.parametrize("i", [0, 1, 2])
@pytest.mark.parametrize("old", [False, True])
def test_nms_matches_reference(cuda, i, old):
    from ov3d_amd import nms
    fx = fixture("nms.npz")
    boxes = fx[f"boxes{i}"]
    assert nms.nms_3d_faster_samecls(boxes, 0.25, old) == fx[f"samecls{i}_{int(old)}"].tolist()
    assert nms.nms_3d_faster(boxes[:, :7], 0.25, old) == fx[f"any{i}_{int(old)}"].tolist()


def test_nms_batched_vs_oracle_with_ties_and_valid_mask(cuda):
    from ov3d_amd import nms
    rs = np.random.RandomState(9)
    B, K = 8, 256
    lo = rs.uniform(-2, 2, (B, K, 3))
    boxes = np.concatenate([lo, lo + rs.uniform(0.3, 1.5, (B, K, 3)),
                            rs.randint(0, 6, (B, K, 1)) / 5.0, rs.randint(0, 3, (B, K, 1))], 2)
    valid = rs.rand(B, K) > 0.2
    keep = nms.nms3d_batched(torch.from_numpy(boxes).to(cuda), 0.25,
                             valid=torch.from_numpy(valid).to(cuda)).cpu().numpy()
    for b in range(B):
        sub = np.nonzero(valid[b])[0]
        _, k = O.nms3d(boxes[b, sub], 0.25)
        exp = np.zeros(K, np.uint8)
        exp[sub] = k
        np.testing.assert_array_equal(keep[b], exp)


def test_nms_boxes_from_corners(cuda):
    from ov3d_amd import nms
    corners = torch.randn(2, 16, 8, 3, device=cuda)
    obj = torch.rand(2, 16, device=cuda)
    cls = torch.randint(0, 5, (2, 16), device=cuda)
    t = nms.nms_boxes_from_corners(corners, obj, cls)
    c64 = corners.double()
    exp = torch.cat([c64.min(2).values, c64.max(2).values, obj.double()[..., None], cls.double()[..., None]], -1)
    assert torch.equal(t, exp)


# ------------------------------------------------------------------ Hungarian
@pytest.mark.parametrize("case", ["real", "ties", "const", "wide", "wide_ties", "scannet"])
def test_hungarian_matches_scipy_golden(cuda, case):
    from ov3d_amd.assignment import hungarian
    fx = fixture("lsap.npz")
    cost = torch.from_numpy(fx[f"{case}_cost"]).to(cuda)
    nact = torch.from_numpy(fx[f"{case}_nact"]).to(cuda)
    inds, mask, status = hungarian(cost, nact)
    assert int(status.abs().sum()) == 0
    np.testing.assert_array_equal(mask.cpu().numpy(), fx[f"{case}_mask"])
    np.testing.assert_array_equal(inds.cpu().numpy(), fx[f"{case}_inds"])


@pytest.mark.parametrize("P,Q,G", [(96, 128, 64),    # costs staged in LDS (SUN shape)
                                   (16, 256, 64),    # global-cost path (C4 shape, > 64 KB)
                                   (24, 32, 48)])    # more GT than queries (transposed solve)
def test_hungarian_vs_oracle_random_ties(cuda, P, Q, G):
    from ov3d_amd.assignment import hungarian
    rng = np.random.default_rng(11)
    cost = rng.integers(0, 4, (P, Q, G)).astype(np.float32) * 0.5
    cost[: P // 2] = rng.standard_normal((P // 2, Q, G)).astype(np.float32)
    nact = rng.integers(0, G + 1, P).astype(np.int32)
    inds, mask, _ = hungarian(torch.from_numpy(cost).to(cuda), torch.from_numpy(nact).to(cuda))
    for p in range(P):
        exp = np.full(Q, -1)
        if nact[p]:
            exp = O.lsap(cost[p, :, :nact[p]])
        m = mask[p].cpu().numpy()
        np.testing.assert_array_equal(m, (exp >= 0).astype(np.float32))
        np.testing.assert_array_equal(inds[p].cpu().numpy(), np.where(exp >= 0, exp, 0))


def test_hungarian_invalid_cost_status(cuda):
    from ov3d_amd.assignment import check_status, hungarian
    cost = torch.zeros(3, 16, 8, device=cuda)
    cost[1, 3, 2] = float("nan")
    cost[2, 0, 7] = float("nan")          # outside nactual: ignored, as in the reference slice
    nact = torch.tensor([4, 4, 4], device=cuda, dtype=torch.int32)
    inds, mask, status = hungarian(cost, nact)
    assert status.tolist() == [0, -1, 0]
    assert mask[1].sum().item() == 0 and mask[0].sum().item() == 4
    with pytest.raises(ValueError, match="invalid numeric"):
        check_status(status)


def test_add_cast_bf16_equals_torch(cuda):
    """ov3d_add_cast_bf16: bf16(a + b) and bf16(a) bit for bit as torch.add into a bf16 output
    and .to(bfloat16) (transformer._MemoryKV's memory + pos / memory rows)."""
    from ov3d_amd import _native
    a = torch.randn(2048, 8, 256, device=cuda) * 3
    b = torch.randn(2048, 8, 256, device=cuda)
    s = torch.empty(a.shape, dtype=torch.bfloat16, device=cuda)
    c = torch.empty(a.shape, dtype=torch.bfloat16, device=cuda)
    _native.call("ov3d_add_cast_bf16", a, 0, b, a.numel(), s, c, like=a)
    ref = torch.empty(a.shape, dtype=torch.bfloat16, device=cuda)
    torch.add(a, b, out=ref)
    assert torch.equal(s, ref)
    assert torch.equal(c, a.to(torch.bfloat16))
    # bf16 memory (the step's encoder output), fp32 pos: the sum in fp32, rounded once (torch's
    # GPU add into a bf16 output rounds the fp32 operand to bf16 first: two roundings)
    ab = a.to(torch.bfloat16)
    _native.call("ov3d_add_cast_bf16", ab, 1, b, a.numel(), s, None, like=a)
    assert torch.equal(s, (ab.float() + b).to(torch.bfloat16))


@pytest.mark.parametrize("C,layout", [(256, "nbc"), (256, "bcn"), (20, "nbc"), (0, "nbc")])
def test_group_rows_bf16_bit_exact(cuda, C, layout):
    """ov3d_group_rows_bf16 (the interim SA's grouped rows: (xyz[idx] - centroid) / r, then the
    features, bf16, zero-padded to a multiple of 8 columns) against the same fp32 arithmetic in
    torch, every bit: channel-contiguous features of the encoder's (N, B, C) rows (three aligned
    16-byte loads per chunk), channel-strided (B, C, N) rows and C % 4 != 0 (per-element loads)"""
    from ov3d_amd import _native
    torch.manual_seed(8)
    B, N, M, S, r = 2, 1024, 128, 32, 0.4
    xyz = torch.rand(B, N, 3, device=cuda) * 2
    nxyz = xyz[:, :M].contiguous()
    idx = torch.randint(0, N, (B, M, S), device=cuda, dtype=torch.int32)
    if layout == "nbc":
        feats = torch.randn(N, B, max(C, 1), device=cuda)[..., :C].permute(1, 2, 0)   # (B, C, N) view
    else:
        feats = torch.randn(B, max(C, 1), N, device=cuda)[:, :C]
    cp = (3 + C + 7) // 8 * 8
    out = torch.empty((B, M, S, cp), dtype=torch.bfloat16, device=cuda)
    st = feats.stride()
    _native.call("ov3d_group_rows_bf16", xyz, nxyz, feats if C else None, st[0], st[2], st[1], idx,
                 B, C, N, M, S, r, 1, cp, out, like=xyz)
    il = idx.long()
    gx = torch.gather(xyz, 1, il.view(B, -1, 1).expand(-1, -1, 3)).view(B, M, S, 3)
    ref = torch.zeros((B, M, S, cp), device=cuda)
    ref[..., :3] = (gx - nxyz[:, :, None, :]) / r
    if C:
        ft = feats.transpose(1, 2)                                          # (B, N, C)
        ref[..., 3:3 + C] = torch.gather(ft, 1, il.view(B, -1, 1).expand(-1, -1, C)).view(B, M, S, C)
    assert torch.equal(out, ref.to(torch.bfloat16))


@pytest.mark.parametrize("C,ldg_kind", [(256, "cp"), (20, "cp"), (256, "odd"), (20, "odd")])
def test_group_bwd_csr_bf16_bit_exact(cuda, C, ldg_kind):
    """ov3d_group_bwd_csr_bf16 (the interim SA grouping's gather-form backward over bf16 row
    gradients) against a torch sum in the inverse's entry order, every bit: the 16-byte chunk
    kernel (ldg = cp, a multiple of 8) and the per-channel kernel (ldg = 3 + C, odd)"""
    from ov3d_amd import _native
    from ov3d_amd import pointnet2_utils as pu
    torch.manual_seed(9)
    B, N, M, S = 2, 512, 256, 16
    idx = torch.randint(0, N, (B, M, S), device=cuda, dtype=torch.int32)
    idx[0, :8] = 7                                   # a point with many entries (> 8 rounds)
    off, rows = pu.group_inverse(idx, N)
    ldg = (3 + C + 7) // 8 * 8 if ldg_kind == "cp" else 3 + C + (0 if (3 + C) % 2 else 1)
    g = torch.randn(B * M * S, ldg, device=cuda).to(torch.bfloat16)
    gf = torch.full((N, B, C), float("nan"), device=cuda).permute(1, 2, 0)   # (B, C, N) view
    st = gf.stride()
    _native.call("ov3d_group_bwd_csr_bf16", g, ldg, off, rows, B, C, N, st[0], st[2], st[1], gf,
                 like=g)
    offc, rowsc = off.cpu().long(), rows.cpu().long()
    deg = offc[1:] - offc[:-1]
    D = int(deg.max())
    ent = torch.full((B * N, D), -1, dtype=torch.long)
    for p in range(B * N):
        ent[p, :deg[p]] = rowsc[offc[p]:offc[p + 1]]
    feat = g[:, 3:3 + C].float()
    acc = torch.zeros((B * N, C), device=cuda)
    ent = ent.to(cuda)
    for k in range(D):
        e = ent[:, k]
        acc = acc + torch.where((e >= 0)[:, None], feat[e.clamp(min=0)], torch.zeros((), device=cuda))
    ref = acc.view(B, N, C).transpose(1, 2)
    assert torch.equal(gf, ref)
