"""GPU parity of the C-ABI kernels against the CPU oracle (tests-only checker).

Bar: bit-exact for integer/index results (voxel representatives, trace,
kNN index sets — including the sets the production normals kernels select —
RANSAC counts and inlier sets); normals and ICP transforms within 1e-5, signed,
on every row (tests/parity.py: the only allowance is a row certified as
decided by a one-ulp libm difference, counted in the report)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import np_restate as NPR
from open3dpypro import ops, synthetic as S
from parity import DebugNeighbors, assert_neighbour_sets, assert_normals

pytestmark = pytest.mark.gpu


def _normal_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max(1), np.minimum(np.abs(a - b).max(1), np.abs(a + b).max(1))


# ------------------------------------------------------------------ AABB
def test_aabb(dev, bunny):
    mn, mx = ops.aabb(torch.from_numpy(bunny).to(dev))
    rmn, rmx = O.aabb(bunny)
    assert np.array_equal(mn, rmn) and np.array_equal(mx, rmx)


def test_aabb_empty(dev):
    mn, mx = ops.aabb(torch.zeros((0, 3), device=dev))
    assert not mn.any() and not mx.any()


# ----------------------------------------------------------------- voxel
@pytest.mark.parametrize("vs,expect_m", [(0.005, 3017), (0.01, 751)])
def test_voxel_bunny(dev, bunny, vs, expect_m):
    out = ops.voxel_down_sample(torch.from_numpy(bunny).to(dev), vs, trace=True)
    rep = out["rep_idx"].cpu().numpy()
    ref, vop, cub = O.voxel_down_sample(bunny, vs, trace=True)
    assert len(rep) == expect_m
    assert np.array_equal(rep, ref)
    assert np.array_equal(out["voxel_of_point"].cpu().numpy(), vop)
    assert np.array_equal(out["cubic_id"].cpu().numpy(), cub)
    assert np.array_equal(out["rep_xyz"].cpu().numpy(), bunny[ref])


@pytest.mark.parametrize("n,seed", [(1, 0), (7, 1), (100_000, 2), (1_000_003, 3)])
def test_voxel_uniform(dev, n, seed):
    pts = S.uniform_cube(n, seed)
    vs = S.voxel_size_for(max(n, 8))
    rep = ops.voxel_down_sample(pts.to(dev), vs)["rep_idx"].cpu().numpy()
    assert np.array_equal(rep, O.voxel_down_sample(pts.numpy(), vs))
    if n <= 100_000:
        assert np.array_equal(rep, NPR.voxel_down_sample(pts.numpy(), vs))


@pytest.mark.parametrize("case", ["uniform", "hot_brick", "spatially_sorted"])
def test_voxel_binning_one_pass_and_fallback(dev, monkeypatch, case):
    """The one-pass binning into fixed per-brick segments (uniform cloud) and
    its fall-back to count + scatter when a brick outgrows its segment (75 %
    of the points in one brick): representatives, trace and the one-call
    normals equal the oracle's / the two-pass path's.  The hot-brick one-call
    run fires the normals on attempt 0's table and must redo them on the
    rebuilt one (geom[10]).  A spatially sorted cloud sends each brick's
    points from one or two blocks, i.e. into one of the brick's segment
    copies: it overflows the copies and retries with one copy per brick."""
    rng = np.random.default_rng(41)
    if case == "uniform":
        n = 400_001
        pts = rng.random((n, 3)).astype(np.float32)
    elif case == "spatially_sorted":
        n = 400_001
        pts = ops.spatial_sort(torch.from_numpy(rng.random((n, 3)).astype(np.float32)).to(dev))[:, :3]
        pts = pts.contiguous().cpu().numpy()
    else:
        n = 400_003
        pts = np.concatenate([rng.random((300_003, 3)) * 0.01, rng.random((100_000, 3))]).astype(np.float32)
        pts = pts[rng.permutation(n)]
    vs = 0.01
    x = torch.from_numpy(pts).to(dev)
    f = ops.voxel_down_sample_normals(x, vs, knn=30)  # first: the one-pass attempt (and its overflow)
    out = ops.voxel_down_sample(x, vs, trace=True)
    ref, vop, cub = O.voxel_down_sample(pts, vs, trace=True)
    assert np.array_equal(out["rep_idx"].cpu().numpy(), ref)
    assert np.array_equal(out["voxel_of_point"].cpu().numpy(), vop)
    assert np.array_equal(out["cubic_id"].cpu().numpy(), cub)
    monkeypatch.setenv("O3DX_VOXEL_TWOPASS", "1")
    a = ops.voxel_down_sample(x, vs, keep_grid=True)
    monkeypatch.delenv("O3DX_VOXEL_TWOPASS")
    assert np.array_equal(a["rep_idx"].cpu().numpy(), ref)
    ref_n = ops.estimate_normals(a["rep_xyz"], knn=30, voxel_grid=a["voxel_grid"])
    assert torch.equal(f["rep_idx"], a["rep_idx"]) and torch.equal(f["normals"], ref_n)


def test_voxel_hash_path_and_bounds(dev):
    # sparse clusters far apart -> grid box >> 2n cells -> hash table path
    rng = np.random.default_rng(5)
    c = rng.uniform(-1000, 1000, (50, 3))
    pts = (c[rng.integers(0, 50, 20000)] + rng.normal(0, 0.05, (20000, 3))).astype(np.float32)
    vs = 0.01
    rep = ops.voxel_down_sample(torch.from_numpy(pts).to(dev), vs)["rep_idx"].cpu().numpy()
    assert np.array_equal(rep, O.voxel_down_sample(pts, vs))
    # explicit bounds that do not contain every point (dense path must fall back)
    mnb = pts.min(0).astype(np.float64) + 100.0
    mxb = mnb + 10.0
    rep = ops.voxel_down_sample(torch.from_numpy(pts).to(dev), 0.5, mnb, mxb)["rep_idx"].cpu().numpy()
    assert np.array_equal(rep, O.voxel_down_sample(pts, 0.5, mnb, mxb))


@pytest.mark.parametrize("path", ["hbin", "hbin_overflow", "global_hash"])
@pytest.mark.parametrize("case", ["clusters", "surface", "surface_2e10"])
def test_voxel_sparse_paths(dev, monkeypatch, path, case):
    """Sparse grids (box >> 2n voxels): the hash-binned reduction (LDS table
    per bin), its fall-back when a bin's table overflows, and the global hash
    table all give the oracle's representatives and trace.  surface_2e10: a
    1.3 m cube at 0.5 mm = 2601^3 = 1.76e10 voxels (a 35-bit voxel id, so the
    per-bin rest takes 23 bits: more than the 20 the round-2 entry layout had
    room for)."""
    monkeypatch.setenv("O3DX_VOXEL_HBIN_MIN", "-1" if path == "global_hash" else "0")
    if path == "hbin_overflow":
        monkeypatch.setenv("O3DX_VOXEL_HBIN_SLOTS", "4")
    rng = np.random.default_rng(15)
    if case == "clusters":
        c = rng.uniform(-1000, 1000, (50, 3))
        pts = (c[rng.integers(0, 50, 60000)] + rng.normal(0, 0.05, (60000, 3))).astype(np.float32)
        vs = 0.01
    elif case == "surface":
        pts = S.box_surface(300_000, 17).numpy()
        vs = 0.0005
    else:
        pts = S.box_surface(300_000, 19, dims=(1.3, 1.3, 1.3)).numpy()
        vs = 0.0005
    out = ops.voxel_down_sample(torch.from_numpy(pts).to(dev), vs, trace=True)
    ref, vop, cub = O.voxel_down_sample(pts, vs, trace=True)
    assert np.array_equal(out["rep_idx"].cpu().numpy(), ref)
    assert np.array_equal(out["voxel_of_point"].cpu().numpy(), vop)
    assert np.array_equal(out["cubic_id"].cpu().numpy(), cub)
    rep = ops.voxel_down_sample(torch.from_numpy(pts).to(dev), vs)["rep_idx"].cpu().numpy()
    assert np.array_equal(rep, ref)


def test_voxel_duplicates_negative(dev):
    rng = np.random.default_rng(9)
    base = rng.uniform(-3, -1, (3000, 3)).astype(np.float32)
    pts = np.concatenate([base, base[::3], base[::7]])
    rep = ops.voxel_down_sample(torch.from_numpy(pts).to(dev), 0.05, trace=True)
    ref, vop, cub = O.voxel_down_sample(pts, 0.05, trace=True)
    assert np.array_equal(rep["rep_idx"].cpu().numpy(), ref)
    assert np.array_equal(rep["cubic_id"].cpu().numpy(), cub)


def test_voxel_errors(dev):
    x = torch.rand(100, 3, device=dev)
    with pytest.raises(RuntimeError, match="voxel_size <= 0"):
        ops.voxel_down_sample(x, 0.0)
    with pytest.raises(RuntimeError, match="too small"):
        ops.voxel_down_sample(x * 1e3, 1e-9)


def test_voxel_empty(dev):
    out = ops.voxel_down_sample(torch.zeros((0, 3), device=dev), 0.1)
    assert out["rep_idx"].numel() == 0


# --------------------------------------------------------------- normals
def test_normals_knn30_bunny_reps(dev, bunny):
    ref_idx = O.voxel_down_sample(bunny, 0.005)
    reps = bunny[ref_idx]
    with DebugNeighbors(len(reps), 30, dev) as dn:
        got = ops.estimate_normals(torch.from_numpy(reps).to(dev), knn=30).cpu().numpy()
    exp = O.estimate_normals(reps, O.KNN, 30)
    assert_normals(got, exp, reps, k=30, what="bunny_reps_knn30")
    assert_neighbour_sets(dn.ids(), reps, 30, "bunny_reps_knn30")


@pytest.mark.parametrize("k", [3, 8, 16, 30, 64])
def test_normals_knn_uniform(dev, k):
    pts = S.uniform_cube(50_000, 11).numpy()
    with DebugNeighbors(len(pts), k, dev) as dn:
        got = ops.estimate_normals(torch.from_numpy(pts).to(dev), knn=k).cpu().numpy()
    exp = O.estimate_normals(pts, O.KNN, k)
    assert_normals(got, exp, pts, k=k, what=f"uniform50k_knn{k}")
    assert_neighbour_sets(dn.ids(), pts, k, f"uniform50k_knn{k}")


def test_normals_hybrid_radius(dev, bunny):
    x = torch.from_numpy(bunny).to(dev)
    for mode, k, r in [(O.HYBRID, 30, 0.01), (O.HYBRID, 8, 0.003), (O.RADIUS, 0, 0.004)]:
        got = ops.estimate_normals(x, mode=mode, knn=k, radius=r).cpu().numpy()
        exp = O.estimate_normals(bunny, mode, k, r)
        assert_normals(got, exp, bunny, mode, k, r, what=f"bunny_mode{mode}_k{k}_r{r}")


def test_normals_prior_orientation(dev, bunny):
    prior = np.tile(np.array([[0.0, 0.0, 1.0]]), (len(bunny), 1))
    got = ops.estimate_normals(torch.from_numpy(bunny).to(dev), knn=20,
                               prior=torch.from_numpy(prior.astype(np.float32)).to(dev)).cpu().numpy()
    exp = O.estimate_normals(bunny, O.KNN, 20, prior=prior)
    assert_normals(got, exp, bunny, k=20, prior=prior, what="bunny_prior_knn20")
    assert (got[:, 2] >= -1e-7).all()


def test_normals_degenerate(dev):
    # fewer than 3 neighbours / identical points -> (0,0,1)
    pts = np.zeros((5, 3), np.float32)
    got = ops.estimate_normals(torch.from_numpy(pts).to(dev), knn=30).cpu().numpy()
    assert np.allclose(got, [[0, 0, 1]] * 5)
    two = np.array([[0, 0, 0], [1, 0, 0]], np.float32)
    got = ops.estimate_normals(torch.from_numpy(two).to(dev), knn=30).cpu().numpy()
    assert np.allclose(got, O.estimate_normals(two, O.KNN, 30))


# ------------------------------------------------------------- kNN search
def test_knn_search_sets(dev, bunny):
    q = bunny[::37]
    idx, d2, cnt = ops.knn_search(torch.from_numpy(bunny).to(dev), torch.from_numpy(q).to(dev), knn=30)
    ridx, rd2, rcnt = O.knn_search(bunny, q, O.KNN, 30)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert np.array_equal(d2.cpu().numpy(), rd2)
    idx, d2, cnt = ops.knn_search(torch.from_numpy(bunny).to(dev), torch.from_numpy(q).to(dev),
                                  mode=O.HYBRID, knn=16, radius=0.004)
    ridx, rd2, rcnt = O.knn_search(bunny, q, O.HYBRID, 16, 0.004)
    assert np.array_equal(cnt.cpu().numpy(), rcnt)
    assert np.array_equal(idx.cpu().numpy(), ridx)


def test_knn_search_outside_queries(dev):
    pts = S.uniform_cube(20000, 4).numpy()
    q = (np.random.default_rng(1).uniform(-1, 2, (500, 3))).astype(np.float32)
    idx, d2, cnt = ops.knn_search(torch.from_numpy(pts).to(dev), torch.from_numpy(q).to(dev), knn=8)
    ridx, rd2, _ = O.knn_search(pts, q, O.KNN, 8)
    assert np.array_equal(idx.cpu().numpy(), ridx)


# ----------------------------------------------------------------- RANSAC
def test_ransac_sampler_matches_oracle():
    a = ops.ransac_samples(12345, 3, 500, 7)
    b = O.ransac_samples(12345, 3, 500, 7)
    assert np.array_equal(a, b)
    assert all(len(set(r)) == 3 for r in a)


@pytest.mark.parametrize("n,iters", [(5000, 100), (300_000, 256)])
def test_ransac_counts_exact(dev, n, iters):
    pts = S.planted_plane(n, 21).numpy()
    samples = O.ransac_samples(n, 3, iters, 5)
    _, _, counts, sums, _ = O.segment_plane(pts, 0.01, 3, iters, samples)
    planes = np.stack([NPR.triangle_plane(*pts[s].astype(np.float64)) for s in samples])
    got = ops.plane_count(torch.from_numpy(pts).to(dev), planes, 0.01)
    assert np.array_equal(got, counts)
    ok = counts > 0
    which = np.nonzero(ok)[0]
    gs, gfx = ops.plane_abs_sum(torch.from_numpy(pts).to(dev), planes, which, 0.01, return_fx=True)
    np.testing.assert_allclose(gs, sums[ok], rtol=1e-12)
    # the exact fx sums: the same integers as the numpy restatement (any split)
    for j, h in enumerate(which[:40]):
        exp = NPR.plane_abs_sum_fx(pts, planes[h], 0.01)
        assert NPR.fx_value(gfx[j]) == NPR.fx_value(exp) == gs[j]


def test_plane_moments_fx_exact(dev):
    """GetPlaneFromPoints moments as fx sums: the same values as the numpy
    restatement over the same inliers (exact integers, any order)."""
    pts = S.planted_plane(200_000, 7).numpy()
    x = torch.from_numpy(pts).to(dev)
    idx = torch.nonzero(torch.from_numpy(np.abs(pts[:, 2] - 0.5) < 0.01)).flatten().to(dev)
    am = np.abs(pts.astype(np.float64)).max(0)
    A = float(am.max())
    s1, f1 = ops.plane_moments(x, idx, absmax=am, return_fx=True)
    sel = pts[idx.cpu().numpy()]
    e1 = NPR.plane_moments_fx(sel, A)
    assert [NPR.fx_value(r) for r in f1] == [NPR.fx_value(r) for r in e1] == list(s1)
    c = s1 / idx.numel()
    s2, f2 = ops.plane_moments(x, idx, centroid=c, absmax=am, return_fx=True)
    e2 = NPR.plane_moments_fx(sel, A, c)
    assert [NPR.fx_value(r) for r in f2] == [NPR.fx_value(r) for r in e2] == list(s2)


@pytest.mark.parametrize("n,iters,ransac_n", [(30_000, 450, 3), (200_000, 1000, 3), (20_000, 100, 5)])
def test_segment_plane_parity(dev, n, iters, ransac_n):
    pts = S.planted_plane(n, 33).numpy()
    samples = O.ransac_samples(n, ransac_n, iters, 9)
    plane, inl = ops.segment_plane(torch.from_numpy(pts).to(dev), 0.01, ransac_n, iters, samples=samples)
    rplane, rinl, _, _, _ = O.segment_plane(pts, 0.01, ransac_n, iters, samples)
    assert np.array_equal(inl.cpu().numpy().astype(np.int64), rinl)
    np.testing.assert_allclose(plane, rplane, rtol=0, atol=1e-9)


@pytest.mark.parametrize("ransac_n", [3, 6])
def test_segment_plane_device_setup_equals_host(dev, monkeypatch, ransac_n):
    """segment_plane's culled path forms the hypotheses on the device
    (k_ransac_setup) with the host's own plane math: the same plane and
    inliers bit for bit as the host-setup path (O3DX_RANSAC_HOST_SETUP), the
    planes of every hypothesis included (through the chosen plane and its
    refit), on a planted plane and on degenerate (repeated-point) samples."""
    n = 100_000
    pts = S.planted_plane(n, 41).numpy()
    samples = O.ransac_samples(n, ransac_n, 500, 13).reshape(500, ransac_n)
    samples[::7, 1] = samples[::7, 0]  # every 7th hypothesis degenerate for ransac_n = 3
    x = torch.from_numpy(pts).to(dev)
    p_dev, i_dev = ops.segment_plane(x, 0.01, ransac_n, 500, samples=samples)
    monkeypatch.setenv("O3DX_RANSAC_HOST_SETUP", "1")
    p_host, i_host = ops.segment_plane(x, 0.01, ransac_n, 500, samples=samples)
    assert np.array_equal(np.asarray(p_dev), np.asarray(p_host))
    assert torch.equal(i_dev, i_host)
    rplane, rinl, _, _, _ = O.segment_plane(pts, 0.01, ransac_n, 500, samples)
    assert np.array_equal(i_dev.cpu().numpy().astype(np.int64), rinl)
    np.testing.assert_allclose(p_dev, rplane, rtol=0, atol=1e-9)


def test_segment_plane_tiny_threshold_device_setup(dev, monkeypatch):
    """A threshold tiny against the coordinates (a plane 1e3 units from the
    origin, thr 2e-6): the culled sweep's guard (6 2^-24 S + 2^-20 thr <
    thr / 2) fails, and the device-setup path replays it on the bounds it
    reads back and recounts with the dense sweep — plane and
    inliers equal the host-setup path's and the oracle's."""
    n = 20_000
    pts = S.planted_plane(n, 43, sigma=1e-6).numpy().astype(np.float64)
    pts = (pts + np.array([1000.0, -700.0, 1000.0])).astype(np.float32)
    samples = O.ransac_samples(n, 3, 300, 17)
    x = torch.from_numpy(pts).to(dev)
    p_dev, i_dev = ops.segment_plane(x, 2e-6, 3, 300, samples=samples)
    monkeypatch.setenv("O3DX_RANSAC_HOST_SETUP", "1")
    p_host, i_host = ops.segment_plane(x, 2e-6, 3, 300, samples=samples)
    assert np.array_equal(np.asarray(p_dev), np.asarray(p_host))
    assert torch.equal(i_dev, i_host)
    rplane, rinl, _, _, _ = O.segment_plane(pts, 2e-6, 3, 300, samples)
    assert np.array_equal(i_dev.cpu().numpy().astype(np.int64), rinl)
    np.testing.assert_allclose(p_dev, rplane, rtol=0, atol=1e-9)


def test_segment_plane_ties_small(dev):
    # tiny cloud: many hypotheses tie in count -> rmse tie-break path
    pts = S.planted_plane(60, 3).numpy()
    samples = O.ransac_samples(60, 3, 200, 1)
    plane, inl = ops.segment_plane(torch.from_numpy(pts).to(dev), 0.05, 3, 200, samples=samples)
    rplane, rinl, _, _, _ = O.segment_plane(pts, 0.05, 3, 200, samples)
    assert np.array_equal(inl.cpu().numpy().astype(np.int64), rinl)
    np.testing.assert_allclose(plane, rplane, atol=1e-9)


@pytest.mark.parametrize("n,thr,seed,prob", [(40, 0.05, 2, 0.99999999), (60, 0.2, 3, 1.0), (200, 0.05, 4, 0.99999999),
                                             (200, 0.3, 5, 1.0), (1000, 0.02, 6, 0.99)])
def test_segment_plane_tie_replay(dev, n, thr, seed, prob):
    """Small clouds where many hypotheses share counts: only the ties the
    sequential selection can consult get their Sigma |d| (replay on the
    counts); the chosen plane and inliers still equal the oracle's."""
    pts = S.planted_plane(n, seed).numpy()
    samples = O.ransac_samples(n, 3, 300, seed)
    plane, inl = ops.segment_plane(torch.from_numpy(pts).to(dev), thr, 3, 300, prob, samples=samples)
    rplane, rinl, _, _, _ = O.segment_plane(pts, thr, 3, 300, samples, probability=prob)
    assert np.array_equal(inl.cpu().numpy().astype(np.int64), rinl)
    np.testing.assert_allclose(plane, rplane, atol=1e-9)


def test_segment_plane_errors(dev):
    x = torch.rand(2, 3, device=dev)
    with pytest.raises(RuntimeError, match="ransac_n"):
        ops.segment_plane(x, 0.01, 3, 10)
    with pytest.raises(RuntimeError, match="Probability"):
        ops.segment_plane(torch.rand(10, 3, device=dev), 0.01, 3, 10, probability=0.0)


# -------------------------------------------------------------------- ICP
def _icp_case(n, seed=1):
    tgt = S.box_surface(n, seed)
    src = S.apply_transform(S.box_surface(n, seed + 1), S.rigid_transform())
    return src.numpy(), tgt.numpy()


def test_icp_accumulate_matches_oracle(dev):
    src, tgt = _icp_case(20000)
    tn = O.estimate_normals(tgt, O.KNN, 30).astype(np.float32)
    T = S.rigid_transform(0.3, (0, 0, 1), (0.001, 0, 0))
    target = ops.ICPTarget(torch.from_numpy(tgt).to(dev), torch.from_numpy(tn).to(dev), 0.02)
    sums, corr, fx = target.accumulate(torch.from_numpy(src).to(dev), T, want_corr=True, return_fx=True)
    ref = O.icp_accumulate(src, tgt, tn, 0.02, T)
    assert sums[28] == ref[28]
    np.testing.assert_allclose(sums[:30], ref[:30], rtol=1e-9, atol=1e-9)
    # the exact fx sums equal the oracle's independent 128-bit restatement
    rfx = O.icp_accumulate_fx(src, tgt, tn, 0.02, T, np.abs(src.astype(np.float64)).max(0))
    assert np.array_equal(fx[:, 2], rfx[:, 2])
    assert np.array_equal(ops.fx_to_double(fx), ops.fx_to_double(rfx))


def test_registration_icp_parity(dev):
    src, tgt = _icp_case(30000)
    tn = O.estimate_normals(tgt, O.KNN, 30).astype(np.float32)
    res = ops.registration_icp(torch.from_numpy(src).to(dev), torch.from_numpy(tgt).to(dev),
                               torch.from_numpy(tn).to(dev), 0.02, max_iteration=30,
                               relative_fitness=0.0, relative_rmse=0.0)
    T, fit, rmse, corr = O.registration_icp(src, tgt, tn, 0.02, max_iteration=30, relative_fitness=0.0,
                                            relative_rmse=0.0)
    np.testing.assert_allclose(res["transformation"], T, atol=1e-5)
    assert abs(res["fitness"] - fit) < 1e-6
    assert abs(res["inlier_rmse"] - rmse) < 1e-6
    Tgt_inv = np.linalg.inv(S.rigid_transform())
    assert np.abs(res["transformation"] - Tgt_inv).max() < 2e-3


@pytest.mark.parametrize("rel", [0.0, 1e-6])
def test_icp_device_loop_equals_host_loop(dev, rel):
    """The loop on the device (ICPTarget.register / o3dx_icp_register: solve,
    update and convergence test in k_icp_finish) gives the same T, fitness,
    rmse and correspondences to the bit as the host loop over accumulate +
    icp_update (the multi-GPU loop's arithmetic), with and without an early
    convergence stop; registration_icp (the same loop after its own target
    build and sort) agrees too."""
    src, tgt = _icp_case(30000, seed=11)
    tn = O.estimate_normals(tgt, O.KNN, 30).astype(np.float32)
    t, n = torch.from_numpy(tgt).to(dev), torch.from_numpy(tn).to(dev)
    target = ops.ICPTarget(t, n, 0.02)
    s4 = ops.spatial_sort(torch.from_numpy(src).to(dev))
    am = np.abs(src.astype(np.float64)).max(0)
    res = target.register(s4, max_iteration=25, relative_fitness=rel, relative_rmse=rel, absmax=am, want_corr=True)
    T = np.eye(4)
    sums, _ = target.accumulate(s4, T, absmax=am)
    fit, rm = sums[28] / len(src), np.sqrt(sums[29] / sums[28])
    for _ in range(25):
        T = ops.icp_update(sums, T)
        pf, pr = fit, rm
        sums, corr = target.accumulate(s4, T, absmax=am, want_corr=True)
        fit, rm = sums[28] / len(src), np.sqrt(sums[29] / sums[28])
        if abs(pf - fit) < rel and abs(pr - rm) < rel:
            break
    assert np.array_equal(res["transformation"], T)
    assert res["fitness"] == fit and res["inlier_rmse"] == rm
    assert torch.equal(res["correspondence_set"], corr)
    one = ops.registration_icp(torch.from_numpy(src).to(dev), t, n, 0.02, max_iteration=25, relative_fitness=rel,
                               relative_rmse=rel)
    assert np.array_equal(one["transformation"], T) and one["fitness"] == fit
    assert torch.equal(one["correspondence_set"], corr)


@pytest.mark.parametrize("n", [300_000, 2_000_000])
def test_icp_skip_proof_equals_full_search(dev, monkeypatch, n):
    """The device loop's skip proof (icp.hip k_icp_step MODE 2: a point keeps
    its match while twice its motion stays below the margin its last
    extended-ball search left) returns the correspondences of a full search
    in every iteration: T, fitness, rmse and the final correspondence set
    equal the loop with every step searching (O3DX_ICP_SKIP=0) to the bit,
    and most converged steps search far fewer points (the debug search
    counters count searched queries only)."""
    from open3dpypro import _native as N
    src, tgt = _icp_case(n, seed=21)
    t = torch.from_numpy(tgt).to(dev)
    n_ = ops.estimate_normals(t, knn=30)
    target = ops.ICPTarget(t, n_, 0.02)
    s4 = ops.spatial_sort(torch.from_numpy(src).to(dev))
    runs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("O3DX_ICP_SKIP", mode)
        N.search_stats(True)
        res = target.register(s4, max_iteration=30, relative_fitness=0.0, relative_rmse=0.0, want_corr=True)
        runs[mode] = (res, N.search_stats()["queries"])
        N.search_stats(False)
    (a, qa), (b, qb) = runs["1"], runs["0"]
    assert np.array_equal(a["transformation"], b["transformation"])
    assert a["fitness"] == b["fitness"] and a["inlier_rmse"] == b["inlier_rmse"]
    assert torch.equal(a["correspondence_set"], b["correspondence_set"])
    assert qb >= 31 * n and qa < 0.5 * qb, (qa, qb)


def test_icp_accumulate_sorted_source_layout(dev):
    src, tgt = _icp_case(30000, seed=4)
    tn = O.estimate_normals(tgt, O.KNN, 30).astype(np.float32)
    T = S.rigid_transform(0.2, (1, 0, 0), (0, 0.002, 0))
    target = ops.ICPTarget(torch.from_numpy(tgt).to(dev), torch.from_numpy(tn).to(dev), 0.02)
    s = torch.from_numpy(src).to(dev)
    s4 = ops.spatial_sort(s)
    assert torch.equal(torch.sort(s4[:, 3].contiguous().view(torch.int32).long())[0],
                       torch.arange(len(src), device=dev))
    a, ca = target.accumulate(s, T, want_corr=True)
    b, cb = target.accumulate(s4, T, want_corr=True)
    assert np.array_equal(a, b)  # fx sums: the order of the source does not matter
    assert torch.equal(ca, cb)
    ref = O.icp_accumulate(src, tgt, tn, 0.02, T)
    np.testing.assert_allclose(b[:30], ref[:30], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("shift", [0.0, 0.006, 0.015, 0.05])
def test_icp_displaced_source_exact(dev, shift):
    """ICP correspondences for sources displaced by up to and beyond
    max_correspondence_distance (ICP's first iterations): the sorted and the
    caller-order source give the same matches, and the moments equal the
    oracle's."""
    src, tgt = _icp_case(40000, seed=6)
    tn = O.estimate_normals(tgt, O.KNN, 30).astype(np.float32)
    T = S.rigid_transform(2.0, (0, 1, 1), (shift, -shift / 2, shift / 3))
    target = ops.ICPTarget(torch.from_numpy(tgt).to(dev), torch.from_numpy(tn).to(dev), 0.02)
    s = torch.from_numpy(src).to(dev)
    a, ca = target.accumulate(s, T, want_corr=True)
    b, cb = target.accumulate(ops.spatial_sort(s), T, want_corr=True)
    assert torch.equal(ca, cb)
    assert np.array_equal(a, b)  # fx sums: the same bits in any source order
    ref = O.icp_accumulate(src, tgt, tn, 0.02, T)
    assert a[28] == ref[28]
    np.testing.assert_allclose(a[:30], ref[:30], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("shift", [0.0, 0.004, 0.012, 0.03, 0.3])
def test_icp_row_walk_correspondences_exact(dev, shift):
    """The 1-NN row walk returns, for every source point, the oracle's
    KDTreeFlann SearchHybrid(p, r, 1) match on the same float64 transformed
    point (the exact (d^2, index) minimum within max_correspondence_distance),
    for sources displaced within, across and far beyond the radius (0.3:
    queries outside the target grid), and the moments equal the oracle's."""
    src, tgt = _icp_case(60000, seed=9)
    tn = O.estimate_normals(tgt, O.KNN, 30).astype(np.float32)
    T = S.rigid_transform(3.0, (1, 2, 0), (shift, shift / 3, -shift / 2))
    target = ops.ICPTarget(torch.from_numpy(tgt).to(dev), torch.from_numpy(tn).to(dev), 0.02)
    s4 = ops.spatial_sort(torch.from_numpy(src).to(dev))
    a, ca = target.accumulate(s4, T, want_corr=True)
    p = src.astype(np.float64)  # the kernel's transform: ((t0 x + t1 y) + t2 z) + t3, unfused
    q = np.stack([((T[r, 0] * p[:, 0] + T[r, 1] * p[:, 1]) + T[r, 2] * p[:, 2]) + T[r, 3] for r in range(3)], 1)
    ridx, _, rc = O.knn_search(tgt, q, O.HYBRID, 1, 0.02)
    exp = np.stack([np.nonzero(rc > 0)[0], ridx[rc > 0, 0]], 1)
    got = ca.cpu().numpy().astype(np.int64)
    got = got[np.argsort(got[:, 0])]
    assert np.array_equal(got, exp)
    ref = O.icp_accumulate(src, tgt, tn, 0.02, T)
    assert a[28] == ref[28]
    np.testing.assert_allclose(a[:30], ref[:30], rtol=1e-9, atol=1e-9)


def test_normals_raw_planted_plane_big_cells(dev):
    """estimate_normals on a raw (not down-sampled) planted-plane cloud whose
    thin dense plane puts > 256 points in many grid cells (the in-cell order
    then comes from the workgroup-per-cell ranking, k_grid_big_cells): every
    row within 1e-5 of the oracle; run to run bit-identical."""
    pts = S.planted_plane(1_000_000, 5, frac=0.8, sigma=0.0005).numpy()
    x = torch.from_numpy(pts).to(dev)
    a = ops.estimate_normals(x, knn=30).cpu().numpy()
    b = ops.estimate_normals(x, knn=30).cpu().numpy()
    assert np.array_equal(a, b)
    assert_normals(a, O.estimate_normals(pts, O.KNN, 30), pts, k=30, what="raw_planted_plane_1m")


@pytest.mark.parametrize("k", [8, 30, 64])
@pytest.mark.parametrize("frac,sigma", [(0.2, 0.002), (0.5, 0.0002)])
def test_normals_nested_grid_planted_plane(dev, k, frac, sigma, monkeypatch):
    """A dense plane inside a sparse volume (C3's composition at 1M): the
    dense cells' queries run on the nested grid (grid.hip "nested grids").
    Every row within 1e-5 of the oracle, neighbour sets bit-exact (debug
    hook), and the normals bit-identical to the run without the nested grid."""
    pts = S.planted_plane(1_000_000, 40 + k, frac=frac, sigma=sigma).numpy()
    x = torch.from_numpy(pts).to(dev)
    with DebugNeighbors(len(pts), k, dev) as dn:
        a = ops.estimate_normals(x, knn=k).cpu().numpy()
    monkeypatch.setenv("O3DX_NESTED_OFF", "1")
    b = ops.estimate_normals(x, knn=k).cpu().numpy()
    monkeypatch.delenv("O3DX_NESTED_OFF")
    assert np.array_equal(a, b)
    assert_neighbour_sets(dn.ids(), pts, k, f"nested_plane_k{k}_f{frac}")
    assert_normals(a, O.estimate_normals(pts, O.KNN, k), pts, k=k, what=f"nested_plane_k{k}_f{frac}")


@pytest.mark.parametrize("k", [5, 30, 64])
@pytest.mark.parametrize("shape", ["cube", "surface", "dups"])
def test_normals_knn_paths_agree(dev, k, shape):
    """The three KNN-normals forms (LDS tile -> wave per query -> register
    top-k) agree: default chain vs wave form over every query vs exact top-k."""
    import os
    if shape == "cube":
        pts = S.uniform_cube(200_000, 12)
    elif shape == "surface":
        pts = S.box_surface(200_000, 13)
    else:  # exact duplicates: ties at d2 = 0 (pairs / triples keep the covariance well posed)
        base = S.uniform_cube(20_000, 14)
        pts = torch.cat([base, base[:5000], base[:5000]])
    x = pts.to(dev)
    outs = {}
    for mode, env in (("chain", None), ("wave", "O3DX_NORMALS_NO_TILES"), ("topk", "O3DX_NORMALS_TOPK")):
        if env:
            os.environ[env] = "1"
        try:
            outs[mode] = ops.estimate_normals(x, knn=k).cpu().numpy()
        finally:
            if env:
                del os.environ[env]
    for mode in ("chain", "wave"):
        e = np.abs(outs[mode] - outs["topk"]).max(1)
        assert np.mean(e < 1e-6) > 0.9999, (mode, e.max())
    p = pts.numpy()
    exp = O.estimate_normals(p, O.KNN, k)
    for mode in ("chain", "wave", "topk"):
        assert_normals(outs[mode], exp, p, k=k, what=f"paths_{shape}_k{k}_{mode}")


def test_normals_knn_degenerate_clusters(dev):
    """40 copies of each of 300 points (neighbourhoods of identical points,
    counters near their packing limits): every form returns finite unit normals
    and the (0, 0, 1) default where the covariance is exactly zero."""
    import os
    base = S.uniform_cube(20_000, 15)
    pts = torch.cat([base, base[:300].repeat(40, 1)]).to(dev)
    for env in (None, "O3DX_NORMALS_NO_TILES", "O3DX_NORMALS_TOPK"):
        if env:
            os.environ[env] = "1"
        try:
            nrm = ops.estimate_normals(pts, knn=30).cpu().numpy()
        finally:
            if env:
                del os.environ[env]
        assert np.isfinite(nrm).all()
        assert np.allclose(np.linalg.norm(nrm, axis=1), 1.0, atol=1e-5)


# ------------------------------------------- voxel grid kept for the normals
@pytest.mark.parametrize("shape", ["cube", "surface", "bunny"])
@pytest.mark.parametrize("k", [5, 30])
def test_normals_on_voxel_grid(dev, bunny, shape, k):
    """voxel_down_sample(keep_grid) + estimate_normals(voxel_grid=): the
    representatives are unchanged, the search grid is read off the voxel
    table, and the normals agree with the sorted-grid path (to float64
    summation order) and with the oracle."""
    if shape == "cube":
        pts, vs = S.uniform_cube(400_000, 21), S.voxel_size_for(400_000)
    elif shape == "surface":
        pts, vs = S.box_surface(400_000, 22), 0.01
    else:
        pts, vs = torch.from_numpy(bunny), 0.002
    x = pts.to(dev)
    a = ops.voxel_down_sample(x, vs, keep_grid=True)
    b = ops.voxel_down_sample(x, vs)
    assert torch.equal(a["rep_idx"], b["rep_idx"]) and torch.equal(a["rep_xyz"], b["rep_xyz"])
    vg = a["voxel_grid"]
    assert vg is not None and vg.m == a["rep_idx"].numel()
    fused = ops.estimate_normals(a["rep_xyz"], knn=k, voxel_grid=vg).cpu().numpy()
    plain = ops.estimate_normals(b["rep_xyz"], knn=k).cpu().numpy()
    e = np.abs(fused - plain).max(1)
    assert np.mean(e < 1e-6) > 0.9999, e.max()
    reps = pts.numpy()[a["rep_idx"].cpu().numpy()]
    exp = O.estimate_normals(reps, O.KNN, k)
    assert_normals(fused, exp, reps, k=k, what=f"voxel_grid_{shape}_k{k}")


def test_normals_on_voxel_grid_modes_and_prior(dev, bunny):
    """Hybrid / radius search and prior orientation over the voxel grid."""
    x = torch.from_numpy(bunny).to(dev)
    a = ops.voxel_down_sample(x, 0.002, keep_grid=True)
    reps, vg = a["rep_xyz"], a["voxel_grid"]
    for mode, kk, r in ((O.HYBRID, 30, 0.01), (O.RADIUS, 0, 0.006)):
        got = ops.estimate_normals(reps, mode=mode, knn=kk, radius=r, voxel_grid=vg).cpu().numpy()
        ref = ops.estimate_normals(reps, mode=mode, knn=kk, radius=r).cpu().numpy()
        assert np.mean(np.abs(got - ref).max(1) < 1e-6) > 0.9999
        if mode == O.HYBRID:
            rp = reps.cpu().numpy()
            assert_normals(got, O.estimate_normals(rp, mode, kk, r), rp, mode=mode, k=kk, radius=r,
                           what="voxel_grid_hybrid")
    prior = -ops.estimate_normals(reps, knn=30)
    got = ops.estimate_normals(reps, knn=30, prior=prior, voxel_grid=vg)
    assert (torch.sum(got * prior, 1) >= 0).all()


def test_voxel_grid_not_kept_when_sparse(dev):
    """Points outside the given bounds force the hash table: no grid is kept
    and estimate_normals takes the sorted-grid path."""
    pts = S.uniform_cube(20_000, 23)
    x = pts.to(dev)
    out = ops.voxel_down_sample(x, 0.05, min_bound=[0.2, 0.2, 0.2], max_bound=[0.8, 0.8, 0.8], keep_grid=True)
    assert out["voxel_grid"] is None
    ref = ops.voxel_down_sample(x, 0.05, min_bound=[0.2, 0.2, 0.2], max_bound=[0.8, 0.8, 0.8])
    assert torch.equal(out["rep_idx"], ref["rep_idx"])


STILE_ENVS = [
    {},
    {"O3DX_STILE_FORCE_FB": "1"},
    {"O3DX_NO_STILE": "1"},
    {"O3DX_STILE_SPLIT": "1"},  # shell blocks + their hand-offs on the side stream
    {"O3DX_STILE_SPLIT": "1", "O3DX_STILE_FORCE_FB": "1"},
]


@pytest.mark.parametrize("env", STILE_ENVS, ids=lambda e: "+".join(f"{k}={v}" for k, v in e.items()) or "default")
@pytest.mark.parametrize("k", [5, 30])
def test_normals_dense_voxel_table(dev, env, k, monkeypatch):
    """Volumetric reps fill their voxels: estimate_normals(voxel_grid=) runs
    straight off the dense voxel table (k_normals_stile; its hand-off path —
    wave form and register top-k over the table — forced for every query by
    O3DX_STILE_FORCE_FB; the sorted-grid path with O3DX_NO_STILE): every row within 1e-5 of
    the oracle, the selected neighbour sets bit-equal to the oracle's.
    Non-cubic box, dims not multiples of the 4^3 tile blocks."""
    n = 200_000
    pts = S.uniform_cube(n, 33) * torch.tensor([1.0, 0.55, 0.3])
    vs = float((0.165 * 4 / n) ** (1 / 3))
    x = pts.to(dev)
    a = ops.voxel_down_sample(x, vs, keep_grid=True)
    vg = a["voxel_grid"]
    assert vg is not None
    m = a["rep_idx"].numel()
    for kk, vv in env.items():
        monkeypatch.setenv(kk, vv)
    with DebugNeighbors(m, k, dev) as dn:
        fused = ops.estimate_normals(a["rep_xyz"], knn=k, voxel_grid=vg).cpu().numpy()
    for kk in env:
        monkeypatch.delenv(kk)
    reps = pts.numpy()[a["rep_idx"].cpu().numpy()]
    exp = O.estimate_normals(reps, O.KNN, k)
    tag = "+".join(f"{kk}={vv}" for kk, vv in env.items()) or "default"
    assert_normals(fused, exp, reps, k=k, what=f"dense_vox_{tag}_k{k}")
    assert_neighbour_sets(dn.ids(), reps, k, f"dense_vox_{tag}_k{k}")


@pytest.mark.parametrize("case", ["cube", "box", "bunny", "sparse", "tiny"])
def test_voxel_down_sample_normals_fused(dev, bunny, case):
    """The one-call pipeline (normals queued before the count read-back) gives
    the two-call results bit for bit — including where the table path does not
    apply (sparse cloud, m < k) and the normals are recomputed."""
    if case == "cube":
        pts, vs = S.uniform_cube(300_000, 51), S.voxel_size_for(300_000)
    elif case == "box":
        pts, vs = S.box_surface(200_000, 52), 0.01
    elif case == "bunny":
        pts, vs = torch.from_numpy(bunny), 0.002
    elif case == "sparse":
        pts, vs = S.uniform_cube(3000, 53), 0.02
    else:
        pts, vs = S.uniform_cube(40, 54), 0.3
    x = pts.to(dev)
    f = ops.voxel_down_sample_normals(x, vs, knn=30)
    a = ops.voxel_down_sample(x, vs, keep_grid=True)
    ref = ops.estimate_normals(a["rep_xyz"], knn=30, voxel_grid=a["voxel_grid"])
    assert torch.equal(f["rep_idx"], a["rep_idx"]) and torch.equal(f["rep_xyz"], a["rep_xyz"])
    assert torch.equal(f["normals"], ref)
    reps = pts.numpy()[a["rep_idx"].cpu().numpy()]
    assert_normals(f["normals"].cpu().numpy(), O.estimate_normals(reps, O.KNN, 30), reps, k=30,
                   what=f"fused_{case}")


@pytest.mark.parametrize("H", [5, 13, 101])
def test_plane_count_shapes(dev, H):
    """Every instantiated shape of the exact count (8 / 16 / 32 hypotheses per
    wave, picked by H) gives the oracle's counts (ragged n and H)."""
    n = 70_001
    pts = S.planted_plane(n, 62).numpy()
    samples = np.random.default_rng(9).integers(0, n, (H, 3)).astype(np.int32)
    planes = np.stack([NPR.triangle_plane(*pts[s].astype(np.float64)) for s in samples])
    got = ops.plane_count(torch.from_numpy(pts).to(dev), planes, 0.01)
    assert np.array_equal(got, NPR.segment_plane_counts(pts, 0.01, samples))


def test_plane_count_window_overflow_and_nonfinite(dev, monkeypatch):
    """Every pair inside the float32 window (points at |d| == thr of z = 0):
    every (batch, hypothesis) block goes through the float64 fix-up; planes
    with NaN coefficients count nothing.  The counts equal the oracle's."""
    n = 1_200_000
    rng = np.random.default_rng(3)
    pts = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), np.full(n, 0.01)], 1).astype(np.float32)
    pts[::3, 2] = -0.01
    planes = np.array([[0.0, 0.0, 1.0, 0.0], [0.0, 0.0, -1.0, 0.0], [0.0, 0.6, 0.8, 0.0]])
    x = torch.from_numpy(pts).to(dev)
    got = ops.plane_count(x, planes, 0.01)
    p64 = pts.astype(np.float64)
    ref = [int((np.abs(NPR.plane_dist(pl, p64)) < 0.01).sum()) for pl in planes]
    assert got.tolist() == ref
    assert (ops.plane_count_upper(x, planes, 0.01) >= got).all()
    bad = np.vstack([planes, [[np.nan, 0.0, 1.0, 0.0]]])
    got = ops.plane_count(x, bad, 0.01)
    assert got[:3].tolist() == ref and got[3] == 0
    assert ops.plane_count_upper(x, bad, 0.01)[3] == 0


@pytest.mark.parametrize("n,H,thr", [(1, 3, 0.01), (17, 5, 0.01), (1025, 33, 0.01), (100_003, 257, 0.01),
                                     (100_003, 257, 1e-7), (1_000_000, 1000, 0.01)])
def test_plane_count_counters_equal_oracle(dev, n, H, thr, monkeypatch):
    """The exact counts equal the oracle's, for
    ragged sizes (n not a multiple of the 1024-point batch, H not of the
    32-hypothesis chunk), degenerate hypotheses, and a threshold below the
    float32 window (lo < 0: the window holds the near-plane points)."""
    pts = S.planted_plane(max(n, 3), 61).numpy()[:n]
    rng = np.random.default_rng(n)
    samples = rng.integers(0, n, (H, 3)).astype(np.int32)
    samples[0] = [0, 0, 0]  # degenerate (collinear / repeated): -1
    planes = np.stack([NPR.triangle_plane(*pts[s].astype(np.float64)) for s in samples])
    x = torch.from_numpy(pts).to(dev)
    got = ops.plane_count(x, planes, thr)
    # segment_plane's sweeps (the culled one, the matrix-core one, the VALU
    # one; O3DX_RANSAC_UPPER forces each): upper bounds, -1 exactly where
    # degenerate; the matrix-core sweep counts only points within its
    # documented band |d| < thr + 2^-17 S_h (+ its own error, < 2^-17 S_h);
    # the VALU sweep only the float32 window's
    p64 = pts.astype(np.float64)
    S_h = np.abs(planes[:, :3]) @ np.abs(p64).max(0) + np.abs(planes[:, 3])
    for env in (None, "cull", "mfma2", "valu"):
        if env:
            monkeypatch.setenv("O3DX_RANSAC_UPPER", env)
        ub = ops.plane_count_upper(x, planes, thr)
        monkeypatch.delenv("O3DX_RANSAC_UPPER", raising=False)
        assert np.array_equal(ub < 0, got < 0) and (ub >= got).all()
        if env in ("valu", "cull") or (env is None and n >= 4096):
            assert (ub - got).max() <= max(8, n // 10000)  # only window points add
        elif n <= 100_003 and env:
            d = np.abs(p64 @ planes[:, :3].T + planes[:, 3])
            band = (d < thr + 2.0 ** -16 * S_h).sum(0)
            ok = got >= 0
            assert (ub[ok] <= band[ok]).all()
    ref = NPR.segment_plane_counts(pts, thr, samples) if n <= 100_003 else None
    if ref is not None:
        assert np.array_equal(got, ref)
    assert got[0] == -1


def test_mfma2_sweep_error_within_documented_bound(dev, monkeypatch):
    """The two-MFMA sweep's own error, |d_mfma - d| < 2^-17 S_h,
    checked directly: with the band switched off (O3DX_RANSAC_BAND_OFF, a test
    hook) the sweep counts |d_mfma| < thr, so for every hypothesis each point
    with |d| < thr - 2^-17 S_h must be counted and none with |d| >= thr +
    2^-17 S_h.  The cloud puts 2048 points per hypothesis at |d| = thr + u
    2^-16 S_h, u uniform in [-1, 1] (float64 distances of the float32 points),
    so about half of them lie outside that band on either side; with the band
    on, every float64 inlier is counted (ub >= exact)."""
    rng = np.random.default_rng(21)
    H, per, thr = 32, 2048, 0.01
    nrm = rng.normal(size=(H, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    off = rng.uniform(-0.3, 0.3, H)
    planes = np.concatenate([nrm, off[:, None]], 1)
    base = rng.uniform(-1, 1, (H, per, 3))
    S_est = np.abs(nrm).sum(1) + np.abs(off)  # |x| <= ~1.2 below: S_h from the cloud itself after
    pts = []
    for h in range(H):
        b = base[h] - ((base[h] @ nrm[h]) + off[h])[:, None] * nrm[h]  # on the plane
        u = rng.uniform(-1, 1, per)
        sgn = rng.choice([-1.0, 1.0], per)
        pts.append(b + (sgn * (thr + u * 2.0 ** -16 * S_est[h]))[:, None] * nrm[h])
    p32 = np.concatenate(pts).astype(np.float32)
    p64 = p32.astype(np.float64)
    S_h = np.abs(planes[:, :3]) @ np.abs(p64).max(0) + np.abs(planes[:, 3])
    d = np.abs(p64 @ planes[:, :3].T + planes[:, 3])  # (n, H)
    x = torch.from_numpy(p32).to(dev)
    monkeypatch.setenv("O3DX_RANSAC_UPPER", "mfma2")
    monkeypatch.setenv("O3DX_RANSAC_BAND_OFF", "1")
    got = ops.plane_count_upper(x, planes, thr)
    monkeypatch.delenv("O3DX_RANSAC_BAND_OFF")
    lo = (d < thr - 2.0 ** -17 * S_h).sum(0)
    hi = (d < thr + 2.0 ** -17 * S_h).sum(0)
    assert ((hi - lo) > per // 3).all()  # the test points straddle the bound
    assert (lo <= got).all() and (got <= hi).all(), (lo, got, hi)
    ub = ops.plane_count_upper(x, planes, thr)
    assert (ub >= (d < thr).sum(0)).all()


def _open3d_counts(p64, planes, thr):
    # Open3D's EvaluateRANSACBasedOnDistance predicate in its own order,
    # |(a x + c z) + (b y + d)| < thr, elementwise float64 (no fma)
    a, b, c, d = (planes[:, k][None, :] for k in range(4))
    x, y, z = (p64[:, k][:, None] for k in range(3))
    return (np.abs((a * x + c * z) + (b * y + d)) < thr).sum(0)


@pytest.mark.parametrize("layout", ["straddle", "cube_plane"])
def test_culled_sweep_bounds(dev, monkeypatch, layout):
    """The culled sweep (k_plane_upper_cull) counts |d32| < hi_h
    over the pairs its box test keeps: an upper bound of Open3D's predicate
    (the box test drops no pair that could count), tight outside the float32
    band.
    'straddle': 2048 points per hypothesis at |d| = thr + u 2^-22 S_h (inside
    the float32 band, scattered over the cloud's box: the float64 path runs
    for most chunks); 'cube_plane': a uniform cube with a planted plane and 300
    random hypotheses, the chunks' boxes both inside and outside the slabs.
    The dense exact count equals Open3D's predicate."""
    rng = np.random.default_rng(23)
    thr = 0.01
    if layout == "straddle":
        H, per = 32, 2048
        nrm = rng.normal(size=(H, 3))
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        off = rng.uniform(-0.3, 0.3, H)
        planes = np.concatenate([nrm, off[:, None]], 1)
        S_est = np.abs(nrm).sum(1) + np.abs(off)
        pts = []
        for h in range(H):
            b = rng.uniform(-1, 1, (per, 3))
            b = b - ((b @ nrm[h]) + off[h])[:, None] * nrm[h]
            u = rng.uniform(-1, 1, per)
            sgn = rng.choice([-1.0, 1.0], per)
            pts.append(b + (sgn * (thr + u * 2.0 ** -22 * S_est[h]))[:, None] * nrm[h])
        p32 = np.concatenate(pts).astype(np.float32)
    else:
        n = 200_000
        p32 = rng.uniform(0, 1, (n, 3)).astype(np.float32)
        on = rng.uniform(size=n) < 0.2
        p32[on, 2] = (0.5 + 0.002 * rng.normal(size=on.sum())).astype(np.float32)
        idx = rng.integers(0, n, (300, 3))
        a, b, c = (p32[idx[:, k]].astype(np.float64) for k in range(3))
        nrm = np.cross(b - a, c - a)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        planes = np.concatenate([nrm, -np.sum(nrm * a, 1, keepdims=True)], 1)
    p64 = p32.astype(np.float64)
    S_h = np.abs(planes[:, :3]) @ np.abs(p64).max(0) + np.abs(planes[:, 3])
    d = np.abs(p64 @ planes[:, :3].T + planes[:, 3])
    g = 6 * 2.0 ** -24 * S_h + 2.0 ** -20 * thr
    lim = (thr + g).astype(np.float32).astype(np.float64)
    lim = np.where(lim < thr + g, np.nextafter(lim.astype(np.float32), np.float32(np.inf)).astype(np.float64), lim)
    x = torch.from_numpy(p32).to(dev)
    monkeypatch.setenv("O3DX_RANSAC_UPPER", "cull")
    ub = ops.plane_count_upper(x, planes, thr)  # segment_plane's sweep
    ref = _open3d_counts(p64, planes, thr)
    assert (ub >= ref).all()
    if layout != "straddle":  # (straddle puts its points in the band on purpose)
        assert (ub - ref).max() <= max(8, len(p32) // 10000)
    else:  # the band points count: no more than the float32 limit (+ its error) lets through
        assert (ub <= (d < lim + g).sum(0)).all()
    if layout == "straddle":  # each hypothesis' own points straddle thr: about half are inliers
        own = np.array([_open3d_counts(p64[h * per:(h + 1) * per], planes[h:h + 1], thr)[0] for h in range(H)])
        assert ((own > per // 4) & (own < 3 * per // 4)).all()
    monkeypatch.delenv("O3DX_RANSAC_UPPER")
    assert np.array_equal(ops.plane_count(x, planes, thr), ref)  # the dense exact count agrees


@pytest.mark.parametrize("n", [1_000_000])
def test_c2_pipeline_full_mantissa_coordinates(dev, n):
    """The C2 step (one-call voxel_down_sample + KNN30 normals on the voxel
    table) on coordinates with full float32 mantissas and an offset origin —
    unlike synthetic.uniform_cube's 2^-24 grid, where the float64 moments are
    exact in any summation order — so the stencil-order sums meet
    non-representable partial sums: reps bit-exact, every normal row within
    1e-5 of the oracle, neighbour sets bit-exact."""
    u = S.uniform_cube(n, 77).double()
    pts = (u * 3.7 + torch.tensor([-1.234567, 0.3141593, 2.7182818], dtype=torch.float64)).float()
    p = pts.numpy()
    assert np.mean(np.abs(p.view(np.int32)) & 0xFF != 0) > 0.9  # low mantissa bits in use
    vs = S.voxel_size_for(n) * 3.7
    x = pts.to(dev)
    f = ops.voxel_down_sample_normals(x, vs, knn=30)
    a = ops.voxel_down_sample(x, vs, keep_grid=True)
    with DebugNeighbors(n, 30, dev) as dn:
        two = ops.estimate_normals(a["rep_xyz"], knn=30, voxel_grid=a["voxel_grid"])
    assert torch.equal(f["rep_idx"], a["rep_idx"]) and torch.equal(f["normals"], two)
    rep = f["rep_idx"].cpu().numpy()
    assert np.array_equal(rep, O.voxel_down_sample(p, vs))
    reps = p[rep]
    m = len(reps)
    assert_normals(f["normals"].cpu().numpy(), O.estimate_normals(reps, O.KNN, 30), reps, k=30,
                   what="c2_full_mantissa_1m")
    assert_neighbour_sets(dn.ids()[:m], reps, 30, "c2_full_mantissa_1m")


def test_grid_radix_path_equals_counting_path(dev, monkeypatch):
    """A surface cloud's fine grid over a large cell array is sorted by a
    stable radix sort of the cell keys (grid.hip, no atomics on the cell
    array, and a large cloud's surface test runs on a 1/8 sample); the
    counting path with the full count (O3DX_GRID_ATOMIC) gives the same
    normals and k-th-distance bounds bit for bit, the ICP target's
    registration the same T, and the blocked spatial sort the same rows."""
    pts = S.box_surface(5_000_000, 61).to(dev)
    src = S.apply_transform(S.box_surface(2_000_000, 62), S.rigid_transform()).to(dev)
    runs = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("O3DX_GRID_ATOMIC", env)
        nrm, kd2 = ops.estimate_normals(pts, knn=30, return_kdist=True)
        tgt = ops.ICPTarget(pts, nrm, 0.02)
        s4 = ops.spatial_sort(src)
        reg = tgt.register(s4, max_iteration=5, relative_fitness=0.0, relative_rmse=0.0)
        runs.append((nrm.cpu(), kd2.cpu(), reg["transformation"], s4.cpu()))
    a, b = runs
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert np.array_equal(a[2], b[2])
    # the spatial sort's order follows its grid's cell size (the sampled
    # surface test may pick another one): the same rows, each exactly once
    ia, ib = a[3][:, 3].contiguous().view(torch.int32), b[3][:, 3].contiguous().view(torch.int32)
    assert torch.equal(a[3][torch.argsort(ia)], b[3][torch.argsort(ib)])
    assert torch.equal(torch.sort(ia).values, torch.arange(ia.numel(), dtype=torch.int32))
