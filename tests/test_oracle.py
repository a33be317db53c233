"""CPU: the oracle (test-only checker) against the reference's own golden
vectors, an independent numpy restatement, scipy and numpy.linalg."""
import os

import numpy as np
import pytest
from scipy.spatial import cKDTree

from oracle import np_restate as NPR
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_torch_branch.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


def test_bunny_voxel_counts(bunny):
    # M = 3,017 @ 0.005 and 751 @ 0.01 on data/bunny.pcd
    assert len(O.voxel_down_sample(bunny, 0.005)) == 3017
    assert len(O.voxel_down_sample(bunny, 0.01)) == 751


@pytest.mark.parametrize("vs", [0.003, 0.005, 0.02])
def test_voxel_cpp_vs_numpy(bunny, vs):
    assert np.array_equal(O.voxel_down_sample(bunny, vs), NPR.voxel_down_sample(bunny, vs))


def test_voxel_trace_consistency(bunny):
    rep, vop, cub = O.voxel_down_sample(bunny, 0.005, trace=True)
    assert np.array_equal(cub.max(1), rep)               # idxmat.max(1) == representative
    assert np.array_equal(vop[rep], np.arange(len(rep)))  # each rep maps to its own row
    assert (cub >= -1).all() and (cub < len(bunny)).all()


def test_voxel_errors():
    x = np.random.rand(10, 3).astype(np.float32)
    with pytest.raises(RuntimeError):
        O.voxel_down_sample(x, 0.0)
    with pytest.raises(RuntimeError):
        O.voxel_down_sample(x * 1e6, 1e-10)
    for par in (False, True):
        with pytest.raises(RuntimeError):
            O.voxel_down_sample(x, -1.0, parallel=par)


@pytest.mark.parametrize("vs", [0.003, 0.005, 0.02])
def test_voxel_parallel_reps_equal_single_pass(bunny, vs):
    # oref_voxel_reps_parallel (used at >= 20M points) == the single pass
    assert np.array_equal(O.voxel_down_sample(bunny, vs, parallel=True), O.voxel_down_sample(bunny, vs, parallel=False))


def test_voxel_parallel_reps_equal_single_pass_large():
    # 3M points with duplicates and negative coordinates, ~1 point per voxel
    # down to many: every voxel's max index, in ascending order
    rng = np.random.default_rng(11)
    x = (rng.random((3_000_000, 3)) * 2 - 1).astype(np.float32)
    x[1::7] = x[::7][: len(x[1::7])]
    for vs in (0.01, 0.05, 0.4):
        a = O.voxel_down_sample(x, vs, parallel=True)
        b = O.voxel_down_sample(x, vs, parallel=False)
        assert len(a) > 1 and np.array_equal(a, b)
    assert len(O.voxel_down_sample(x[:0], 0.1, parallel=True)) == 0


def test_knn_sets_vs_scipy(bunny):
    q = bunny[::101]
    idx, d2, cnt = O.knn_search(bunny, q, O.KNN, 30)
    tree = cKDTree(bunny.astype(np.float64))
    dd, ii = tree.query(q.astype(np.float64), k=30)
    for a, b in zip(idx, ii):
        assert set(a) == set(b)


def test_fast_eigen_vs_eigh():
    rng = np.random.default_rng(0)
    A = rng.normal(size=(500, 3, 3))
    C = A @ A.transpose(0, 2, 1)
    cov6 = np.stack([C[:, 0, 0], C[:, 0, 1], C[:, 0, 2], C[:, 1, 1], C[:, 1, 2], C[:, 2, 2]], 1)
    v = O.fast_eigen3x3(cov6)
    for c, n in zip(C, v):
        w, U = np.linalg.eigh(c)
        assert min(np.abs(U[:, 0] - n).max(), np.abs(U[:, 0] + n).max()) < 1e-6
    # degenerate inputs: identity -> (0,0,1); zero -> zero vector
    out = O.fast_eigen3x3(np.array([[1, 0, 0, 1, 0, 1], [0, 0, 0, 0, 0, 0]], np.float64))
    assert np.allclose(out[0], [0, 0, 1]) and not out[1].any()


def test_normals_vs_numpy_restatement(bunny):
    pts = bunny.astype(np.float64)
    n = O.estimate_normals(bunny, O.KNN, 30)
    for i in range(0, len(bunny), 1201):
        idx = NPR.neighbours(pts, pts[i], 0, 30, 0)
        v, _ = NPR.smallest_eigvec(NPR.covariance(pts, idx))
        assert min(np.abs(v - n[i]).max(), np.abs(v + n[i]).max()) < 1e-8


def test_oracle_normals_match_reference_torch_normals(gold):
    """Pinned by the reference's own TorchNormals (cdist + SVD, k=16): same axis."""
    x = gold["x_normals"]
    ref = gold["torch_normals_k16"]
    got = O.estimate_normals(x, O.KNN, 16)
    err = np.minimum(np.abs(got - ref).max(1), np.abs(got + ref).max(1))
    assert err.max() <= 1e-5  # measured 5.9e-7: same kNN sets, float32 SVD rounding


def test_voxel_torch_branch_restatement(gold):
    """Pinned: the restatement of the reference's cuda VoxelDownsample branch
    reproduces its output exactly (indices and order)."""
    x, vs, ref = gold["x_voxel"], float(gold["torch_voxel_size"]), gold["torch_voxel_rep_idx"]
    rep = NPR.voxel_torch_hash(x, vs)
    key = NPR.torch_hash_keys(x, vs)
    # same hash groups in the same (ascending key) order; the member chosen
    # inside a group is unspecified in the reference (unstable torch.sort)
    assert np.array_equal(key[rep], key[ref])
    assert np.all(np.diff(key[ref]) > 0)


def test_ransac_batched_restatement(gold):
    plane, cnt = NPR.ransac_batched_fp32(gold["x_plane"], 0.01, gold["torch_ransac_samples"], 256)
    assert cnt == int(gold["torch_ransac_inliers"])
    np.testing.assert_allclose(plane, gold["torch_ransac_plane"], atol=1e-6)
    # Open3D-rule scoring of the same plane (float64, strict <) agrees to a few points
    pl = gold["torch_ransac_plane"]
    n64 = int((NPR.plane_dist(pl, gold["x_plane"].astype(np.float64)) < 0.01).sum())
    assert abs(n64 - cnt) <= 3


def test_ransac_sampler():
    s = O.ransac_samples(100, 3, 1000, 42)
    assert s.min() >= 0 and s.max() < 100
    assert all(len(set(r)) == 3 for r in s)
    assert np.array_equal(s, O.ransac_samples(100, 3, 1000, 42))


def test_segment_plane_oracle(bunny):
    s = O.ransac_samples(len(bunny), 3, 200, 3)
    plane, inl, counts, sums, best = O.segment_plane(bunny, 0.01, 3, 200, s)
    assert np.array_equal(counts[counts >= 0], NPR.segment_plane_counts(bunny, 0.01, s)[counts >= 0])
    d = NPR.plane_dist(NPR.triangle_plane(*bunny[s[best]].astype(np.float64)), bunny.astype(np.float64))
    assert np.array_equal(inl, np.nonzero(d < 0.01)[0])
    assert abs(np.linalg.norm(plane[:3]) - 1) < 1e-12
    with pytest.raises(RuntimeError):
        O.segment_plane(bunny[:2], 0.01, 3, 10, np.zeros((10, 3), np.int32))


def test_icp_oracle_recovers_transform():
    import torch  # noqa: F401  (synthetic uses torch on CPU)
    from open3dpypro import synthetic as S

    tgt = S.box_surface(20000, 1).numpy()
    Tgt = S.rigid_transform()
    src = S.apply_transform(S.box_surface(20000, 2), Tgt).numpy()
    tn = O.estimate_normals(tgt, O.KNN, 30)
    T, fit, rmse, corr = O.registration_icp(src, tgt, tn, 0.02, max_iteration=30)
    assert np.abs(T - np.linalg.inv(Tgt)).max() < 1e-4
    assert fit > 0.99 and len(corr) == int(round(fit * len(src)))


# ---------------------------------------------------------------------------
# The float64 boundary: the oracle takes float64 coordinates as Open3D does
# (oracle.py _f64); a float32 cloud is upcast exactly, so its results are the
# ones the float32 oracle gave (bunny: voxel counts, normals, RANSAC).
def test_oracle_float64_input_equals_float32_upcast(bunny):
    b64 = bunny.astype(np.float64)
    assert np.array_equal(O.voxel_down_sample(bunny, 0.005), O.voxel_down_sample(b64, 0.005))
    assert np.array_equal(O.estimate_normals(bunny, O.KNN, 30), O.estimate_normals(b64, O.KNN, 30))
    s = O.ransac_samples(len(bunny), 3, 100, 5)
    p32, i32 = O.segment_plane(bunny, 0.01, 3, 100, s)[:2]
    p64, i64 = O.segment_plane(b64, 0.01, 3, 100, s)[:2]
    assert np.array_equal(p32, p64) and np.array_equal(i32, i64)


def test_oracle_float64_keys_not_rounded():
    """A float64 cloud keeps its values: voxel keys of points straddling a
    voxel face that float32 rounding moves across it differ."""
    x = np.array([[500000.0, 0, 0], [500000.0 + 0.2 - 1e-9, 0, 0], [500000.0 + 0.2 + 1e-9, 0, 0]])
    rep = O.voxel_down_sample(x, 0.2, min_bound=x.min(0), max_bound=x.max(0))
    assert len(rep) == 2  # the float32 values are all 500000.0 or 500000.1875: one voxel
    assert len(O.voxel_down_sample(x.astype(np.float32), 0.2)) == 1


def test_icp_offset_conditioning():
    """Open3D's point-to-plane system on raw coordinates at a LAS-like offset:
    J = [p x n; n] with |p| ~ 5e5 makes the 6x6 normal matrix singular in
    float64, and the oracle's T becomes rounding noise (a permuted source
    moves it, it misses the motion by metres).  At a 1e4 m offset the same
    registration is well-posed (T stable to ~1e-9).  The float64 GPU parity
    tests (tests/test_gpu_f64.py test_f64_icp) therefore check the ~5e5 scan
    in its recentred frame and full-mantissa clouds at 1e4 m."""
    import torch  # noqa: F401
    from open3dpypro import synthetic as S

    n = 60_000
    M = S.rigid_transform(1.0, t=(0.2, -0.12, 0.08))
    perm = np.random.default_rng(0).permutation(n)
    spread = {}
    for name, off in (("1e4", (12345.678, 23456.789, 98.765)), ("las", S.LAS_OFFSET)):
        tgt = S.las_scene(n, seed=0, offset=off).numpy()
        src = S.las_scene(n, seed=1, T=M, offset=off).numpy()
        tn = O.estimate_normals(tgt, O.KNN, 30)
        kw = dict(max_iteration=30, relative_fitness=0, relative_rmse=0)
        T1 = O.registration_icp(src, tgt, tn, 0.8, **kw)[0]
        T2 = O.registration_icp(src[perm], tgt, tn, 0.8, **kw)[0]
        spread[name] = np.abs(T1 - T2).max()
    assert spread["1e4"] < 1e-7, spread
    assert spread["las"] > 1e-4, spread


# ---------------------------------------------------------------------------
# The glue around the hot path, pinned by the reference's OWN outputs
# (tests/golden/ref_glue.npz, written by `python tests/golden/make_golden.py
# glue` from /root/reference/open3dpypro/processors.py in this container):
# the test-side restatements (oracle/np_restate.py) AND the build's processors
# (open3dpypro.processors, on numpy / torch-CPU data: no GPU involved) must
# reproduce them bit for bit.
GLUE = os.path.join(os.path.dirname(__file__), "golden", "ref_glue.npz")
PN_CASES = ["np_f32", "np_f64", "np_f32_6col", "torch_f32", "torch_f64", "np_f32_antiparallel", "np_f64_parallel",
            "torch_f32_unnormalised"]


@pytest.fixture(scope="module")
def glue():
    return np.load(GLUE, allow_pickle=False)


def _pn_inputs(glue, case):
    import torch

    x = glue[f"pn_{case}_x"]
    return (torch.from_numpy(x.copy()) if case.startswith("torch") else x.copy()), [float(v) for v in
                                                                                   glue[f"pn_{case}_plane"]]


@pytest.mark.parametrize("case", PN_CASES)
def test_plane_normalize_restatement_vs_reference(glue, case):
    """np_restate.rotate_to_plane_ref == the reference's PlaneNormalize
    (processors.py:709-744) on its own recorded outputs: xyz and T bit-equal,
    in the data's dtype, the anti-parallel normal giving R = I."""
    data, plane = _pn_inputs(glue, case)
    xyz, T = NPR.rotate_to_plane_ref(data, plane)
    xyz = xyz.numpy() if hasattr(xyz, "numpy") else xyz
    T = T.numpy() if hasattr(T, "numpy") else T
    assert np.array_equal(xyz, glue[f"pn_{case}_out"][:, :3])
    assert np.array_equal(T.astype(np.float64), glue[f"pn_{case}_T"])
    if case.endswith("antiparallel"):
        assert np.array_equal(T[:3, :3], np.eye(3))


@pytest.mark.parametrize("case", PN_CASES)
def test_plane_normalize_processor_vs_reference(glue, case):
    """The build's Processors.PlaneNormalize == the reference's on the same
    inputs: the whole output (extra columns passed through) and forward_T."""
    from open3dpypro import Processors
    from open3dpypro.PointCloudMat import PointCloudMat, ShapeType

    data, plane = _pn_inputs(glue, case)
    st = ShapeType.XYZ if data.shape[1] == 3 else ShapeType.XYZRGB
    pn = Processors.PlaneNormalize(uuid="PlaneNormalize:glue", detection_uuid="det")
    out, _ = pn.validate([PointCloudMat(shape_type=st).build(data)], {"det": [plane]})
    got = out[0].data()
    got = got.numpy() if hasattr(got, "numpy") else got
    assert got.dtype == glue[f"pn_{case}_out"].dtype
    assert np.array_equal(got, glue[f"pn_{case}_out"])
    assert np.array_equal(np.asarray(pn.forward_T[0], np.float64), glue[f"pn_{case}_T"])


def test_plane_detection_flip_ema_restatement_vs_reference(glue):
    """np_restate.plane_flip_ref + ema_ref == the reference's PlaneDetection
    CPU branch (processors.py:640-650, 697) given the same segment_plane
    planes, over 3 frames, at alpha 0.1 and at the default alpha 0 (the
    published plane then stays [0, 0, 0, 0]); the torch branch's EMA over its
    own recorded per-frame planes (already d >= 0: the flip leaves them)."""
    for alpha in (0.1, 0.0):
        best = [0.0, 0.0, 0.0, 0.0]
        for i, pl in enumerate(glue["pd_planes"]):
            best = NPR.ema_ref(best, NPR.plane_flip_ref(pl), alpha)
            assert np.array_equal(np.asarray(best), glue[f"pd_cpu_meta_alpha{alpha}"][i])
    best = [0.0, 0.0, 0.0, 0.0]
    for i, pl in enumerate(glue["pdt_planes"]):
        pl = pl.astype(np.float32)  # the torch branch's plane is a float32 array: plane * alpha stays float32
        assert pl[3] >= 0 and np.array_equal(NPR.plane_flip_ref(pl), pl)
        best = NPR.ema_ref(best, NPR.plane_flip_ref(pl), 0.1)
        assert np.array_equal(np.asarray(best), glue["pdt_meta_alpha0.1"][i])


def test_plane_detection_processor_flip_ema_vs_reference(glue, monkeypatch):
    """The build's Processors.PlaneDetection flip + EMA == the reference's on
    the same segment_plane planes (injected on both sides: the RANSAC itself
    is pinned against the oracle by the GPU suite), 3 frames, alpha 0.1 and
    0: meta[uuid] bit-equal after every frame."""
    import torch

    from open3dpypro import Processors, ops, processors
    from open3dpypro.PointCloudMat import PointCloudMat, ShapeType

    monkeypatch.setattr(processors, "_xyz", lambda a: torch.as_tensor(np.asarray(a))[:, :3].float())
    for alpha in (0.1, 0.0):
        it = iter(glue["pd_planes"])
        monkeypatch.setattr(ops, "segment_plane", lambda *a, **k: (np.asarray(next(it), np.float64), None))
        pd = Processors.PlaneDetection(uuid="PlaneDetection:glue", distance_threshold=0.01, alpha=alpha, seed=1)
        frames = glue["pd_frames"]
        mats = [PointCloudMat(shape_type=ShapeType.XYZ).build(frames[0].copy())]
        pd.validate(mats, {}, run=False)
        for i, f in enumerate(frames):
            meta = {}
            pd.forward_raw([f.copy()], [], meta)
            assert np.array_equal(np.asarray(meta[pd.uuid][0]), glue[f"pd_cpu_meta_alpha{alpha}"][i])


def test_random_sample_radius_selection_vs_reference(glue):
    """RandomSample (processors.py:320-365) and RadiusSelection (:367-416):
    the build's processors on numpy and torch-CPU data, with the reference's
    seeds, equal the reference's recorded outputs (same RNG draws; the numpy
    radius branch returns float64 xyz, the torch one every column)."""
    import torch

    from open3dpypro import Processors

    x = glue["rs_x"]
    rs = Processors.RandomSample(n_samples=1000)
    np.random.seed(5)
    assert np.array_equal(rs.forward_raw([x.copy()])[0], glue["rs_np_out"])
    torch.manual_seed(5)
    assert np.array_equal(rs.forward_raw([torch.from_numpy(x.copy())])[0].numpy(), glue["rs_torch_out"])
    r = float(glue["rsel_radius"])
    sel = Processors.RadiusSelection(radius=r)
    got = sel.forward_raw([x.copy()])[0]
    assert got.dtype == np.float64 and np.array_equal(got, glue["rsel_np_out"])
    assert np.array_equal(sel.forward_raw([torch.from_numpy(x.copy())])[0].numpy(), glue["rsel_torch_out"])
    q = x[:, :3].astype(np.float64)  # the restated mask (PointCloud.py:264-265)
    assert np.array_equal(q[(q[:, 0] ** 2 + q[:, 1] ** 2 + q[:, 2] ** 2) ** 0.5 <= r], glue["rsel_np_out"])


def test_icp_update_sincos_tolerance():
    """The library's ICP update (icp.hip vec6_to_mat4 via det_sincos, the same
    bits on host and device) against Open3D's std::sin / std::cos (the
    oracle's registration_icp, o3d_restate.cpp): per update the rotation
    entries differ by at most ~2 ulp (test_host.py
    test_icp_solve_rotation_angles_host); over 30 iterations of C3's problem
    the loop driven by the library's update stays within 1e-12 of the
    oracle's T with the same fitness, i.e. the every-ICP-test bar (T within
    1e-5 of the oracle) is met with 7 orders of magnitude to spare.
    Tolerance statement: T parity is asserted at 1e-5, the
    sin/cos choice accounts for <= 1e-12 of it."""
    import open3dpypro as o3p
    from open3dpypro import synthetic as S
    n = 20000
    tgt = S.box_surface(n, 1).numpy()
    src = S.apply_transform(S.box_surface(n, 2), S.rigid_transform()).numpy()
    tn = O.estimate_normals(tgt, O.KNN, 30).astype(np.float32)
    Tr, fr, rr, _ = O.registration_icp(src, tgt, tn, 0.02, max_iteration=30, relative_fitness=0, relative_rmse=0)
    T = np.eye(4)
    for _ in range(30):
        T = o3p.ops.icp_update(O.icp_accumulate(src, tgt, tn, 0.02, T), T)
    sums = O.icp_accumulate(src, tgt, tn, 0.02, T)
    assert np.abs(T - Tr).max() < 1e-12
    assert sums[28] / n == fr and abs(np.sqrt(sums[29] / sums[28]) - rr) < 1e-12
