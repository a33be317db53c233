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
