"""GPU: the float64 boundary (include/o3dx.h "float64 boundary", VERDICT r4
item 1).  Open3D keeps points as float64 (reference PointCloud.py:99-102) and
computes voxel keys (:338-341), kNN distances and normals (:68-73), RANSAC
distances (:75-77) and ICP on them.  A LAS-like scan at a ~5e5 m offset with
full-mantissa float64 coordinates is not float32-representable: PointCloud
keeps it in float64 and runs the o3dx_*_f64 kernels, which must give the
oracle's results on the same float64 input (the oracle takes float64 as
Open3D does; oracle/oracle.py _f64).
"""
import numpy as np
import pytest
import torch

from open3dpypro import PointCloud, ops, synthetic as S
from open3dpypro.PointCloud import _f32_exact
from open3dpypro.params import KDTreeSearchParamHybrid, KDTreeSearchParamRadius
from oracle import oracle as O
from parity import DebugNeighbors, assert_neighbour_sets, assert_normals

pytestmark = pytest.mark.gpu
N = 1_000_000
VS = 0.2  # metres: ~6 points per occupied voxel on the scan's surfaces


@pytest.fixture(scope="module")
def las(dev):
    return S.las_scene(N, seed=0, device=dev)


@pytest.fixture(scope="module")
def las_np(las):
    return las.cpu().numpy()


def test_las_cloud_is_not_float32(las_np):
    """The test cloud is what the verdict asks for: float32 rounding moves it."""
    assert las_np.dtype == np.float64 and np.abs(las_np).max() > 4e5
    moved = las_np.astype(np.float32).astype(np.float64) != las_np
    assert moved.mean() > 0.99


def test_pointcloud_dispatch(las_np):
    pc = PointCloud(las_np)
    assert pc._wide and pc._hot_points().dtype == torch.float64
    assert np.array_equal(pc.get_points(), las_np)
    mn, mx = pc.get_aabb()
    assert np.array_equal(mn, las_np.min(0)) and np.array_equal(mx, las_np.max(0))
    exact = PointCloud(las_np.astype(np.float32).astype(np.float64))  # float32 values: the fast path
    assert not exact._wide and exact._hot_points().dtype == torch.float32
    sub = pc.select_by_bool(np.arange(N) % 3 == 0)
    assert sub._wide and np.array_equal(sub.get_points(), las_np[::3])


def test_f64_voxel_reps_and_trace_exact(las, las_np):
    out = ops.voxel_down_sample(las, VS, trace=True)
    rep, vop, cub = O.voxel_down_sample(las_np, VS, trace=True)
    assert np.array_equal(out["rep_idx"].cpu().numpy(), rep)
    assert np.array_equal(out["voxel_of_point"].cpu().numpy(), vop)
    assert np.array_equal(out["cubic_id"].cpu().numpy(), cub)
    assert torch.equal(out["rep_xyz"], las[out["rep_idx"].long()])
    # the float32 path on the rounded cloud decides differently: the float64 path is needed
    r32 = O.voxel_down_sample(las_np.astype(np.float32), VS)
    assert not np.array_equal(r32, rep)


def test_f64_voxel_down_sample_api(las_np):
    pc = PointCloud(las_np)
    ds = pc.voxel_down_sample(VS)
    rep = O.voxel_down_sample(las_np, VS)
    assert np.array_equal(ds.get_points(), las_np[rep])
    cloud, idxmat, vec = pc.voxel_down_sample_and_trace(VS)
    _, _, cub = O.voxel_down_sample(las_np, VS, trace=True)
    assert np.array_equal(idxmat, cub) and len(vec) == len(rep)


def test_f64_normals_knn30(las, las_np):
    """estimate_normals(KNN30) on the 1M-point scan: every row within 1e-5 of
    the oracle (Open3D's sequential float64 raw moments in (d^2, index)
    order), neighbour sets bit-exact."""
    with DebugNeighbors(N, 30, las.device) as dn:
        got = ops.estimate_normals(las, knn=30).cpu().numpy()
    ref = O.estimate_normals(las_np, O.KNN, 30)
    assert_normals(got, ref, las_np, k=30, what="f64_las_knn30")
    assert_neighbour_sets(dn.ids(), las_np, 30, "f64_las_knn30")


@pytest.mark.parametrize("handoff", ["wave", "wave_keep1", "lane"])
@pytest.mark.parametrize("k", [30, 16, 5])
def test_f64_normals_tiles_equal_lane_form(las, monkeypatch, k, handoff):
    """The float64 LDS tiles (frame-distance selection, exact (d^2, index)
    order, sequential float64 moments) give the lane-per-query form's normals
    bit for bit (O3DX_F64_NO_TILES=1), hand-offs included — the tiles'
    hand-offs served a wave per query (k_normals_knn64_wave, default) or a lane
    each (O3DX_F64_NO_WAVE) — and the same k-th distance bounds."""
    if handoff == "lane":
        monkeypatch.setenv("O3DX_F64_NO_WAVE", "1")
    if handoff == "wave_keep1":  # the wave form hands nearly every query on
        monkeypatch.setenv("O3DX_F64_WAVE_KEEP", "1")
    a, kd_a = ops.estimate_normals(las, knn=k, return_kdist=True)
    monkeypatch.delenv("O3DX_F64_NO_WAVE", raising=False)
    monkeypatch.delenv("O3DX_F64_WAVE_KEEP", raising=False)
    monkeypatch.setenv("O3DX_F64_NO_TILES", "1")
    b, kd_b = ops.estimate_normals(las, knn=k, return_kdist=True)
    assert torch.equal(a, b)
    assert torch.equal(kd_a, kd_b)


def test_f64_normals_tiles_reps_vs_oracle(las_np, dev):
    """The tiles on the voxel representatives of the scan (5 cm-ish spacing,
    the f64_las bench leg's shape) against the oracle, sets bit-exact."""
    reps = las_np[O.voxel_down_sample(las_np, 0.05)]
    x = torch.as_tensor(reps, device=dev)
    with DebugNeighbors(len(reps), 30, dev) as dn:
        got = ops.estimate_normals(x, knn=30).cpu().numpy()
    assert_normals(got, O.estimate_normals(reps, O.KNN, 30), reps, k=30, what="f64_las_reps_tiles")
    assert_neighbour_sets(dn.ids(), reps, 30, "f64_las_reps_tiles")


def test_f64_normals_pointcloud_reps(las_np):
    """The pipeline of the reference (voxel_down_sample -> estimate_normals)
    through the drop-in API on the float64 scan."""
    pc = PointCloud(las_np).voxel_down_sample(VS).estimate_normals()
    reps = las_np[O.voxel_down_sample(las_np, VS)]
    assert_normals(pc.get_normals(), O.estimate_normals(reps, O.KNN, 30), reps, k=30, what="f64_las_reps")


@pytest.mark.parametrize("mode", ["hybrid", "radius"])
def test_f64_normals_hybrid_radius(dev, mode):
    n = 200_000
    x = S.las_scene(n, seed=3, device=dev)
    xn = x.cpu().numpy()
    r = 0.3
    if mode == "hybrid":
        pc = PointCloud(xn).estimate_normals(param=KDTreeSearchParamHybrid(radius=r, max_nn=30))
        ref = O.estimate_normals(xn, O.HYBRID, 30, r)
        assert_normals(pc.get_normals(), ref, xn, mode=O.HYBRID, k=30, radius=r, what="f64_hybrid")
    else:
        pc = PointCloud(xn).estimate_normals(param=KDTreeSearchParamRadius(radius=r))
        ref = O.estimate_normals(xn, O.RADIUS, 0, r)
        assert_normals(pc.get_normals(), ref, xn, mode=O.RADIUS, k=0, radius=r, what="f64_radius")


def test_f64_knn_search(las_np, dev):
    pc = PointCloud(las_np)
    q = las_np[::997][:512] + 0.01
    idx, d2, cnt = ops.knn_search(pc._hot_points(), torch.as_tensor(q, device=dev), knn=16)
    ri, rd, rc = O.knn_search(las_np, q, O.KNN, 16)
    assert np.array_equal(idx.cpu().numpy(), ri) and np.array_equal(d2.cpu().numpy(), rd)
    k, ii, dd = pc.get_KDtree().search_knn_vector_3d(las_np[12345], 8)
    assert k == 8 and ii[0] == 12345 and dd[0] == 0.0


def test_f64_segment_plane(las, las_np):
    """segment_plane on the float64 scan: every hypothesis count exact, the
    plane and the inliers identical to the oracle's SegmentPlane."""
    samples = O.ransac_samples(N, 3, 1000, 11)
    plane, inl = ops.segment_plane(las, 0.05, 3, 1000, samples=samples)
    rplane, rinl, counts, _, best = O.segment_plane(las_np, 0.05, 3, 1000, samples)
    assert np.array_equal(inl.cpu().numpy(), rinl)
    # the refit (GetPlaneFromPoints) sums in a different order than Open3D's
    # sequential loop; d = -n.c carries |c| ~ 5e5 times any change of n, so
    # the planes are compared as geometry: normals within 1e-9 and the two
    # planes within 1 um of each other over the whole scene box
    np.testing.assert_allclose(plane[:3], rplane[:3], atol=1e-9)
    lo, hi = las_np.min(0), las_np.max(0)
    corners = np.array([[a, b, c] for a in (lo[0], hi[0]) for b in (lo[1], hi[1]) for c in (lo[2], hi[2])])
    gap = np.abs((corners @ plane[:3] + plane[3]) - (corners @ rplane[:3] + rplane[3]))
    assert gap.max() < 1e-6, gap.max()
    planes = ops.planes_from_samples(las_np[samples.reshape(-1)].reshape(-1, 3, 3), 3)
    assert np.array_equal(ops.plane_count(las, planes[:64], 0.05), counts[:64])
    pc_plane, pc_inl = PointCloud(las_np).segment_plane(0.05, 3, 1000, samples=samples)
    assert np.array_equal(np.asarray(pc_inl), rinl)


# ICP: Open3D's point-to-plane normal matrix on raw coordinates has entries
# ~|p|^2 against ~1: at a ~5e5 m offset its condition (~1e22) exceeds
# float64's reach and the oracle's own T is rounding noise (permuting the
# source moves it by 6e-2 and it misses the motion by ~300 m: tests/test_oracle.py
# test_icp_offset_conditioning).  Parity is therefore checked where the
# problem is well-posed: full-mantissa float64 clouds at a 1e4 m offset, and
# the ~5e5 m scan in the recentred frame users register it in.
@pytest.mark.parametrize("frame", ["offset_1e4", "las_recentred"])
def test_f64_icp(dev, frame):
    n = 1_000_000
    M = S.rigid_transform(1.0, t=(0.2, -0.12, 0.08))
    off = (12345.678, 23456.789, 98.765) if frame == "offset_1e4" else S.LAS_OFFSET
    tgt = S.las_scene(n, seed=0, offset=off, device=dev)
    src = S.las_scene(n, seed=1, T=M, offset=off, device=dev)
    if frame == "las_recentred":
        c = tgt.mean(0)
        tgt, src = tgt - c, src - c
    assert not _f32_exact(src.cpu().numpy())
    tn = ops.estimate_normals(tgt, knn=30)
    res = ops.registration_icp(src, tgt, tn, 0.8, max_iteration=30, relative_fitness=0, relative_rmse=0,
                               return_corr=False)
    T, fit, rmse, _ = O.registration_icp(src.cpu().numpy(), tgt.cpu().numpy(), tn.cpu().numpy(), 0.8,
                                         max_iteration=30, relative_fitness=0, relative_rmse=0)
    np.testing.assert_allclose(res["transformation"], T, atol=1e-5)
    assert abs(res["fitness"] - fit) < 1e-6 and abs(res["inlier_rmse"] - rmse) < 1e-6
    assert fit == 1.0


def test_f64_registration_icp_api(dev):
    n = 200_000
    off = (12345.678, 23456.789, 98.765)
    M = S.rigid_transform(1.0, t=(0.2, -0.12, 0.08))
    tgt = PointCloud(S.las_scene(n, seed=0, offset=off).numpy()).estimate_normals()
    src = PointCloud(S.las_scene(n, seed=1, T=M, offset=off).numpy())
    assert src._wide and tgt._wide
    r = src.registration_icp(tgt, 0.8, max_iteration=30, relative_fitness=0, relative_rmse=0)
    T, fit, _, corr = O.registration_icp(src.get_points(), tgt.get_points(), tgt.get_normals(), 0.8,
                                         max_iteration=30, relative_fitness=0, relative_rmse=0)
    np.testing.assert_allclose(r.transformation, T, atol=1e-5)
    assert abs(r.fitness - fit) < 1e-6 and len(r.correspondence_set) == len(corr)


def test_f64_pcd_f8_roundtrip(tmp_path, las_np):
    """A PCD with F8 coordinates (DATA binary) keeps its float64 values."""
    pts = las_np[:5000]
    path = tmp_path / "f8.pcd"
    hdr = ("# .PCD v0.7\nVERSION 0.7\nFIELDS x y z\nSIZE 8 8 8\nTYPE F F F\nCOUNT 1 1 1\n"
           f"WIDTH {len(pts)}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {len(pts)}\nDATA binary\n")
    path.write_bytes(hdr.encode() + np.ascontiguousarray(pts, "<f8").tobytes())
    pc = PointCloud().read_pcd(str(path))
    assert pc._wide and np.array_equal(pc.get_points(), pts)


@pytest.mark.parametrize("form", ["unsorted", "sorted_f64"])
@pytest.mark.parametrize("skip", ["1", "0"])
def test_f64_icp_target_register_forms(dev, monkeypatch, form, skip):
    """ICPTarget(float64).register on an unsorted float64 source of > 200k
    points with no absmax (the source bounds run through the float64 AABB
    scratch) and on a spatial_sort_f64 source: the same T, fitness and rmse as
    registration_icp_f64, with and without the skip proof."""
    monkeypatch.setenv("O3DX_ICP_SKIP", skip)
    n = 300_000
    off = (12345.678, 23456.789, 98.765)
    M = S.rigid_transform(1.0, t=(0.2, -0.12, 0.08))
    tgt = S.las_scene(n, seed=0, offset=off, device=dev)
    src = S.las_scene(n, seed=1, T=M, offset=off, device=dev)
    tn = ops.estimate_normals(tgt, knn=30)
    ref = ops.registration_icp(src, tgt, tn, 0.8, max_iteration=20, relative_fitness=0, relative_rmse=0,
                               return_corr=False)
    target = ops.ICPTarget(tgt, tn, 0.8)
    s = src if form == "unsorted" else ops.spatial_sort_f64(src)
    res = target.register(s, max_iteration=20, relative_fitness=0, relative_rmse=0)
    np.testing.assert_allclose(res["transformation"], ref["transformation"], atol=1e-9)
    assert abs(res["fitness"] - ref["fitness"]) < 1e-12
    assert abs(res["inlier_rmse"] - ref["inlier_rmse"]) < 1e-9


def test_f64_icp_target_sorted_dtype_mismatch(dev):
    """A sorted source whose dtype does not match the target's raises instead
    of casting (the index column's encoding differs between the two forms)."""
    n = 5000
    off = (12345.678, 23456.789, 98.765)
    tgt64 = S.las_scene(n, seed=0, offset=off, device=dev)
    tn = ops.estimate_normals(tgt64, knn=30)
    t64 = ops.ICPTarget(tgt64, tn, 0.8)
    src32 = (S.las_scene(n, seed=1, offset=off, device=dev) - torch.tensor(off, dtype=torch.float64,
                                                                          device=dev)).float()
    with pytest.raises(RuntimeError, match="sorted source"):
        t64.register(ops.spatial_sort(src32), max_iteration=2)
    tgt32 = (tgt64 - torch.tensor(off, dtype=torch.float64, device=dev)).float()
    t32 = ops.ICPTarget(tgt32, ops.estimate_normals(tgt32, knn=30), 0.8)
    with pytest.raises(RuntimeError, match="sorted source"):
        t32.register(ops.spatial_sort_f64(src32.double()), max_iteration=2)


def test_f64_registration_icp_warns_at_georeferenced_offset():
    """registration_icp on a raw georeferenced scan (the
    ~5e5 m offset) warns that the point-to-plane system is ill-conditioned
    there (for Open3D as well) and names the remedy; the 1e4 m case does not."""
    n = 20_000
    src = PointCloud(S.las_scene(n, seed=1).numpy())
    tgt = PointCloud(S.las_scene(n, seed=0).numpy()).estimate_normals()
    with pytest.warns(RuntimeWarning, match="re-centred frame"):
        src.registration_icp(tgt, 0.8, max_iteration=2)
    off = (12345.678, 23456.789, 98.765)
    s2 = PointCloud(S.las_scene(n, seed=1, offset=off).numpy())
    t2 = PointCloud(S.las_scene(n, seed=0, offset=off).numpy()).estimate_normals()
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        s2.registration_icp(t2, 0.8, max_iteration=2)
