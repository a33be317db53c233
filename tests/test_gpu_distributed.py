"""GPU: the sharded ICP driver with the HIP accumulate kernel as each rank's
`accumulate` — two ranks (gloo rendezvous on 127.0.0.1) sharing the one GPU of
the test box, against the single-process device loop and the oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from open3dpypro import distributed as D
from open3dpypro import ops, synthetic as S

from parity import assert_normals
from test_distributed import spawn

pytestmark = pytest.mark.gpu


def _clouds():
    tgt = S.box_surface(200_000, 1).numpy()
    src = S.box_surface(200_000, 2).numpy()
    Tg = S.rigid_transform()
    src = (src.astype(np.float64) @ Tg[:3, :3].T + Tg[:3, 3]).astype(np.float32)
    return src, tgt


def _rank(rank, world):
    dev = torch.device("cuda:0")
    src, tgt = _clouds()
    t = torch.from_numpy(tgt).to(dev)
    tn = ops.estimate_normals(t, knn=30)
    target = ops.ICPTarget(t, tn, 0.02)
    a, b = D.shard_range(len(src), world, rank)
    return D.registration_icp_sharded(torch.from_numpy(src[a:b]).to(dev), target, max_iteration=20)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_icp_on_device_matches_single(world):
    """ICP with the source sharded over ranks (HIP kernels, fx moments summed
    over the ranks): T, fitness and rmse the same bits as the single-GPU
    o3dx_registration_icp_point_to_plane, and within 1e-5 of the oracle."""
    res = spawn(_rank, world=world)
    src, tgt = _clouds()
    dev = torch.device("cuda:0")
    t = torch.from_numpy(tgt).to(dev)
    tn = ops.estimate_normals(t, knn=30)
    one = ops.registration_icp(torch.from_numpy(src).to(dev), t, tn, 0.02, max_iteration=20, return_corr=False)
    for T, f, r in res:
        assert np.array_equal(T, one["transformation"]) and f == one["fitness"] and r == one["inlier_rmse"]
    To, fo, ro = O.registration_icp(src, tgt, tn.cpu().numpy(), 0.02, max_iteration=20)[:3]
    assert np.abs(one["transformation"] - To).max() < 1e-5 and abs(one["fitness"] - fo) < 1e-5


def _c4_rank(rank, world):
    dev = torch.device("cuda:0")
    pts = S.uniform_cube(400_000, 33)
    g = torch.arange(rank, pts.shape[0], world, dtype=torch.int64)
    rg, rx, nrm = D.voxel_normals_slabs(pts[g].to(dev), g.to(dev), 0.02, knn=30)
    return rg, nrm


def test_c4_slabs_on_device_match_single():
    """Two ranks (gloo rendezvous, shared GPU) run the slab decomposition with
    the HIP voxel / normals kernels: reps bit-exact, normals bit-identical to
    the single-GPU call (results independent of the GPU count)
    and within 1e-5 of the oracle on every row."""
    res = spawn(_c4_rank)
    dev = torch.device("cuda:0")
    pts = S.uniform_cube(400_000, 33).to(dev)
    mn, mx = ops.aabb(pts)
    out = ops.voxel_down_sample(pts, 0.02, mn, mx)
    ref = ops.estimate_normals(out["rep_xyz"], knn=30).cpu().numpy()
    g = np.concatenate([r[0] for r in res])
    nn = np.concatenate([r[1] for r in res])
    o = np.argsort(g)
    assert np.array_equal(g[o], out["rep_idx"].cpu().numpy().astype(np.int64))
    assert np.array_equal(nn[o], ref)
    reps = out["rep_xyz"].cpu().numpy()
    assert_normals(nn[o], O.estimate_normals(reps, O.KNN, 30), reps, k=30, what="c4_slabs_2ranks_device")


def _clustered_rank(rank, world):
    from test_distributed import CL_VS, _clustered_cloud
    dev = torch.device("cuda:0")
    pts, _ = _clustered_cloud(world)
    g = torch.arange(rank, len(pts), world, dtype=torch.int64)
    rg, rx, nrm = D.voxel_normals_slabs(torch.from_numpy(pts)[g].to(dev), g.to(dev), CL_VS, knn=30)
    return rg, nrm


def test_c4_slabs_clustered_on_device():
    """The clustered cloud whose far-from-face reps need a wider halo: the
    device kernels' k-th-distance bounds drive the halo check, and the slab
    result equals the single-GPU one bit for bit."""
    from test_distributed import CL_VS, _clustered_cloud
    res = spawn(_clustered_rank)
    dev = torch.device("cuda:0")
    pts, _ = _clustered_cloud(2)
    x = torch.from_numpy(pts).to(dev)
    mn, mx = ops.aabb(x)
    out = ops.voxel_down_sample(x, CL_VS, mn, mx)
    ref = ops.estimate_normals(out["rep_xyz"], knn=30).cpu().numpy()
    g = np.concatenate([r[0] for r in res])
    nn = np.concatenate([r[1] for r in res])
    o = np.argsort(g)
    assert np.array_equal(g[o], out["rep_idx"].cpu().numpy().astype(np.int64))
    assert np.array_equal(nn[o], ref)


def _presorted_share(pts, vs, rank, world):
    """the rows of this rank's x-slab (a spatially tiled dataset), ascending"""
    mn, mx = ops.aabb(pts)
    keys = D.slab_bounds(mn, mx, vs, world)
    kx = torch.floor((pts[:, 0].double() - float(mn[0])) / vs).to(torch.int64)
    return torch.nonzero((kx >= keys[rank]) & (kx < keys[rank + 1])).flatten()


def _hollow_cloud():
    """1.2M uniform points with the band |x - 0.5| < 0.12 thinned to 1 in 200:
    over 2 slabs (face at x = 0.5) the reps near the face have their k-th
    neighbour ~7 voxels away, so the first halos (3, 6 voxel layers) fail the
    proof and the halo widens; the slabs stay dense enough for the deferred
    step's voxel tables."""
    n = 1_200_000
    pts = S.uniform_cube(n, 46)
    keep = ((pts[:, 0] - 0.5).abs() >= 0.12) | (torch.arange(n) % 200 == 0)
    return pts[keep].contiguous(), S.voxel_size_for(n)


def _hollow_rank(rank, world):
    dev = torch.device("cuda:0")
    pts, vs = _hollow_cloud()
    x = pts.to(dev)
    g = _presorted_share(x, vs, rank, world)
    tl = {}
    rg, rx, nrm = D.voxel_normals_slabs(x[g].contiguous(), g, vs, knn=30, presorted=True, timings=tl)
    return rg, nrm, sorted(tl)


def test_c4_slabs_presorted_deferred_widens_halo():
    """The deferred slab step (presorted slabs: the window's counts stay on the
    device, halo packets / merge / proof by library kernels, one verdict read
    per round) on a cloud whose reps near the face need a wider halo: it takes
    the deferred path, widens the halo on the verdict, and the result equals
    the single-GPU one bit for bit."""
    res = spawn(_hollow_rank)
    dev = torch.device("cuda:0")
    pts, vs = _hollow_cloud()
    x = pts.to(dev)
    mn, mx = ops.aabb(x)
    out = ops.voxel_down_sample(x, vs, mn, mx)
    ref = ops.estimate_normals(out["rep_xyz"], knn=30).cpu().numpy()
    g = np.concatenate([r[0] for r in res])
    nn = np.concatenate([r[1] for r in res])
    o = np.argsort(g)
    assert np.array_equal(g[o], out["rep_idx"].cpu().numpy().astype(np.int64))
    assert np.array_equal(nn[o], ref)
    for _, _, stamps in res:
        assert "reps_queued" in stamps  # the deferred path ran
        assert sum(1 for k in stamps if k.startswith("verdict")) >= 2, stamps  # the halo was widened


def _gap_rank(rank, world):
    """presorted over 3 ranks, the middle slab empty (nothing in the middle
    third of x): every rank takes the synchronous path alike"""
    dev = torch.device("cuda:0")
    n = 300_000
    pts = S.uniform_cube(n, 45)
    pts[:, 0] = torch.where(pts[:, 0] < 0.5, pts[:, 0] * 0.6, 0.4 + pts[:, 0] * 0.6)
    x = pts.to(dev)
    vs = S.voxel_size_for(n)
    g = _presorted_share(x, vs, rank, world)
    tl = {}
    rg, rx, nrm = D.voxel_normals_slabs(x[g].contiguous(), g, vs, knn=30, presorted=True, timings=tl)
    return rg, nrm, sorted(tl)


def test_c4_presorted_empty_slab_takes_sync_path():
    """A presorted cloud with an empty slab: the bounds all-reduce's smallest
    count is 0, so every rank takes the synchronous form alike; the result is
    the single-GPU one."""
    res = spawn(_gap_rank, world=3)
    dev = torch.device("cuda:0")
    n = 300_000
    pts = S.uniform_cube(n, 45)
    pts[:, 0] = torch.where(pts[:, 0] < 0.5, pts[:, 0] * 0.6, 0.4 + pts[:, 0] * 0.6)
    x = pts.to(dev)
    vs = S.voxel_size_for(n)
    mn, mx = ops.aabb(x)
    out = ops.voxel_down_sample(x, vs, mn, mx)
    ref = ops.estimate_normals(out["rep_xyz"], knn=30).cpu().numpy()
    g = np.concatenate([r[0] for r in res])
    nn = np.concatenate([r[1] for r in res])
    o = np.argsort(g)
    assert np.array_equal(g[o], out["rep_idx"].cpu().numpy().astype(np.int64))
    assert res[1][0].size == 0
    for _, _, stamps in res:
        assert "reps_queued" not in stamps
    # the two non-empty slabs' normals: every row within 1e-5 of the oracle
    reps = out["rep_xyz"].cpu().numpy()
    assert_normals(nn[o], O.estimate_normals(reps, O.KNN, 30), reps, k=30, what="c4_gap_slabs")


def _wide_cloud():
    """1000 blobs of 300 points (sigma 0.3 m) scattered over a 1 km cube, 5 cm
    voxels: the slab grid's cross-section (20000^2 voxels) dwarfs the points,
    so the fixed-size halo packets (hk x layer rows) are out of the question
    (they allocated by the grid, not by the data)."""
    rng = np.random.default_rng(5)
    c = rng.random((1000, 3)) * 1000.0
    p = (c[:, None, :] + rng.normal(0.0, 0.3, (1000, 300, 3))).reshape(-1, 3)
    return p.astype(np.float32), 0.05


def _wide_rank(rank, world):
    dev = torch.device("cuda:0")
    pts, vs = _wide_cloud()
    g = torch.arange(rank, len(pts), world, dtype=torch.int64)
    rg, rx, nrm = D.voxel_normals_slabs(torch.from_numpy(pts)[g].to(dev), g.to(dev), vs, knn=30)
    return rg, nrm


def test_c4_slabs_sparse_wide_cloud_on_device():
    """A wide, sparse cloud over 2 ranks: the halo goes by counted rows, and
    the slab result equals the single-GPU one bit for bit."""
    res = spawn(_wide_rank)
    dev = torch.device("cuda:0")
    pts, vs = _wide_cloud()
    x = torch.from_numpy(pts).to(dev)
    mn, mx = ops.aabb(x)
    out = ops.voxel_down_sample(x, vs, mn, mx)
    ref = ops.estimate_normals(out["rep_xyz"], knn=30).cpu().numpy()
    g = np.concatenate([r[0] for r in res])
    nn = np.concatenate([r[1] for r in res])
    o = np.argsort(g)
    assert np.array_equal(g[o], out["rep_idx"].cpu().numpy().astype(np.int64))
    assert np.array_equal(nn[o], ref)


def test_kdist_bound_is_an_upper_bound(dev):
    """estimate_normals(return_kdist=True): every row's bound >= the exact
    squared k-th-neighbour distance, and tight (within 1 %), on all paths."""
    pts = S.uniform_cube(300_000, 8)
    vs = S.voxel_size_for(300_000)
    a = ops.voxel_down_sample(pts.to(dev), vs, keep_grid=True)
    reps = a["rep_xyz"]
    r = reps.cpu().numpy()
    exact = O.knn_search(r, r, O.KNN, 30)[1][:, 29]
    for vg in (a["voxel_grid"], None):
        _, kd2 = ops.estimate_normals(reps, knn=30, voxel_grid=vg, return_kdist=True)
        kd2 = kd2.cpu().numpy().astype(np.float64)
        assert np.all(kd2 >= exact)
        assert np.all(kd2 <= exact * 1.01)


def _c4_presorted_rank(rank, world):
    dev = torch.device("cuda:0")
    n = 1_000_000
    vs = S.voxel_size_for(n)
    pts = S.uniform_cube(n, 44).to(dev)
    mn, mx = ops.aabb(pts)
    keys = D.slab_bounds(mn, mx, vs, world)
    kx = torch.floor((pts[:, 0].double() - float(mn[0])) / vs).to(torch.int64)
    g = torch.nonzero((kx >= keys[rank]) & (kx < keys[rank + 1])).flatten()
    rg, rx, nrm = D.voxel_normals_slabs(pts[g].contiguous(), g, vs, knn=30, presorted=True)
    return rg, nrm


@pytest.mark.parametrize("world", [2, 3])
def test_c4_slabs_presorted_on_device(world):
    """The bench's C4 step (points already in their slabs, voxel-table normals
    on own + halo reps): reps and normals bit-identical to one GPU's."""
    res = spawn(_c4_presorted_rank, world=world)
    dev = torch.device("cuda:0")
    n = 1_000_000
    vs = S.voxel_size_for(n)
    pts = S.uniform_cube(n, 44).to(dev)
    out = ops.voxel_down_sample(pts, vs, keep_grid=True)
    ref = ops.estimate_normals(out["rep_xyz"], knn=30, voxel_grid=out["voxel_grid"]).cpu().numpy()
    g = np.concatenate([r[0] for r in res])
    nn = np.concatenate([r[1] for r in res])
    o = np.argsort(g)
    assert np.array_equal(g[o], out["rep_idx"].cpu().numpy().astype(np.int64))
    assert np.array_equal(nn[o], ref)


def _c4_stray_rank(rank, world):
    """presorted slabs on the device (the dense x-window branch) with one point
    of rank 0's slab handed to the last rank only"""
    dev = torch.device("cuda:0")
    n = 1_000_000
    vs = S.voxel_size_for(n)
    pts = S.uniform_cube(n, 44).to(dev)
    mn, mx = ops.aabb(pts)
    keys = D.slab_bounds(mn, mx, vs, world)
    kx = torch.floor((pts[:, 0].double() - float(mn[0])) / vs).to(torch.int64)
    owner = torch.searchsorted(torch.tensor(keys[1:-1], dtype=torch.int64, device=dev), kx, right=True)
    stray = int(torch.nonzero(owner == 0)[0])
    owner[stray] = world - 1
    g = torch.nonzero(owner == rank).flatten()
    out = []
    for fn in (lambda: D.voxel_normals_slabs(pts[g].contiguous(), g, vs, knn=30, presorted=True),
               lambda: D.voxel_slabs(pts[g].contiguous(), g, vs, presorted=True)):
        try:
            fn()
            out.append("returned")
        except RuntimeError as e:
            out.append("raised: " + str(e))
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_c4_presorted_stray_point_raises_on_every_rank_device(world):
    """the dense-window branch turns a stray presorted point into
    the all-reduced verdict (every rank raises, no rank blocks), for the
    normals step and the voxel-only step alike."""
    res = spawn(_c4_stray_rank, world=world)
    for r in res:
        assert all(v.startswith("raised") and "outside" in v for v in r), res


# ------------------------------------------------------ C4 at its own size
C4_N = 50_000_000


def _c4_big_rank(rank, world, presorted):
    dev = torch.device("cuda:0")
    vs = S.voxel_size_for(C4_N)
    pts = S.uniform_cube(C4_N, 0, device=dev)
    if presorted:
        mn, mx = ops.aabb(pts)
        keys = D.slab_bounds(mn, mx, vs, world)
        kx = torch.floor((pts[:, 0].double() - float(mn[0])) / vs).to(torch.int64)
        g = torch.nonzero((kx >= keys[rank]) & (kx < keys[rank + 1])).flatten()
        del kx
    else:
        g = torch.arange(rank, C4_N, world, dtype=torch.int64, device=dev)
    x = pts[g].contiguous()
    del pts
    rg, _, nrm = D.voxel_normals_slabs(x, g, vs, knn=30, presorted=presorted)
    return rg, nrm


@pytest.mark.parametrize("world,presorted", [(2, True), (4, True), (2, False), (4, False)])
def test_c4_50m_slabs_match_single(world, presorted):
    """C4 at BASELINE configs[3]'s size: one 50M-point cloud over 2 and 4
    ranks (gloo rendezvous, the ranks share the one GPU of the test box),
    points already in their slabs (presorted, the bench's layout) or an
    arbitrary share moved to their slab owners: representatives and normals
    bit-identical to the single-GPU call (whose neighbour sets are checked
    bit-exact against the oracle at 50M in test_gpu_scale)."""
    res = spawn(_C4Big(presorted), world=world)
    dev = torch.device("cuda:0")
    pts = S.uniform_cube(C4_N, 0, device=dev)
    out = ops.voxel_down_sample_normals(pts, S.voxel_size_for(C4_N), knn=30)
    del pts
    g = np.concatenate([r[0] for r in res])
    o = np.argsort(g, kind="stable")
    assert np.array_equal(g[o], out["rep_idx"].cpu().numpy().astype(np.int64))
    nn = np.concatenate([r[1] for r in res])
    assert np.array_equal(nn[o], out["normals"].cpu().numpy())


class _C4Big:
    """picklable per-rank entry (spawn)"""

    def __init__(self, presorted):
        self.presorted = presorted

    def __call__(self, rank, world):
        return _c4_big_rank(rank, world, self.presorted)


# --------------------------------------------------------------------- C5
C5_N, C5_VS = 2_000_000, 0.002


def _c5_clouds(world, tiled):
    tgt = S.box_surface(C5_N, 1)
    src = S.apply_transform(S.box_surface(C5_N, 2), S.rigid_transform())
    if not tiled:
        return tgt, src
    out = []
    for c in (tgt, src):  # a spatially tiled dataset: the cloud is its slabs in rank order
        mn = c.double().min(0).values.numpy()
        mx = c.double().max(0).values.numpy()
        keys = D.slab_bounds(mn, mx, C5_VS, world)
        kx = torch.floor((c[:, 0].double() - float(mn[0])) / C5_VS).to(torch.int64)
        owner = torch.searchsorted(torch.tensor(keys[1:-1], dtype=torch.int64), kx, right=True)
        out.append(c[torch.argsort(owner, stable=True)].contiguous())
    return out[0], out[1]


def _c5_share(c, world, rank, tiled):
    if not tiled:
        return torch.arange(rank, c.shape[0], world, dtype=torch.int64)
    mn = c.double().min(0).values.numpy()
    mx = c.double().max(0).values.numpy()
    keys = D.slab_bounds(mn, mx, C5_VS, world)
    kx = torch.floor((c[:, 0].double() - float(mn[0])) / C5_VS).to(torch.int64)
    return torch.nonzero((kx >= keys[rank]) & (kx < keys[rank + 1])).flatten()


class _C5Rank:
    def __init__(self, tiled):
        self.tiled = tiled

    def __call__(self, rank, world):
        dev = torch.device("cuda:0")
        tgt, src = _c5_clouds(world, self.tiled)
        gt, gs = _c5_share(tgt, world, rank, self.tiled), _c5_share(src, world, rank, self.tiled)
        out = D.pipeline_sharded(tgt[gt].to(dev), gt.to(dev), src[gs].to(dev), gs.to(dev), C5_VS, knn=30,
                                 distance_threshold=0.002, num_iterations=300, seed=7,
                                 max_correspondence_distance=0.02, icp_iterations=10, presorted=self.tiled)
        return (out["target_rep_gidx"], out["target_normals"], out["plane"], out["plane_inlier_rows"],
                out["transformation"], out["fitness"], out["inlier_rmse"], out["target_reps"], out["source_reps"])


@pytest.mark.parametrize("world,tiled", [(2, True), (3, True), (2, False)])
def test_c5_pipeline_sharded_matches_single(world, tiled):
    """C5 (BASELINE configs[4]) over the ranks: target voxel reps + KNN30
    normals on x-slabs with the halo exchange, source voxel reps on its own
    slabs, segment_plane with the rows sharded (exact counts and fx sums),
    ICP with the source sharded and the fx moments all-reduced per
    iteration.  Against the single-GPU chain (ops.voxel_down_sample ->
    estimate_normals -> segment_plane -> registration_icp) on the same cloud:
    reps, normals, plane, inliers, T, fitness and rmse all bit-identical.
    tiled: the dataset is its slabs in rank order (positions by prefix sums);
    otherwise an interleaved share (positions by an index all-gather)."""
    res = spawn(_C5Rank(tiled), world=world)
    dev = torch.device("cuda:0")
    tgt, src = _c5_clouds(world, tiled)
    vt = ops.voxel_down_sample(tgt.to(dev), C5_VS, keep_grid=True)
    treps = vt["rep_xyz"]
    tn = ops.estimate_normals(treps, knn=30, voxel_grid=vt["voxel_grid"])
    sreps = ops.voxel_down_sample(src.to(dev), C5_VS)["rep_xyz"]
    M = treps.shape[0]
    samples = ops.ransac_samples(M, 3, 300, 7)
    plane, inl = ops.segment_plane(treps, 0.002, 3, 300, samples=samples)
    icp = ops.registration_icp(sreps, treps, tn, 0.02, max_iteration=10, relative_fitness=0.0, relative_rmse=0.0,
                               return_corr=False)
    g = np.concatenate([r[0] for r in res])
    o = np.argsort(g, kind="stable")
    assert np.array_equal(g[o], vt["rep_idx"].cpu().numpy().astype(np.int64))
    assert np.array_equal(np.concatenate([r[1] for r in res])[o], tn.cpu().numpy())
    rows = np.sort(np.concatenate([r[3] for r in res]))
    assert np.array_equal(rows, inl.cpu().numpy().astype(np.int64)) and len(rows) > 0
    for r in res:
        assert r[7] == M and r[8] == sreps.shape[0]
        assert np.array_equal(r[2], plane)
        assert np.array_equal(r[4], icp["transformation"])
        assert r[5] == icp["fitness"] and r[6] == icp["inlier_rmse"]
    assert np.abs(icp["transformation"] - np.linalg.inv(S.rigid_transform())).max() < 1e-3


# ------------------------------------------ sharded ICP: the device loop
def _icp_window_dev_rank(rank, world, margin, rel):
    """target AND source in x-slabs, each rank a WindowedTarget: the device
    loop (o3dx_icp_shard_*) with window stops when T leaves a window"""
    dev = torch.device("cuda:0")
    src, tgt = _clouds()
    t = torch.from_numpy(tgt).to(dev)
    tn = ops.estimate_normals(t, knn=30)
    cut_t = np.quantile(tgt[:, 0], np.linspace(0, 1, world + 1)[1:-1])
    cut_s = np.quantile(src[:, 0], np.linspace(0, 1, world + 1)[1:-1])
    pos = np.nonzero(np.searchsorted(cut_t, tgt[:, 0], side="right") == rank)[0]
    mine = np.searchsorted(cut_s, src[:, 0], side="right") == rank
    p = torch.from_numpy(pos).to(dev)
    target = D.WindowedTarget(t[p].contiguous(), tn[p].contiguous(), p, 0.02, margin=margin)
    T, f, r = D.registration_icp_sharded(torch.from_numpy(src[mine]).to(dev), target, max_iteration=20,
                                         relative_fitness=rel, relative_rmse=rel, n_source_total=len(src))
    return T, f, r, target.fetches


@pytest.mark.parametrize("world,margin,rel", [(2, 0.0, 0.0), (3, None, 1e-6)])
def test_sharded_icp_device_loop_windowed(world, margin, rel):
    """The sharded device loop with the target spread over the ranks too:
    margin 0 makes nearly every update leave some window, so the loop stops
    on the device, the windows are refetched and the loop resumes (the
    matches of the old window are not reused); with Open3D's relative
    criteria the loop may also converge early on every rank alike.  T,
    fitness and rmse equal the single-GPU device loop's to the bit."""
    import functools

    res = spawn(functools.partial(_icp_window_dev_rank, margin=margin, rel=rel), world=world)
    src, tgt = _clouds()
    dev = torch.device("cuda:0")
    t = torch.from_numpy(tgt).to(dev)
    tn = ops.estimate_normals(t, knn=30)
    one = ops.registration_icp(torch.from_numpy(src).to(dev), t, tn, 0.02, max_iteration=20, relative_fitness=rel,
                               relative_rmse=rel, return_corr=False)
    for T, f, r, fetches in res:
        assert np.array_equal(T, one["transformation"]) and f == one["fitness"] and r == one["inlier_rmse"]
    if margin == 0.0:
        assert max(r[3] for r in res) > 1  # the window-stop path ran


def _icp_skip_off_rank(rank, world):
    import os
    os.environ["O3DX_ICP_SKIP"] = "0"
    return _rank(rank, world)


def test_sharded_icp_device_loop_full_search():
    """O3DX_ICP_SKIP=0: every step of the sharded device loop searches in
    full; the same T as the skip-proof loop's (and the single GPU's)."""
    res = spawn(_icp_skip_off_rank, world=2)
    res2 = spawn(_rank, world=2)
    for (T, f, r), (T2, f2, r2) in zip(res, res2):
        assert np.array_equal(T, T2) and f == f2 and r == r2
