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
    shard = ops.spatial_sort(torch.from_numpy(src[a:b]).to(dev))
    return D.registration_icp_point_to_plane(lambda T: target.accumulate(shard, T)[0], len(src), max_iteration=20)


def test_sharded_icp_on_device_matches_single():
    (Ta, fa, ra), (Tb, fb, rb) = spawn(_rank)
    assert np.array_equal(Ta, Tb) and fa == fb and ra == rb
    T1, f1, r1 = _rank(0, 1)
    assert np.abs(Ta - T1).max() < 1e-9 and abs(fa - f1) < 1e-12
    src, tgt = _clouds()
    tn = O.estimate_normals(tgt, O.KNN, 30)
    To, fo, ro = O.registration_icp(src, tgt, tn, 0.02, max_iteration=20)[:3]
    assert np.abs(T1 - To).max() < 1e-5 and abs(f1 - fo) < 1e-5


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
