"""CPU: the multi-GPU path's collectives with torch.distributed `gloo`,
world size 2 (one process per rank, rendezvous on 127.0.0.1).  The per-rank
compute is the oracle (test infrastructure) so these run without a GPU; the
GPU box runs the same helpers over RCCL with the HIP kernels as `accumulate`.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import np_restate as NPR
from oracle import oracle as O
from open3dpypro import distributed as D
from open3dpypro import synthetic as S

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _plain(v):
    """torch tensors -> numpy (tensors in a queue would be shared through a
    socket that dies with the child process)."""
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    if isinstance(v, (tuple, list)):
        return type(v)(_plain(x) for x in v)
    return v


def _run(rank, world, port, fn, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _plain(fn(rank, world))))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, e))
    finally:
        dist.destroy_process_group()


def spawn(fn, world=WORLD):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_run, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        r, v = q.get(timeout=300)
        out[r] = v
    for p in ps:
        p.join(timeout=60)
    for r, v in out.items():
        if isinstance(v, Exception):
            raise v
    return [out[r] for r in range(world)]


# ---------------------------------------------------------------- AABB
def _aabb_rank(rank, world):
    pts = S.uniform_cube(5000, 3 + rank).numpy() * (rank + 1) - rank
    mn, mx = O.aabb(pts)
    return D.global_aabb(mn, mx)


def test_global_aabb_two_ranks():
    res = spawn(_aabb_rank)
    allp = np.concatenate([S.uniform_cube(5000, 3 + r).numpy() * (r + 1) - r for r in range(WORLD)])
    mn, mx = O.aabb(allp)
    for gmn, gmx in res:
        assert np.array_equal(gmn, mn) and np.array_equal(gmx, mx)


# ---------------------------------------------------------------- voxel slabs
def test_voxel_slabs_partition_reps():
    """x-slabs aligned to the global voxel grid: per-slab voxel reps (with the
    global min/max bound) are exactly the single-GPU reps, split by owner."""
    pts = S.uniform_cube(40_000, 21).numpy()
    vs = 0.05
    mn, mx = O.aabb(pts)
    full = O.voxel_down_sample(pts, vs, mn, mx)
    for world in (2, 3, 4):
        keys = D.slab_bounds(mn, mx, vs, world)
        kx = np.floor((pts[:, 0].astype(np.float64) - mn[0]) / vs).astype(np.int64)
        owner = D.slab_of(kx, keys)
        got = []
        for r in range(world):
            idx = np.nonzero(owner == r)[0]
            rep = O.voxel_down_sample(pts[idx], vs, mn, mx)
            got.append(idx[rep])
        got = np.sort(np.concatenate(got))
        assert np.array_equal(got, np.sort(full))


# ---------------------------------------------------------------- RANSAC counts
def _ransac_rank(rank, world):
    pts = S.planted_plane(20_000, 5).numpy()
    samples = O.ransac_samples(len(pts), 3, 64, 11)
    a, b = D.shard_range(len(pts), world, rank)
    # planes come from the replicated sample list; each rank counts its shard
    p64 = pts.astype(np.float64)
    counts = []
    for s in samples:
        pl = NPR.triangle_plane(p64[s[0]], p64[s[1]], p64[s[2]])
        counts.append(-1 if not pl.any() else int((NPR.plane_dist(pl, p64[a:b]) < 0.01).sum()))
    return D.allreduce_counts(np.array(counts, np.int64))


def test_ransac_counts_allreduce_exact():
    res = spawn(_ransac_rank)
    pts = S.planted_plane(20_000, 5).numpy()
    samples = O.ransac_samples(len(pts), 3, 64, 11)
    ref = NPR.segment_plane_counts(pts, 0.01, samples)
    for got in res:
        assert np.array_equal(got, ref)


# ---------------------------------------------------------------- ICP
def _icp_clouds():
    tgt = S.box_surface(20_000, 1).numpy()
    src = S.box_surface(20_000, 2).numpy()
    Tgt = S.rigid_transform()
    src = (src.astype(np.float64) @ Tgt[:3, :3].T + Tgt[:3, 3]).astype(np.float32)
    tn = O.estimate_normals(tgt, O.KNN, 30)
    return src, tgt, tn


def _icp_rank(rank, world):
    src, tgt, tn = _icp_clouds()
    a, b = D.shard_range(len(src), world, rank)
    shard = src[a:b]
    return D.registration_icp_point_to_plane(lambda T: O.icp_accumulate(shard, tgt, tn, 0.05, T),
                                             len(src), max_iteration=15)


def test_icp_sharded_matches_single():
    res = spawn(_icp_rank)
    src, tgt, tn = _icp_clouds()
    T1, f1, r1 = D.registration_icp_point_to_plane(lambda T: O.icp_accumulate(src, tgt, tn, 0.05, T),
                                                   len(src), max_iteration=15)
    (Ta, fa, ra), (Tb, fb, rb) = res
    assert np.array_equal(Ta, Tb) and fa == fb and ra == rb  # every rank solved the same bits
    assert np.abs(Ta - T1).max() < 1e-9
    assert abs(fa - f1) < 1e-12 and abs(ra - r1) < 1e-9
    # and the loop is the oracle's registration_icp
    To, fo, ro = O.registration_icp(src, tgt, tn, 0.05, max_iteration=15)[:3]
    assert np.abs(T1 - To).max() < 1e-9 and abs(f1 - fo) < 1e-12


def test_shard_range_covers():
    for n in (0, 1, 7, 1000, 1001):
        for world in (1, 2, 3, 8):
            parts = [D.shard_range(n, world, r, align=4) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))


# ---------------------------------------------------------------- C4 slabs
def _o3_voxel(p, vs, mn, mx):
    return torch.from_numpy(O.voxel_down_sample(p.numpy(), vs, mn, mx).astype(np.int64))


def _o3_normals(p, k):
    """oracle normals + the exact squared k-th-neighbour distance per row"""
    x = p.numpy()
    kk = min(k, len(x))
    kd2 = O.knn_search(x, x, O.KNN, kk)[1][:, kk - 1].copy() if len(x) else np.zeros(0)
    return torch.from_numpy(O.estimate_normals(x, O.KNN, k)), torch.from_numpy(kd2)


def _c4_cloud():
    return S.uniform_cube(60_000, 31)


def _c4_rank(rank, world):
    pts = _c4_cloud()
    n = pts.shape[0]
    # an arbitrary (non-spatial) initial share: every world-th point
    g = torch.arange(rank, n, world, dtype=torch.int64)
    return D.voxel_normals_slabs(pts[g], g, 0.05, knn=30, voxel_fn=_o3_voxel, normals_fn=_o3_normals)


def _check_slabs(res, pts, vs, k=30):
    mn, mx = O.aabb(pts)
    rep = O.voxel_down_sample(pts, vs, mn, mx)
    nrm = O.estimate_normals(pts[rep], O.KNN, k)
    g = np.concatenate([r[0] for r in res])
    nn = np.concatenate([r[2] for r in res])
    o = np.argsort(g)
    assert np.array_equal(g[o], rep.astype(np.int64))
    assert np.array_equal(nn[o], nrm)
    for r in res:  # each slab's reps are ascending and their xyz are the input points
        assert np.all(np.diff(r[0]) > 0)
        assert np.array_equal(r[1], pts[r[0]])


@pytest.mark.parametrize("world", [2, 3])
def test_c4_slabs_match_single(world):
    """Voxel reps and KNN30 normals of a cloud split over x-slabs (with the
    halo exchange) equal the single-process result: same reps, same normals
    bit for bit (the oracle sums each neighbourhood in the same order)."""
    res = spawn(_c4_rank, world=world)
    _check_slabs(res, _c4_cloud().numpy(), 0.05)


def _c4_misplaced_rank(rank, world):
    """presorted slabs with ONE point of rank 0's slab handed to the last rank
    only: every rank must raise, none may block in a later collective"""
    pts = _c4_cloud()
    vs = 0.05
    mn, mx = O.aabb(pts.numpy())
    keys = D.slab_bounds(mn, mx, vs, world)
    kx = np.floor((pts[:, 0].double().numpy() - mn[0]) / vs).astype(np.int64)
    owner = np.searchsorted(np.asarray(keys[1:-1]), kx, side="right")
    stray = int(np.flatnonzero(owner == 0)[0])
    owner[stray] = world - 1
    g = torch.from_numpy(np.flatnonzero(owner == rank).astype(np.int64))
    try:
        D.voxel_normals_slabs(pts[g], g, vs, knn=30, voxel_fn=_o3_voxel, normals_fn=_o3_normals, presorted=True)
    except RuntimeError as e:
        return "raised: " + str(e)
    return "returned"


@pytest.mark.parametrize("world", [2, 3])
def test_c4_presorted_stray_point_raises_on_every_rank(world):
    """a presorted point outside its slab is reported on EVERY rank
    (the verdict is all-reduced before anyone raises), not only on the rank
    holding it while its peers wait in the halo exchange."""
    res = spawn(_c4_misplaced_rank, world=world)
    assert all(r.startswith("raised") and "outside" in r for r in res), res


# A clustered cloud that defeats a halo check limited to the reps near a face:
# dense blobs sit on every interior slab face (their reps near the face have
# tiny k-th-neighbour distances), the sparse background keeps a band of 0.04
# clear around each face, so a background rep at 0.04 from a face (beyond the
# initial 3-voxel halo of 0.015) has k-th neighbours ~0.12 away across it.
CL_VS = 0.005


def _clustered_cloud(world):
    nkeys = int(np.floor(1.0 / CL_VS)) + 1
    faces = [((nkeys * r) // world) * CL_VS for r in range(1, world)]
    bg = S.uniform_cube(6000, 41).numpy().astype(np.float64)
    keep = np.ones(len(bg), bool)
    for f in faces:
        keep &= np.abs(bg[:, 0] - f) >= 0.04
    parts = [bg[keep], np.array([[0.0, 0.5, 0.5], [1.0, 0.5, 0.5]])]  # anchors: x bounds exactly [0, 1]
    rng = np.random.default_rng(42)
    for f in faces:
        d = rng.normal(size=(20000, 3))
        d *= (0.02 * rng.uniform(0, 1, (20000, 1)) ** (1 / 3)) / np.linalg.norm(d, axis=1, keepdims=True)
        parts.append(np.array([f, 0.9, 0.9]) + d)
    return np.concatenate(parts).astype(np.float32), faces


def _clustered_rank(rank, world):
    pts, _ = _clustered_cloud(world)
    g = torch.arange(rank, len(pts), world, dtype=torch.int64)
    return D.voxel_normals_slabs(torch.from_numpy(pts)[g], g, CL_VS, knn=30, voxel_fn=_o3_voxel,
                                 normals_fn=_o3_normals)


@pytest.mark.parametrize("world", [2, 3])
def test_c4_slabs_clustered_halo(world):
    pts, faces = _clustered_cloud(world)
    # the case really exercises the hole: some rep farther than the initial
    # halo H from every face still has true neighbours beyond H across one
    mn, mx = O.aabb(pts)
    rep = O.voxel_down_sample(pts, CL_VS, mn, mx)
    r = pts[rep]
    dk = np.sqrt(O.knn_search(r, r, O.KNN, 30)[1][:, 29])
    t = np.min(np.abs(r[:, :1].astype(np.float64) - np.array(faces)[None, :]), 1)
    H0 = 3 * CL_VS
    assert np.any((t >= H0) & (dk > t + H0))
    res = spawn(_clustered_rank, world=world)
    _check_slabs(res, pts, CL_VS)


# ----------------------------------------------------- exact (fx) sharded sums
class OracleBackend:
    """The per-rank compute of distributed.segment_plane_sharded /
    registration_icp_sharded restated on the CPU (oracle: test infrastructure)
    — the same interface as distributed._HipBackend, fx sums from numpy /
    the oracle's 128-bit restatement."""

    def absmax(self, x):
        p = x.numpy().astype(np.float64)
        return np.abs(p).max(0) if len(p) else np.zeros(3)

    def rows_f64(self, x, idx):
        return x[idx].double()

    def plane_count(self, x, planes, thr):
        p = x.numpy().astype(np.float64)
        out = []
        for pl in planes:
            if not pl.any():
                out.append(-1)
            elif not np.all(np.isfinite(pl)):
                out.append(0)
            else:
                out.append(int((NPR.plane_dist(pl, p) < thr).sum()))
        return np.array(out, np.int64)

    def plane_count_upper(self, x, planes, thr, absmax):
        # a valid upper bound that differs from the exact count, so the exact
        # rounds of the sharded selection (o3dx_ransac_needed) are exercised
        c = self.plane_count(x, planes, thr)
        return np.where(c >= 0, c + np.arange(len(c)) % 3, c)

    def abs_sum_fx(self, x, planes, which, thr):
        return np.stack([NPR.plane_abs_sum_fx(x.numpy(), planes[w], thr) for w in which])

    def plane_inliers(self, x, plane, thr):
        p = x.numpy().astype(np.float64)
        return torch.from_numpy(np.nonzero(NPR.plane_dist(plane, p) < thr)[0].astype(np.int64))

    def moments_fx(self, x, idx, centroid, absmax):
        return NPR.plane_moments_fx(x.numpy()[idx.numpy()], float(np.max(absmax)), centroid)

    def icp_target(self, tgt, tn, max_corr):
        return (tgt.numpy(), tn.numpy(), max_corr)

    def icp_source(self, src):
        return src.numpy()

    def icp_accumulate_fx(self, target, src, T, absmax):
        tgt, tn, mc = target
        return O.icp_accumulate_fx(src, tgt, tn, mc, T, absmax)

    # the slab steps of distributed.pipeline_sharded
    def voxel(self, p, vs, mn, mx):
        return _o3_voxel(p, vs, mn, mx)

    def normals(self, p, k):
        n, kd = _o3_normals(p, k)
        return n.float(), kd


def _plane_cloud():
    pts = S.planted_plane(30_000, 12, frac=0.3).numpy()
    return pts


def _plane_rank(rank, world, thr=0.01):
    from open3dpypro import distributed as Dm
    pts = _plane_cloud()
    pos = torch.arange(rank, len(pts), world, dtype=torch.int64)  # interleaved rows: not rank-ordered
    samples = O.ransac_samples(len(pts), 3, 300, 21)
    plane, inl = Dm.segment_plane_sharded(torch.from_numpy(pts)[pos], pos, len(pts), thr, 3, 300, samples=samples,
                                          backend=OracleBackend())
    return plane, pos[inl]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_segment_plane_sharded_bit_identical(world):
    """RANSAC with the rows spread over the ranks (sampled rows summed as bit
    patterns, integer counts, fx tie sums and refit moments): plane and
    inliers the same bits as one process, and equal to the oracle's
    SegmentPlane (inliers exactly, the plane within its float64-summation
    rounding)."""
    res = spawn(_plane_rank, world=world)
    p1, i1 = _plane_rank(0, 1)
    for pl, _ in res:
        assert np.array_equal(pl, p1)
    inl = np.sort(np.concatenate([r[1] for r in res]))
    assert np.array_equal(inl, i1)
    pts = _plane_cloud()
    rplane, rinl, *_ = O.segment_plane(pts, 0.01, 3, 300, O.ransac_samples(len(pts), 3, 300, 21))
    assert np.array_equal(i1, rinl)
    np.testing.assert_allclose(p1, rplane, rtol=0, atol=1e-12)


def _icp_fx_rank(rank, world):
    from open3dpypro import distributed as Dm
    src, tgt, tn = _icp_clouds()
    a, b = D.shard_range(len(src), world, rank)
    be = OracleBackend()
    target = be.icp_target(torch.from_numpy(tgt), torch.from_numpy(tn.astype(np.float32)), 0.05)
    return Dm.registration_icp_sharded(torch.from_numpy(src[a:b]), target, max_iteration=12, backend=be)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_icp_sharded_fx_bit_identical(world):
    """Point-to-plane ICP with the source sharded: the fx moments make T,
    fitness and rmse the same bits for 1, 2 and 3 ranks; the loop is the
    oracle's registration_icp to 1e-9."""
    res = spawn(_icp_fx_rank, world=world)
    T1, f1, r1 = _icp_fx_rank(0, 1)
    for T, f, r in res:
        assert np.array_equal(T, T1) and f == f1 and r == r1
    src, tgt, tn = _icp_clouds()
    To, fo, ro = O.registration_icp(src, tgt, tn.astype(np.float32), 0.05, max_iteration=12)[:3]
    assert np.abs(T1 - To).max() < 1e-9 and abs(f1 - fo) < 1e-12 and abs(r1 - ro) < 1e-9


def test_fx_rows_oracle_vs_numpy():
    """The oracle's 128-bit fx ICP sums and their float64 values against the
    plain float64 sums (the same terms): equal to within the fx rounding."""
    src, tgt, tn = _icp_clouds()
    T = S.rigid_transform(0.5, (0, 1, 0), (0.002, 0, 0))
    am = np.abs(src.astype(np.float64)).max(0)
    fx = O.icp_accumulate_fx(src, tgt, tn, 0.05, T, am)
    ref = O.icp_accumulate(src, tgt, tn, 0.05, T)
    vals = np.array([NPR.fx_value(r) for r in fx[:30]])
    assert vals[28] == ref[28]
    np.testing.assert_allclose(vals, ref[:30], rtol=1e-11, atol=1e-13)


def _icp_window_rank(rank, world, margin):
    """target AND source in x-slabs (C5's layout): WindowedTarget per rank"""
    from open3dpypro import distributed as Dm
    src, tgt, tn = _icp_clouds()
    be = OracleBackend()
    cut_t = np.quantile(tgt[:, 0], np.linspace(0, 1, world + 1)[1:-1])
    cut_s = np.quantile(src[:, 0], np.linspace(0, 1, world + 1)[1:-1])
    pos = np.nonzero(np.searchsorted(cut_t, tgt[:, 0], side="right") == rank)[0]
    mine = np.searchsorted(cut_s, src[:, 0], side="right") == rank
    target = Dm.WindowedTarget(torch.from_numpy(tgt[pos]), torch.from_numpy(tn[pos].astype(np.float32)),
                               torch.from_numpy(pos), 0.05, margin=margin, backend=be)
    T, f, r = Dm.registration_icp_sharded(torch.from_numpy(src[mine]), target, max_iteration=12, backend=be,
                                          n_source_total=len(src))
    return T, f, r, target.fetches, target.rows_held


@pytest.mark.parametrize("world,margin", [(2, 0.0), (3, 0.0), (3, None), (8, 0.0)])
def test_icp_windowed_target_bit_identical(world, margin):
    """ICP with the target spread over x-slabs too (distributed.WindowedTarget:
    each rank holds only the target rows within reach of its source under the
    current T, refetched by all ranks together when T moves a need past its
    window; margin 0 refetches at nearly every step): T, fitness and rmse the
    same bits as the replicated target on one process, with each rank holding
    a part of the target."""
    import functools
    res = spawn(functools.partial(_icp_window_rank, margin=margin), world=world)
    T1, f1, r1 = _icp_fx_rank(0, 1)
    src, tgt, tn = _icp_clouds()
    for T, f, r, fetches, held in res:
        assert np.array_equal(T, T1) and f == f1 and r == r1
        assert fetches >= 1 and held < len(tgt)
    if margin == 0.0:
        assert max(r[3] for r in res) > 1


def test_deferred_slab_eligibility_is_global():
    """The deferred slab step's eligibility (distributed._deferred_eligible)
    depends only on values every rank holds alike — the slab keys, the layer,
    the halo width and the smallest / largest point count — so all ranks take
    the same path; an empty rank, a window too sparse for a dense table, a
    halo packet larger than the data or a union table beyond the dense rule
    each send every rank to the synchronous form."""
    keys = D.slab_bounds([0.0, 0.0, 0.0], [1.0, 1.0, 1.0], 0.01, 4)  # 101 keys, widest slab 26
    layer = 101 * 101
    assert D._deferred_eligible(keys, layer, 3, 2_000_000, 2_500_000)
    assert not D._deferred_eligible(keys, layer, 3, 0, 2_500_000)           # an empty rank
    assert not D._deferred_eligible(keys, 50_000_000, 3, 2_000_000, 2_500_000)  # sparse window
    assert not D._deferred_eligible(keys, layer, 2000, 2_000_000, 2_500_000)   # halo packets beyond the data
    big = D.slab_bounds([0.0, 0.0, 0.0], [1.0, 1.0, 1.0], 0.001, 2)        # 1001 keys, layer 1e6
    assert not D._deferred_eligible(big, 1001 * 1001, 3, 100_000, 100_000)


# ------------------------------------------------------ eight ranks (one node)
def _weak_cloud(world):
    """C2-per-GPU layout (bench.py's N-rank headline): world unit cubes of
    points side by side along x, one uniform cloud over [0,world) x [0,1)^2"""
    p = S.uniform_cube(20_000 * world, 37)
    p[:, 0] *= float(world)
    return p


def _weak_rank(rank, world):
    pts = _weak_cloud(world)
    g = torch.arange(rank, pts.shape[0], world, dtype=torch.int64)  # interleaved: the point exchange runs
    return D.voxel_normals_slabs(pts[g], g, 0.05, knn=30, voxel_fn=_o3_voxel, normals_fn=_o3_normals)


def test_c4_slabs_eight_ranks():
    """the slab decomposition on 8 ranks (gloo), each slab one
    unit cube of the weak-scaling layout: reps and normals equal to one
    process's, bit for bit."""
    res = spawn(_weak_rank, world=8)
    _check_slabs(res, _weak_cloud(8).numpy(), 0.05)


def _pipe_clouds():
    tgt = S.box_surface(100_000, 1)
    src = S.apply_transform(S.box_surface(100_000, 2), S.rigid_transform())
    return tgt, src


def _pipe_rank(rank, world):
    tgt, src = _pipe_clouds()
    gt = torch.arange(rank, tgt.shape[0], world, dtype=torch.int64)
    gs = torch.arange(rank, src.shape[0], world, dtype=torch.int64)
    out = D.pipeline_sharded(tgt[gt], gt, src[gs], gs, 0.01, knn=30, distance_threshold=0.002, num_iterations=200,
                             seed=7, max_correspondence_distance=0.02, icp_iterations=6, backend=OracleBackend())
    return (out["target_rep_gidx"], out["target_normals"], out["plane"], out["plane_inlier_rows"],
            out["transformation"], out["fitness"], out["inlier_rmse"], out["target_reps"], out["source_reps"])


@pytest.mark.parametrize("world", [2, 8])
def test_pipeline_sharded_ranks_match_one(world):
    """C5's chain (distributed.pipeline_sharded: slab voxel reps + normals of
    the target, slab reps of the source, sharded RANSAC, sharded ICP with a
    windowed target) on 2 and 8 gloo ranks with the oracle as each rank's
    compute: every output the same bits as the chain on one process."""
    res = spawn(_pipe_rank, world=world)
    one = _plain(_pipe_rank(0, 1))
    g = np.concatenate([r[0] for r in res])
    o = np.argsort(g, kind="stable")
    assert np.array_equal(g[o], one[0])
    assert np.array_equal(np.concatenate([r[1] for r in res])[o], one[1])
    assert np.array_equal(np.sort(np.concatenate([r[3] for r in res])), np.sort(one[3])) and len(one[3]) > 0
    for r in res:
        assert np.array_equal(r[2], one[2]) and r[7] == one[7] and r[8] == one[8]
        assert np.array_equal(r[4], one[4]) and r[5] == one[5] and r[6] == one[6]
    assert one[5] > 0.9 and np.abs(one[4] - np.linalg.inv(S.rigid_transform())).max() < 2e-3
