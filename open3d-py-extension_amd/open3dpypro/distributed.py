"""Multi-GPU plumbing for the hot path: one process per GPU, torch.distributed
(RCCL over xGMI on the GPU box; gloo for the CPU tests).

The path shards by space with no data-path collective except where the
algorithm itself exchanges:

  * AABB: a 6-value min/max all-reduce (`global_aabb`);
  * voxel slabs: x-slabs aligned to the global voxel grid, so every voxel
    (and its representative) belongs to exactly one rank (`slab_bounds`,
    `slab_of`);
  * RANSAC: per-hypothesis integer counts, summed exactly (`allreduce_counts`);
  * ICP: the 29 float64 moments per iteration, all-gathered and summed in
    rank order, so every rank solves the same 6x6 system to the same bits
    (`allreduce_icp_sums`, `registration_icp_point_to_plane`);
  * voxel + normals of one cloud over x-slabs (C4): points to their slab
    owner, then one halo exchange of the representatives near each slab face
    (`voxel_normals_slabs`).

Every function takes an optional process group; with no initialised process
group they degrade to the single-process identity.
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N


def _world(group=None) -> Tuple[int, int]:
    if not (dist.is_available() and dist.is_initialized()):
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _comm_device(group=None) -> torch.device:
    """Tensors for collectives live on the GPU under RCCL, on the CPU under gloo."""
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def global_aabb(local_min, local_max, group=None) -> Tuple[np.ndarray, np.ndarray]:
    """Global (min_bound, max_bound) from every rank's local bounds (f64).
    A rank with no points passes +inf / -inf."""
    world, _ = _world(group)
    v = np.concatenate([np.asarray(local_min, np.float64), -np.asarray(local_max, np.float64)])
    if world > 1:
        t = torch.from_numpy(v).to(_comm_device(group))
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        v = t.cpu().numpy()
    return v[:3].copy(), -v[3:].copy()


def slab_bounds(min_bound, max_bound, voxel_size: float, world: int):
    """Voxel-aligned x-slab boundaries: rank r owns the voxels whose x key
    floor((x - min_x) / vs) lies in [keys[r], keys[r+1]).  The voxel key is
    Open3D's (PointCloud.py:338-341 -> VoxelDownSampleAndTrace), so a voxel
    never straddles two ranks and the union of the ranks' representatives is
    the single-GPU result."""
    if voxel_size <= 0:
        raise RuntimeError("voxel_size must be > 0")
    nkeys = int(math.floor((float(max_bound[0]) - float(min_bound[0])) / voxel_size)) + 1
    return [(nkeys * r) // world for r in range(world + 1)]


def slab_of(x_key: np.ndarray, keys) -> np.ndarray:
    """Owner rank of each x voxel key (host helper for planning / tests)."""
    return np.searchsorted(np.asarray(keys[1:-1]), x_key, side="right")


def allreduce_counts(counts: np.ndarray, group=None) -> np.ndarray:
    """Exact sum of integer per-hypothesis counts (RANSAC with the points
    sharded and the hypothesis list replicated).  Degenerate hypotheses are -1
    on every rank (the planes are replicated) and stay -1."""
    world, _ = _world(group)
    c = np.asarray(counts, np.int64)
    if world == 1:
        return c.copy()
    t = torch.from_numpy(c.copy()).to(_comm_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    out = t.cpu().numpy()
    return np.where(c < 0, -1, out)


def allreduce_icp_sums(sums: np.ndarray, group=None) -> np.ndarray:
    """Sum of every rank's ICP moment vector (float64, N.ICP_NSUMS), gathered and
    added in rank order so that all ranks hold identical bits."""
    world, _ = _world(group)
    s = np.asarray(sums, np.float64)
    if world == 1:
        return s.copy()
    dev = _comm_device(group)
    mine = torch.from_numpy(s.copy()).to(dev)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    acc = np.zeros_like(s)
    for p in parts:  # fixed order: rank 0, 1, ...
        acc = acc + p.cpu().numpy()
    return acc


def registration_icp_point_to_plane(accumulate: Callable[[np.ndarray], np.ndarray], n_source_total: int,
                                    init=None, max_iteration: int = 30, relative_fitness: float = 1e-6,
                                    relative_rmse: float = 1e-6, group=None):
    """Open3D registration_icp (point-to-plane) with the source sharded over
    ranks and the target replicated.  `accumulate(T) -> sums` computes this
    rank's moments (e.g. `ops.ICPTarget.accumulate(src_shard, T)[0]`); the
    loop mirrors o3dx_registration_icp_point_to_plane with the moments
    all-reduced once per iteration.  Returns (T, fitness, inlier_rmse)."""
    T = np.eye(4) if init is None else np.array(init, np.float64).reshape(4, 4)
    solve = N.load().o3dx_icp_solve_point_to_plane

    def metrics(sm):
        c = sm[28]
        if c <= 0 or n_source_total == 0:
            return 0.0, 0.0
        return c / n_source_total, math.sqrt(sm[29] / c)

    sums = allreduce_icp_sums(accumulate(T), group)
    fit, rm = metrics(sums)
    for _ in range(max_iteration):
        upd = np.zeros((4, 4), np.float64)
        solve(np.ascontiguousarray(sums).ctypes.data_as(N.ctypes.c_void_p),
              upd.ctypes.data_as(N.ctypes.c_void_p))
        T = upd @ T
        pf, pr = fit, rm
        sums = allreduce_icp_sums(accumulate(T), group)
        fit, rm = metrics(sums)
        if abs(pf - fit) < relative_fitness and abs(pr - rm) < relative_rmse:
            break
    return T, fit, rm


def _exchange(dest: torch.Tensor, world: int, group, *tensors):
    """all_to_all of the rows of each tensor to rank dest[i] (rows keep their
    relative order per source rank; sources are concatenated in rank order)."""
    cd = _comm_device(group)
    order = torch.argsort(dest, stable=True)
    send = torch.bincount(dest, minlength=world).to(torch.int64).to(cd)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    ss, rs = send.tolist(), recv.tolist()
    out = []
    for t in tensors:
        src = t[order].contiguous().to(cd)
        dst = torch.empty((sum(rs),) + tuple(t.shape[1:]), dtype=t.dtype, device=cd)
        dist.all_to_all_single(dst, src, output_split_sizes=rs, input_split_sizes=ss, group=group)
        out.append(dst.to(t.device))
    return out


def voxel_normals_slabs(xyz: torch.Tensor, gidx: torch.Tensor, voxel_size: float, knn: int = 30, group=None,
                        voxel_fn=None, normals_fn=None, halo: Optional[float] = None, presorted: bool = False):
    """C4: voxel_down_sample + estimate_normals(KNN) of one cloud spread over
    the ranks, decomposed into x-slabs aligned to the global voxel grid.

    `xyz` (n,3) float32 and `gidx` (n,) int64 global point indices are this
    rank's (arbitrary) share of the cloud.  Steps: global AABB (all-reduce);
    points to their slab owner (all-to-all); local voxel reps with the GLOBAL
    bounds, rows kept in global-index order so the max-index rep and every
    index tie-break equal the single-GPU ones; reps within `halo` of a slab
    face to the neighbour rank (all-to-all: the one exchange of this path);
    normals on own + halo reps.

    Halo proof, for EVERY own rep (not only those near a face): a rep p at
    distance t from its nearest interior slab face misses only points farther
    than t + H (they lie more than H beyond that face, or beyond a farther
    one), so its k nearest within own + halo are its true k nearest when its
    k-th-neighbour distance in the union is below t + H.  The normals kernels
    return an upper bound of that distance per row (o3dx estimate_normals
    kth_d2), so the check costs no extra search; when any rep on any rank
    fails it, H doubles and the exchange + normals repeat.  Returns (rep
    global indices ascending, rep xyz, normals) of this rank's slab; the union
    over ranks is the single-GPU result.  Compute defaults to the HIP kernels
    (ops); tests inject the oracle (normals_fn(p, k) -> (normals, kth_d2)).

    presorted: the caller guarantees every point already lies in this rank's
    slab and the rows are in ascending global index (a spatially tiled
    dataset): the point all-to-all is skipped (a point outside the slab makes
    the voxel call fail loudly)."""
    from . import ops

    if voxel_fn is None and normals_fn is None and xyz.is_cuda:
        return _voxel_normals_slabs_device(xyz, gidx, voxel_size, knn, group, halo, presorted)
    world, rank = _world(group)
    if voxel_fn is None:
        def voxel_fn(p, vs, mn, mx):
            return ops.voxel_down_sample(p, vs, mn, mx, with_xyz=False)["rep_idx"].long()
    if normals_fn is None:
        def normals_fn(p, k):
            return ops.estimate_normals(p, knn=k, return_kdist=True)
    # 1. global bounds (a rank with no points contributes nothing)
    if xyz.shape[0] > 0:
        lmn = xyz.double().min(0).values.cpu().numpy()
        lmx = xyz.double().max(0).values.cpu().numpy()
    else:
        lmn, lmx = np.full(3, np.inf), np.full(3, -np.inf)
    mn, mx = global_aabb(lmn, lmx, group)
    # 2. points to their slab owner, then into global-index order
    keys = slab_bounds(mn, mx, voxel_size, world)
    kx = torch.floor((xyz[:, 0].double() - float(mn[0])) / voxel_size).to(torch.int64)
    inner = torch.tensor(keys[1:-1], dtype=torch.int64, device=xyz.device)
    owner = torch.searchsorted(inner, kx, right=True)
    if world > 1:
        xyz, gidx = _exchange(owner, world, group, xyz, gidx)
    o = torch.argsort(gidx)
    xyz, gidx = xyz[o].contiguous(), gidx[o].contiguous()
    # 3. local reps with the global bounds
    rep = voxel_fn(xyz, voxel_size, mn, mx)
    rxyz, rg = xyz[rep].contiguous(), gidx[rep].contiguous()
    x_lo = float(mn[0]) + keys[rank] * voxel_size
    x_hi = float(mn[0]) + keys[rank + 1] * voxel_size
    t_lo = rxyz[:, 0].double() - x_lo  # distance to the slab faces
    t_hi = x_hi - rxyz[:, 0].double()
    inf = torch.full_like(t_lo, np.inf)
    t = torch.minimum(t_lo if rank > 0 else inf, t_hi if rank < world - 1 else inf)  # interior faces only
    H = float(halo) if halo else 3.0 * voxel_size
    min_width = min(keys[r + 1] - keys[r] for r in range(world)) * voxel_size
    n_total = int(_allreduce_int(rg.numel(), group))
    while True:
        if world > 1 and H >= min_width:
            raise RuntimeError("voxel_normals_slabs: the kNN halo is wider than a slab; use fewer ranks")
        # 4. halo exchange with the neighbour slabs
        if world > 1:
            send_lo = (t_lo < H) & (rank > 0)
            send_hi = (t_hi < H) & (rank < world - 1)
            dest = torch.cat([torch.full((int(send_lo.sum()),), rank - 1, dtype=torch.int64, device=rxyz.device),
                              torch.full((int(send_hi.sum()),), rank + 1, dtype=torch.int64, device=rxyz.device)])
            hx, hg = _exchange(dest, world, group, torch.cat([rxyz[send_lo], rxyz[send_hi]]),
                               torch.cat([rg[send_lo], rg[send_hi]]))
        else:
            hx, hg = rxyz[:0], rg[:0]
        ux, ug = torch.cat([rxyz, hx]), torch.cat([rg, hg])
        o = torch.argsort(ug)
        ux, ug = ux[o].contiguous(), ug[o].contiguous()
        own = torch.searchsorted(ug, rg)  # positions of the own reps in the union
        # 5. normals on own + halo reps, with each row's k-th-distance bound
        nrm, kd2 = normals_fn(ux, knn)
        # 6. verify every own rep (see above); fewer than k points in the
        # union while the cloud holds more cannot be verified at all
        ok = 1.0
        if world > 1 and rg.numel():
            if ux.shape[0] < min(knn, n_total):
                ok = 0.0
            else:
                dk = torch.sqrt(kd2[own].double().to(t.device))
                ok = 1.0 if bool((dk < (t + H) * (1.0 - 1e-9)).all()) else 0.0
        flag = torch.tensor([ok], dtype=torch.float64, device=_comm_device(group))
        if world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if flag.item() == 1.0:
            break
        H *= 2.0
    return rg, rxyz, nrm[own]


def _voxel_normals_slabs_device(xyz, gidx, voxel_size, knn, group, halo, presorted):
    """The HIP form of voxel_normals_slabs: every rank keeps a voxel table of
    its slab widened by the halo (global keys, x-key window), so the normals
    run straight off the table (k_normals_stile) on own + halo reps; the halo
    is a whole number of voxel layers.  Same contract and halo proof."""
    from . import ops

    world, rank = _world(group)
    vs = float(voxel_size)
    # 1. global bounds
    if xyz.shape[0] > 0:
        lmn, lmx = ops.aabb(xyz)
    else:
        lmn, lmx = np.full(3, np.inf), np.full(3, -np.inf)
    mn, mx = global_aabb(lmn, lmx, group)
    keys = slab_bounds(mn, mx, vs, world)
    k_lo, k_hi, nkeys = keys[rank], keys[rank + 1], keys[-1]
    # 2. points to their slab owner (unless the input is already tiled)
    if world > 1 and not presorted:
        kx = torch.floor((xyz[:, 0].double() - float(mn[0])) / vs).to(torch.int64)
        inner = torch.tensor(keys[1:-1], dtype=torch.int64, device=xyz.device)
        xyz, gidx = _exchange(torch.searchsorted(inner, kx, right=True), world, group, xyz, gidx)
        o = torch.argsort(gidx)
        xyz, gidx = xyz[o].contiguous(), gidx[o].contiguous()
    # 3. own reps: keys of the global grid, the slab's x keys only (a dense
    # window table when the slab is not sparse — the same rule as the
    # library's dense voxel table, 2n + 2^20 cells — else the hash path)
    dims = np.floor(np.maximum(np.asarray(mx) - np.asarray(mn), 0.0) / vs) + 1
    layer = int(dims[1] * dims[2])
    n_loc = int(xyz.shape[0])
    dense = (k_hi - k_lo + 6) * layer <= 2 * n_loc + (1 << 20)
    if k_hi > k_lo and n_loc > 0:
        if dense:
            out = ops.voxel_down_sample_window(xyz, vs, mn, mx, k_lo, k_hi)
        else:
            out = ops.voxel_down_sample(xyz, vs, mn, mx)
        rep = out["rep_idx"].long()
        rxyz, rg = out["rep_xyz"], gidx[rep].contiguous()
    else:
        rxyz, rg = xyz[:0], gidx[:0]
    kxr = torch.floor((rxyz[:, 0].double() - float(mn[0])) / vs).to(torch.int64)
    x_lo, x_hi = float(mn[0]) + k_lo * vs, float(mn[0]) + k_hi * vs
    inf = torch.full((rxyz.shape[0],), np.inf, dtype=torch.float64, device=rxyz.device)
    t = torch.minimum(rxyz[:, 0].double() - x_lo if rank > 0 else inf,
                      x_hi - rxyz[:, 0].double() if rank < world - 1 else inf)
    hk = max(1, int(math.ceil(float(halo) / vs))) if halo else 3
    min_keys = min(keys[r + 1] - keys[r] for r in range(world))
    n_total = _allreduce_int(rg.numel(), group)
    table = None
    while True:
        if world > 1 and hk >= min_keys:
            raise RuntimeError("voxel_normals_slabs: the kNN halo is wider than a slab; use fewer ranks")
        # 4. halo: the own reps of the hk voxel layers next to each interior face
        if world > 1:
            send_lo = (kxr < k_lo + hk) & (rank > 0)
            send_hi = (kxr >= k_hi - hk) & (rank < world - 1)
            dest = torch.cat([torch.full((int(send_lo.sum()),), rank - 1, dtype=torch.int64, device=rxyz.device),
                              torch.full((int(send_hi.sum()),), rank + 1, dtype=torch.int64, device=rxyz.device)])
            hx, hg = _exchange(dest, world, group, torch.cat([rxyz[send_lo], rxyz[send_hi]]),
                               torch.cat([rg[send_lo], rg[send_hi]]))
            ux, ug = torch.cat([rxyz, hx]), torch.cat([rg, hg])
            o = torch.argsort(ug)
            ux, ug = ux[o].contiguous(), ug[o].contiguous()
            own = torch.searchsorted(ug, rg)
        else:
            ux, ug, own = rxyz, rg, None
        # 5. the union's voxel table over the slab + halo window, normals off it
        kx0, kx1 = max(k_lo - hk, 0), min(k_hi + hk, nkeys)
        if ux.shape[0] > 0 and (kx1 - kx0) * layer <= 2 * int(ux.shape[0]) + (1 << 20):
            grid = ops.voxel_table(ux, vs, mn, mx, kx0, kx1, table)
            table = grid.pts
            nrm, kd2 = ops.estimate_normals(ux, knn=knn, voxel_grid=grid, return_kdist=True)
        elif ux.shape[0] > 0:  # sparse slab: the normals sort the union into their own grid
            nrm, kd2 = ops.estimate_normals(ux, knn=knn, return_kdist=True)
        else:
            nrm, kd2 = ux.new_zeros((0, 3)), ux.new_zeros((0,))
        if own is not None:
            nrm, kd2 = nrm[own], kd2[own]
        # 6. verify every own rep: a missing point lies more than t + hk*vs away
        ok = 1.0
        if world > 1 and rg.numel():
            if ux.shape[0] < min(knn, n_total):
                ok = 0.0
            else:
                ok = 1.0 if bool((torch.sqrt(kd2.double()) < (t + hk * vs) * (1.0 - 1e-9)).all()) else 0.0
        flag = torch.tensor([ok], dtype=torch.float64, device=_comm_device(group))
        if world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if flag.item() == 1.0:
            break
        hk *= 2
    return rg, rxyz, nrm


def _allreduce_int(v: int, group=None) -> int:
    world, _ = _world(group)
    if world == 1:
        return int(v)
    t = torch.tensor([int(v)], dtype=torch.int64, device=_comm_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item())


def shard_range(n: int, world: int, rank: int, align: int = 1) -> Tuple[int, int]:
    """Contiguous [a, b) share of n items for `rank` (boundaries multiples of `align`)."""
    per = -(-n // world)
    per = -(-per // align) * align
    a = min(n, rank * per)
    return a, min(n, a + per)


__all__ = ["global_aabb", "slab_bounds", "slab_of", "allreduce_counts", "allreduce_icp_sums",
           "registration_icp_point_to_plane", "voxel_normals_slabs", "shard_range"]
