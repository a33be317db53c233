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
    (`allreduce_icp_sums`, `registration_icp_point_to_plane`).

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


def shard_range(n: int, world: int, rank: int, align: int = 1) -> Tuple[int, int]:
    """Contiguous [a, b) share of n items for `rank` (boundaries multiples of `align`)."""
    per = -(-n // world)
    per = -(-per // align) * align
    a = min(n, rank * per)
    return a, min(n, a + per)


__all__ = ["global_aabb", "slab_bounds", "slab_of", "allreduce_counts", "allreduce_icp_sums",
           "registration_icp_point_to_plane", "shard_range"]
