"""Tensor-level hot-path ops: torch-ROCm tensors in, torch tensors out.

Each op is a thin call into libo3dx.so (include/o3dx.h); the tensor is only
the device array container.  Inputs: (N,3) contiguous on a ROCm GPU — float32,
or float64 for the float64 boundary (o3dx_*_f64: the hot-path ops computed on
the caller's float64 values, as Open3D computes them on its float64 storage).
PointCloud passes float64 only for clouds float32 cannot hold.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import _native as N


def _xyz(t: torch.Tensor, what="points") -> torch.Tensor:
    N.require_device(t, what)
    if t.ndim != 2 or t.shape[1] != 3:
        raise RuntimeError(f"{what} must have shape (n, 3), got {tuple(t.shape)}")
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _is64(t) -> bool:
    return isinstance(t, torch.Tensor) and t.dtype == torch.float64


def _xyz64(t: torch.Tensor, what="points") -> torch.Tensor:
    N.require_device(t, what)
    if t.ndim != 2 or t.shape[1] != 3:
        raise RuntimeError(f"{what} must have shape (n, 3), got {tuple(t.shape)}")
    return t.to(torch.float64).contiguous()


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _np_ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def aabb(xyz: torch.Tensor):
    """(min_bound, max_bound) as float64 numpy — get_min_bound/get_max_bound."""
    L = N.load()
    if _is64(xyz):
        x = _xyz64(xyz)
        n = x.shape[0]
        ws = N.workspace(L.o3dx_aabb_f64_workspace_bytes(n), x.device, "aabb")
        out = np.zeros(6, np.float64)
        N.check(L.o3dx_aabb_f64(N.ptr(x), n, _np_ptr(out), N.ptr(ws), ws.numel(), N.stream_ptr(x.device)), "aabb")
        return out[:3].copy(), out[3:].copy()
    x = _xyz(xyz)
    n = x.shape[0]
    ws = N.workspace(L.o3dx_aabb_workspace_bytes(n), x.device)
    out = np.zeros(6, np.float64)
    N.check(L.o3dx_aabb(N.ptr(x), n, _np_ptr(out), N.ptr(ws), ws.numel(), N.stream_ptr(x.device)), "aabb")
    return out[:3].copy(), out[3:].copy()


def aabb_device(xyz: torch.Tensor) -> torch.Tensor:
    """(6,) float64 device tensor {min, max} of the cloud, asynchronous
    (o3dx_aabb_device; zeros for an empty cloud)."""
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    ws = N.workspace(L.o3dx_aabb_workspace_bytes(n), x.device, "aabb")
    out = torch.empty(6, dtype=torch.float64, device=x.device)
    N.check(L.o3dx_aabb_device(N.ptr(x), n, N.ptr(out), N.ptr(ws), ws.numel(), N.stream_ptr(x.device)), "aabb_device")
    return out


def voxel_down_sample(xyz: torch.Tensor, voxel_size: float, min_bound=None, max_bound=None,
                      with_xyz: bool = True, trace: bool = False, keep_grid: bool = False):
    """Open3D VoxelDownSampleAndTrace + idxmat.max(1) + _select_by_idx.

    Returns dict: rep_idx (M,) int32 ascending; rep_xyz (M,3) (if with_xyz);
    voxel_of_point (N,) int32 and cubic_id (M,8) int32 (if trace);
    voxel_grid (if keep_grid): the voxel table for estimate_normals(...,
    voxel_grid=) on the representatives' points (rep_xyz), or None when the
    grid was too sparse to keep.  float64 points: o3dx_voxel_down_sample_f64
    (keys from the float64 coordinates; rep_xyz float64; no voxel table)."""
    if _is64(xyz):
        return _voxel_down_sample_f64(xyz, voxel_size, min_bound, max_bound, with_xyz, trace, keep_grid)
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    dev = x.device
    ws = N.workspace(L.o3dx_voxel_workspace_bytes(n), dev)
    rep = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    rxyz = torch.empty((max(n, 1), 3), dtype=torch.float32, device=dev) if with_xyz else None
    vop = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if trace else None
    cub = torch.empty(max(8 * n, 8), dtype=torch.int32, device=dev) if trace else None
    mnb = None if min_bound is None else _c(min_bound, np.float64)
    mxb = None if max_bound is None else _c(max_bound, np.float64)
    m = np.zeros(1, np.int64)
    cells = 0
    if keep_grid and n > 0:
        # a table buffer for the largest grid the library keeps: the bounds
        # (and the AABB when they are not given) stay on the library's side,
        # no extra host round trip
        cells = int(L.o3dx_voxel_grid_capacity(n))
    geom = np.zeros(12, np.float64)
    if cells > 0:
        vox = torch.empty((cells, 4), dtype=torch.float32, device=dev)
        rc = L.o3dx_voxel_down_sample_grid(N.ptr(x), n, _np_ptr(mnb), _np_ptr(mxb), float(voxel_size), N.ptr(rep),
                                           N.ptr(rxyz), _np_ptr(m), N.ptr(vop), N.ptr(cub), N.ptr(vox), cells,
                                           _np_ptr(geom), N.ptr(ws), ws.numel(), N.stream_ptr(dev))
    else:
        rc = L.o3dx_voxel_down_sample(N.ptr(x), n, _np_ptr(mnb), _np_ptr(mxb), float(voxel_size), N.ptr(rep),
                                      N.ptr(rxyz), _np_ptr(m), N.ptr(vop), N.ptr(cub), N.ptr(ws), ws.numel(),
                                      N.stream_ptr(dev))
    N.check(rc, "voxel_down_sample")
    M = int(m[0])
    out = {"rep_idx": rep[:M]}
    if with_xyz:
        out["rep_xyz"] = rxyz[:M]
    if trace:
        out["voxel_of_point"] = vop[:n]
        out["cubic_id"] = cub[: 8 * M].view(M, 8)
    if keep_grid:
        out["voxel_grid"] = VoxelGrid(geom, vox, M) if geom[7] == 1.0 else None
    return out


def _voxel_down_sample_f64(xyz, voxel_size, min_bound, max_bound, with_xyz, trace, keep_grid):
    x = _xyz64(xyz)
    L = N.load()
    n = x.shape[0]
    dev = x.device
    ws = N.workspace(L.o3dx_voxel_f64_workspace_bytes(n), dev)
    rep = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    rxyz = torch.empty((max(n, 1), 3), dtype=torch.float64, device=dev) if with_xyz else None
    vop = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if trace else None
    cub = torch.empty(max(8 * n, 8), dtype=torch.int32, device=dev) if trace else None
    mnb = None if min_bound is None else _c(min_bound, np.float64)
    mxb = None if max_bound is None else _c(max_bound, np.float64)
    m = np.zeros(1, np.int64)
    N.check(L.o3dx_voxel_down_sample_f64(N.ptr(x), n, _np_ptr(mnb), _np_ptr(mxb), float(voxel_size), N.ptr(rep),
                                         N.ptr(rxyz), _np_ptr(m), N.ptr(vop), N.ptr(cub), N.ptr(ws), ws.numel(),
                                         N.stream_ptr(dev)), "voxel_down_sample")
    M = int(m[0])
    out = {"rep_idx": rep[:M]}
    if with_xyz:
        out["rep_xyz"] = rxyz[:M]
    if trace:
        out["voxel_of_point"] = vop[:n]
        out["cubic_id"] = cub[: 8 * M].view(M, 8)
    if keep_grid:
        out["voxel_grid"] = None
    return out


def voxel_down_sample_window(xyz: torch.Tensor, voxel_size: float, min_bound, max_bound, kx0: int, kx1: int,
                             keep_grid: bool = False):
    """Slab form of voxel_down_sample (include/o3dx.h o3dx_voxel_down_sample_window):
    keys of the GLOBAL min_bound, only the x keys [kx0, kx1) materialised.
    Returns dict rep_idx, rep_xyz (and voxel_grid if keep_grid)."""
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    dev = x.device
    ws = N.workspace(L.o3dx_voxel_workspace_bytes(n), dev)
    rep = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    rxyz = torch.empty((max(n, 1), 3), dtype=torch.float32, device=dev)
    m = np.zeros(1, np.int64)
    geom = np.zeros(12, np.float64)
    cells = int(L.o3dx_voxel_grid_capacity(n)) if keep_grid and n > 0 else 0
    vox = torch.empty((max(cells, 1), 4), dtype=torch.float32, device=dev) if cells else None
    N.check(L.o3dx_voxel_down_sample_window(N.ptr(x), n, _np_ptr(_c(min_bound, np.float64)),
                                            _np_ptr(_c(max_bound, np.float64)), float(voxel_size), int(kx0), int(kx1),
                                            N.ptr(rep), N.ptr(rxyz), _np_ptr(m), N.ptr(vox), cells, _np_ptr(geom),
                                            N.ptr(ws), ws.numel(), N.stream_ptr(dev)), "voxel_down_sample_window")
    M = int(m[0])
    out = {"rep_idx": rep[:M], "rep_xyz": rxyz[:M]}
    if keep_grid:
        out["voxel_grid"] = VoxelGrid(geom, vox, M) if geom[7] == 1.0 else None
    return out


def voxel_table(xyz: torch.Tensor, voxel_size: float, min_bound, max_bound, kx0: int, kx1: int,
                table: Optional[torch.Tensor] = None, status: Optional[torch.Tensor] = None):
    """VoxelGrid of points holding at most one point per voxel (a slab's own +
    halo representatives), over the x-key window [kx0, kx1) of the global grid
    (o3dx_voxel_table_build).  `table`: an optional (cells, 4) float32 buffer.
    `status`: a zeroed int64 device tensor — the deferred form
    (o3dx_voxel_table_build_deferred): no host wait, non-finite rows skipped,
    error bits OR-ed into status[0] (1: a point outside the window, 2: two
    points in one voxel) for the caller to check."""
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    dev = x.device
    mnb, mxb = _c(min_bound, np.float64), _c(max_bound, np.float64)
    dims = np.floor(np.maximum(mxb - mnb, 0.0) / voxel_size) + 1
    cells = int((kx1 - kx0) * dims[1] * dims[2])
    if table is None or table.shape[0] < cells:
        table = torch.empty((cells, 4), dtype=torch.float32, device=dev)
    geom = np.zeros(12, np.float64)
    ws = N.workspace(L.o3dx_voxel_table_workspace_bytes(), dev, "table")
    if status is not None:  # deferred: no host wait, error bits OR-ed into status[0] on the device
        N.check(L.o3dx_voxel_table_build_deferred(N.ptr(x), n, _np_ptr(mnb), _np_ptr(mxb), float(voxel_size),
                                                  int(kx0), int(kx1), N.ptr(table), table.shape[0], _np_ptr(geom),
                                                  N.ptr(status), N.stream_ptr(dev)), "voxel_table")
        return VoxelGrid(geom, table, n)
    N.check(L.o3dx_voxel_table_build(N.ptr(x), n, _np_ptr(mnb), _np_ptr(mxb), float(voxel_size), int(kx0), int(kx1),
                                     N.ptr(table), table.shape[0], _np_ptr(geom), N.ptr(ws), ws.numel(),
                                     N.stream_ptr(dev)), "voxel_table")
    return VoxelGrid(geom, table, n)


def voxel_down_sample_normals(xyz: torch.Tensor, voxel_size: float, knn: int = 30, min_bound=None, max_bound=None):
    """voxel_down_sample(keep_grid=True) + estimate_normals(KNN knn, voxel_grid=) on the
    representatives in one library call (o3dx_voxel_down_sample_normals): the
    normals are queued behind the voxel kernels without a host round trip.
    Returns dict rep_idx, rep_xyz, normals (M,3) float32, voxel_grid."""
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    dev = x.device
    if n == 0:
        e = torch.empty((0, 3), dtype=torch.float32, device=dev)
        return {"rep_idx": torch.empty(0, dtype=torch.int32, device=dev), "rep_xyz": e, "normals": e.clone(),
                "voxel_grid": None}
    ws = N.workspace(L.o3dx_voxel_workspace_bytes(n), dev)
    nws = N.workspace(L.o3dx_normals_workspace_bytes(n), dev, "normals")
    rep = torch.empty(n, dtype=torch.int32, device=dev)
    rxyz = torch.empty((n, 3), dtype=torch.float32, device=dev)
    nrm = torch.empty((n, 3), dtype=torch.float32, device=dev)
    cells = int(L.o3dx_voxel_grid_capacity(n))
    vox = torch.empty((cells, 4), dtype=torch.float32, device=dev)
    mnb = None if min_bound is None else _c(min_bound, np.float64)
    mxb = None if max_bound is None else _c(max_bound, np.float64)
    m = np.zeros(1, np.int64)
    geom = np.zeros(12, np.float64)
    N.check(L.o3dx_voxel_down_sample_normals(N.ptr(x), n, _np_ptr(mnb), _np_ptr(mxb), float(voxel_size), int(knn),
                                             N.ptr(rep), N.ptr(rxyz), N.ptr(nrm), _np_ptr(m), N.ptr(vox), cells,
                                             _np_ptr(geom), N.ptr(ws), ws.numel(), N.ptr(nws), nws.numel(),
                                             N.stream_ptr(dev)), "voxel_down_sample_normals")
    M = int(m[0])
    return {"rep_idx": rep[:M], "rep_xyz": rxyz[:M], "normals": nrm[:M],
            "voxel_grid": VoxelGrid(geom, vox, M) if geom[7] == 1.0 else None}


class VoxelGrid:
    """The voxel table of a voxel_down_sample(keep_grid=True): per voxel the
    representative's (x, y, z, output row) (row -1 empty) + the grid geometry.
    Lets estimate_normals on the M representatives skip sorting them into a
    search grid (include/o3dx.h o3dx_estimate_normals_voxel)."""

    def __init__(self, geom: np.ndarray, pts: torch.Tensor, m: int):
        self.geom = np.ascontiguousarray(geom, np.float64)
        self.pts = pts
        self.m = int(m)


def estimate_normals(xyz: torch.Tensor, mode: int = N.SEARCH_KNN, knn: int = 30, radius: float = 0.0,
                     prior: Optional[torch.Tensor] = None, voxel_grid: Optional[VoxelGrid] = None,
                     return_kdist: bool = False):
    """Open3D EstimateNormals(search_param, fast_normal_computation=True) -> (N,3) float32.

    voxel_grid: the VoxelGrid of the voxel_down_sample that produced `xyz`
    (its rep_xyz); the search grid is then read off the voxel table.
    return_kdist (KNN only): also return (N,) float32 upper bounds of each
    point's squared k-th-neighbour distance (for halo checks of sharded runs).
    float64 points: o3dx_estimate_normals_f64 (sets and moments from the
    float64 coordinates; voxel_grid is not used)."""
    if _is64(xyz):
        return _estimate_normals_f64(xyz, mode, knn, radius, prior, return_kdist)
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    dev = x.device
    out = torch.empty((max(n, 1), 3), dtype=torch.float32, device=dev)
    if return_kdist and mode != N.SEARCH_KNN:
        raise ValueError("return_kdist needs KNN search")
    kd2 = torch.empty(max(n, 1), dtype=torch.float32, device=dev) if return_kdist else None
    pr = None if prior is None else _xyz(prior.to(dev), "prior normals")
    ws = N.workspace(L.o3dx_normals_workspace_bytes(n), dev)
    if voxel_grid is not None:
        if voxel_grid.m != n or voxel_grid.pts.device != dev:
            raise ValueError("voxel_grid does not belong to these points")
        rc = L.o3dx_estimate_normals_voxel(_np_ptr(voxel_grid.geom), N.ptr(voxel_grid.pts), N.ptr(x), n, int(mode),
                                           int(knn), float(radius), N.ptr(pr), N.ptr(out), N.ptr(kd2), N.ptr(ws),
                                           ws.numel(), N.stream_ptr(dev))
    else:
        rc = L.o3dx_estimate_normals(N.ptr(x), n, int(mode), int(knn), float(radius), N.ptr(pr), N.ptr(out),
                                     N.ptr(kd2), N.ptr(ws), ws.numel(), N.stream_ptr(dev))
    N.check(rc, "estimate_normals")
    if return_kdist:
        return out[:n], kd2[:n]
    return out[:n]


def _estimate_normals_f64(xyz, mode, knn, radius, prior, return_kdist):
    x = _xyz64(xyz)
    L = N.load()
    n = x.shape[0]
    dev = x.device
    if return_kdist and mode != N.SEARCH_KNN:
        raise ValueError("return_kdist needs KNN search")
    out = torch.empty((max(n, 1), 3), dtype=torch.float32, device=dev)
    kd2 = torch.empty(max(n, 1), dtype=torch.float32, device=dev) if return_kdist else None
    pr = None if prior is None else _xyz(prior.to(dev), "prior normals")
    ws = N.workspace(L.o3dx_normals_f64_workspace_bytes(n), dev)
    N.check(L.o3dx_estimate_normals_f64(N.ptr(x), n, int(mode), int(knn), float(radius), N.ptr(pr), N.ptr(out),
                                        N.ptr(kd2), N.ptr(ws), ws.numel(), N.stream_ptr(dev)), "estimate_normals")
    if return_kdist:
        return out[:n], kd2[:n]
    return out[:n]


def knn_search(xyz: torch.Tensor, queries: torch.Tensor, mode: int = N.SEARCH_KNN, knn: int = 30,
               radius: float = 0.0):
    """Batched KDTreeFlann search: (idx (nq,K) int32, d2 (nq,K) float64, count (nq,) int32).
    float64 points: o3dx_knn_search_f64 (queries taken as float64)."""
    if _is64(xyz):
        x = _xyz64(xyz)
        q = _xyz64(queries.to(x.device), "queries")
        L = N.load()
        n, nq = x.shape[0], q.shape[0]
        dev = x.device
        K = int(knn)
        idx = torch.empty((max(nq, 1), K), dtype=torch.int32, device=dev)
        d2 = torch.empty((max(nq, 1), K), dtype=torch.float64, device=dev)
        cnt = torch.empty(max(nq, 1), dtype=torch.int32, device=dev)
        ws = N.workspace(L.o3dx_knn_f64_workspace_bytes(n), dev)
        N.check(L.o3dx_knn_search_f64(N.ptr(x), n, N.ptr(q), nq, int(mode), K, float(radius), N.ptr(idx), N.ptr(d2),
                                      N.ptr(cnt), N.ptr(ws), ws.numel(), N.stream_ptr(dev)), "knn_search")
        return idx[:nq], d2[:nq], cnt[:nq]
    x = _xyz(xyz)
    q = _xyz(queries.to(x.device), "queries")
    L = N.load()
    n, nq = x.shape[0], q.shape[0]
    dev = x.device
    K = int(knn)
    idx = torch.empty((max(nq, 1), K), dtype=torch.int32, device=dev)
    d2 = torch.empty((max(nq, 1), K), dtype=torch.float64, device=dev)
    cnt = torch.empty(max(nq, 1), dtype=torch.int32, device=dev)
    ws = N.workspace(L.o3dx_knn_workspace_bytes(n), dev)
    rc = L.o3dx_knn_search(N.ptr(x), n, N.ptr(q), nq, int(mode), K, float(radius), N.ptr(idx), N.ptr(d2), N.ptr(cnt),
                           N.ptr(ws), ws.numel(), N.stream_ptr(dev))
    N.check(rc, "knn_search")
    return idx[:nq], d2[:nq], cnt[:nq]


def search_one(xyz: torch.Tensor, query, mode: int = N.SEARCH_KNN, knn: int = 30, radius: float = 0.0):
    """One KDTreeFlann query of any size (o3dx_search_one): (k, idx (k,) int32,
    d2 (k,) float64) on the device, sorted by (d^2, index).  mode KNN: the knn
    nearest; RADIUS: every point with d^2 < radius^2; HYBRID: the knn nearest
    of those.  float32 or float64 points (the cloud's own coordinates)."""
    f64 = _is64(xyz)
    x = _xyz64(xyz) if f64 else _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    q = _c(np.asarray(query, np.float64).reshape(3), np.float64)
    cap = n if mode == N.SEARCH_RADIUS else min(int(knn), n)
    idx = torch.empty(max(cap, 1), dtype=torch.int32, device=x.device)
    d2 = torch.empty(max(cap, 1), dtype=torch.float64, device=x.device)
    cnt = np.zeros(1, np.int64)
    ws = N.workspace(L.o3dx_search_one_workspace_bytes(n), x.device, "search")
    N.check(L.o3dx_search_one(N.ptr(x), 1 if f64 else 0, n, _np_ptr(q), int(mode), int(knn), float(radius),
                              N.ptr(idx), N.ptr(d2), cap, _np_ptr(cnt), N.ptr(ws), ws.numel(),
                              N.stream_ptr(x.device)), "search_one")
    k = int(cnt[0])
    return k, idx[:k], d2[:k]


def ransac_samples(n: int, ransac_n: int, num_iterations: int, seed: int) -> np.ndarray:
    """Open3D RandomSampler over mt19937(seed): (iters, ransac_n) int32."""
    out = np.empty((max(num_iterations, 1), ransac_n), np.int32)
    N.check(N.load().o3dx_ransac_samples(int(n), int(ransac_n), int(num_iterations), int(seed) & (2**64 - 1),
                                         _np_ptr(out)), "ransac_samples")
    return out[:num_iterations]


def segment_plane(xyz: torch.Tensor, distance_threshold: float, ransac_n: int, num_iterations: int,
                  probability: float = 0.99999999, samples: Optional[np.ndarray] = None, seed: int = 0):
    """Open3D SegmentPlane -> (plane float64[4], inliers (k,) int32 ascending on device).
    float64 points: o3dx_segment_plane_f64 (exact counts on the float64 coordinates)."""
    f64 = _is64(xyz)
    x = _xyz64(xyz) if f64 else _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    dev = x.device
    if not (0.0 < probability <= 1.0):
        raise RuntimeError("Probability must be > 0 or <= 1.0")
    if ransac_n < 3:
        raise RuntimeError("ransac_n should be set to higher than or equal to 3.")
    if n < ransac_n:
        raise RuntimeError("There must be at least 'ransac_n' points.")
    if samples is None:
        samples = ransac_samples(n, ransac_n, num_iterations, seed)
    s = _c(samples, np.int32).reshape(num_iterations, ransac_n)
    plane = np.zeros(4, np.float64)
    inl = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    k = np.zeros(1, np.int64)
    wsb = (L.o3dx_segment_plane_f64_workspace_bytes if f64 else L.o3dx_segment_plane_workspace_bytes)
    ws = N.workspace(wsb(n, num_iterations), dev)
    fn = L.o3dx_segment_plane_f64 if f64 else L.o3dx_segment_plane
    rc = fn(N.ptr(x), n, float(distance_threshold), int(ransac_n), int(num_iterations), float(probability),
            _np_ptr(s), _np_ptr(plane), N.ptr(inl), _np_ptr(k), N.ptr(ws), ws.numel(), N.stream_ptr(dev))
    N.check(rc, "segment_plane")
    return plane, inl[: int(k[0])]


def plane_count(xyz: torch.Tensor, planes: np.ndarray, distance_threshold: float) -> np.ndarray:
    """Exact per-hypothesis inlier counts (-1 for degenerate planes); float64
    points: o3dx_plane_count_f64."""
    f64 = _is64(xyz)
    x = _xyz64(xyz) if f64 else _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    P = _c(planes, np.float64).reshape(-1, 4)
    H = P.shape[0]
    counts = np.zeros(max(H, 1), np.int64)
    ws = N.workspace(L.o3dx_plane_count_workspace_bytes(n, H), x.device)
    fn = L.o3dx_plane_count_f64 if f64 else L.o3dx_plane_count
    N.check(fn(N.ptr(x), n, _np_ptr(P), H, float(distance_threshold), _np_ptr(counts), N.ptr(ws),
                               ws.numel(), N.stream_ptr(x.device)), "plane_count")
    return counts[:H]


def plane_count_upper(xyz: torch.Tensor, planes: np.ndarray, distance_threshold: float, absmax=None) -> np.ndarray:
    """Upper bounds of the per-hypothesis inlier counts (>= exact; -1 for
    degenerate planes), o3dx_plane_count_upper; absmax: the cloud's |x|,|y|,|z|
    bounds (None: its own)."""
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    P = _c(planes, np.float64).reshape(-1, 4)
    H = P.shape[0]
    counts = np.zeros(max(H, 1), np.int64)
    am = None if absmax is None else _c(absmax, np.float64)
    ws = N.workspace(L.o3dx_plane_count_workspace_bytes(n, H), x.device)
    N.check(L.o3dx_plane_count_upper(N.ptr(x), n, _np_ptr(P), H, float(distance_threshold),
                                     None if am is None else _np_ptr(am), _np_ptr(counts), N.ptr(ws), ws.numel(),
                                     N.stream_ptr(x.device)), "plane_count_upper")
    return counts[:H]


def ransac_needed(counts, known, planes, n: int, ransac_n: int, probability: float = 0.99999999) -> np.ndarray:
    """The hypotheses without an exact count (known False) that Open3D's
    selection replay on `counts` consults (o3dx_ransac_needed); empty: the
    selection on these counts is the exact one."""
    c = _c(counts, np.int64)
    k8 = _c(np.asarray(known, bool).astype(np.uint8), np.uint8)
    P = _c(planes, np.float64).reshape(-1, 4)
    out = np.zeros(max(len(c), 1), np.int32)
    k = np.zeros(1, np.int32)
    N.check(N.load().o3dx_ransac_needed(_np_ptr(c), _np_ptr(k8), _np_ptr(P), len(c), int(n), int(ransac_n),
                                        float(probability), _np_ptr(out), _np_ptr(k)), "ransac_needed")
    return out[: int(k[0])].copy()


def plane_abs_sum(xyz: torch.Tensor, planes: np.ndarray, which, distance_threshold: float, return_fx: bool = False):
    """Sigma |d| over |d| < thr of the hypotheses `which` (exact fx sums):
    float64 (L,), and with return_fx their (L, 4) int64 fx rows."""
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    P = _c(planes, np.float64).reshape(-1, 4)
    w = _c(which, np.int32)
    sums = np.zeros(max(len(w), 1), np.float64)
    fx = np.zeros((max(len(w), 1), 4), np.int64)
    ws = N.workspace(L.o3dx_plane_count_workspace_bytes(n, max(len(w), 1)), x.device)
    N.check(L.o3dx_plane_abs_sum(N.ptr(x), n, _np_ptr(P), _np_ptr(w), len(w), float(distance_threshold),
                                 _np_ptr(sums), _np_ptr(fx), N.ptr(ws), ws.numel(), N.stream_ptr(x.device)),
            "plane_abs_sum")
    return (sums[: len(w)], fx[: len(w)]) if return_fx else sums[: len(w)]


def ransac_tied(counts, planes, n: int, ransac_n: int, probability: float = 0.99999999) -> np.ndarray:
    """Hypotheses whose Sigma|d| Open3D's selection can consult (o3dx_ransac_tied)."""
    c = _c(counts, np.int64)
    P = _c(planes, np.float64).reshape(-1, 4)
    out = np.zeros(max(len(c), 1), np.int32)
    k = np.zeros(1, np.int32)
    N.check(N.load().o3dx_ransac_tied(_np_ptr(c), _np_ptr(P), len(c), int(n), int(ransac_n), float(probability),
                                      _np_ptr(out), _np_ptr(k)), "ransac_tied")
    return out[: int(k[0])].copy()


def fx_to_double(fx) -> np.ndarray:
    """fx rows {lo, hi, q, 0} (int64, k x 4) -> float64 (k,), correctly rounded
    (o3dx_fx_to_double): the one conversion every path uses."""
    f = _c(fx, np.int64).reshape(-1, 4)
    out = np.zeros(max(len(f), 1), np.float64)
    N.check(N.load().o3dx_fx_to_double(_np_ptr(f), len(f), _np_ptr(out)), "fx_to_double")
    return out[: len(f)]


def absmax(xyz: torch.Tensor) -> np.ndarray:
    """|x|,|y|,|z| bounds of a cloud (from its AABB), float64 (3,)."""
    if xyz.shape[0] == 0:
        return np.zeros(3)
    mn, mx = aabb(xyz)
    return np.maximum(np.abs(mn), np.abs(mx))


def planes_from_samples(coords: np.ndarray, ransac_n: int) -> np.ndarray:
    """(H, ransac_n, 3) float64 sample coordinates -> (H, 4) planes
    (ComputeTrianglePlane / GetPlaneFromPoints, o3dx_planes_from_samples)."""
    c = _c(coords, np.float64).reshape(-1, ransac_n, 3)
    out = np.zeros((max(len(c), 1), 4), np.float64)
    N.check(N.load().o3dx_planes_from_samples(_np_ptr(c), len(c), int(ransac_n), _np_ptr(out)), "planes_from_samples")
    return out[: len(c)]


def plane_from_points(pts: np.ndarray) -> np.ndarray:
    p = _c(pts, np.float64).reshape(-1, 3)
    out = np.zeros(4, np.float64)
    N.check(N.load().o3dx_plane_from_points(_np_ptr(p), len(p), _np_ptr(out)), "plane_from_points")
    return out


def ransac_select(counts, sums, planes, n, ransac_n, probability=0.99999999) -> int:
    c = _c(counts, np.int64)
    s = _c(sums, np.float64)
    P = _c(planes, np.float64).reshape(-1, 4)
    return int(N.load().o3dx_ransac_select(_np_ptr(c), _np_ptr(s), _np_ptr(P), len(c), int(n), int(ransac_n),
                                           float(probability)))


def plane_inliers(xyz: torch.Tensor, plane, distance_threshold: float) -> torch.Tensor:
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    pl = _c(plane, np.float64)
    idx = torch.empty(max(n, 1), dtype=torch.int32, device=x.device)
    k = np.zeros(1, np.int64)
    ws = N.workspace(2 * n + 65536, x.device)
    N.check(L.o3dx_plane_inliers(N.ptr(x), n, _np_ptr(pl), float(distance_threshold), N.ptr(idx), _np_ptr(k),
                                 N.ptr(ws), ws.numel(), N.stream_ptr(x.device)), "plane_inliers")
    return idx[: int(k[0])]


def _plane_pts(xyz: torch.Tensor):
    """(tensor, entry point) for the plane selection: float64 coordinates go to
    o3dx_plane_select_f64 unrounded, anything else as float32."""
    if isinstance(xyz, torch.Tensor) and xyz.dtype == torch.float64:
        N.require_device(xyz, "points")
        if xyz.ndim != 2 or xyz.shape[1] != 3:
            raise RuntimeError(f"points must have shape (n, 3), got {tuple(xyz.shape)}")
        return xyz.contiguous(), N.load().o3dx_plane_select_f64
    return _xyz(xyz), N.load().o3dx_plane_select


def plane_select(xyz: torch.Tensor, plane, thickness, invert: bool = False) -> torch.Tensor:
    """Ascending int32 device indices of the points within `thickness` of the
    plane (|s| < thickness, or thickness[0] < s < thickness[1] for a tuple),
    complemented with `invert`; s = distance2plane (reference PointCloud.py:
    278-290, 400-404).  o3dx_plane_select (float32 points) or
    o3dx_plane_select_f64 (float64 points)."""
    x, fn = _plane_pts(xyz)
    L = N.load()
    n = x.shape[0]
    pl = _c(plane, np.float64).reshape(4)
    band = isinstance(thickness, tuple)
    lo, hi = (float(thickness[0]), float(thickness[1])) if band else (0.0, float(thickness))
    idx = torch.empty(max(n, 1), dtype=torch.int32, device=x.device)
    k = np.zeros(1, np.int64)
    ws = N.workspace(int(L.o3dx_plane_select_workspace_bytes(n)), x.device)
    N.check(fn(N.ptr(x), n, _np_ptr(pl), int(band), lo, hi, int(bool(invert)), None, N.ptr(idx), _np_ptr(k),
               N.ptr(ws), ws.numel(), N.stream_ptr(x.device)), "plane_select")
    return idx[: int(k[0])]


def plane_distance(xyz: torch.Tensor, plane) -> torch.Tensor:
    """float64 signed distance of every point to the plane, in the order of the
    reference's distance2plane (PointCloud.py:400-404).  o3dx_plane_select(_f64)."""
    x, fn = _plane_pts(xyz)
    n = x.shape[0]
    pl = _c(plane, np.float64).reshape(4)
    out = torch.empty(n, dtype=torch.float64, device=x.device)
    N.check(fn(N.ptr(x), n, _np_ptr(pl), 0, 0.0, 0.0, 0, N.ptr(out), None, None, None, 0,
               N.stream_ptr(x.device)), "plane_distance")
    return out


def plane_moments(xyz: torch.Tensor, idx: Optional[torch.Tensor], centroid=None, absmax=None,
                  return_fx: bool = False):
    """GetPlaneFromPoints moments over idx (exact fx sums): {x,y,z} (pass 1) or
    centred {xx,xy,xz,yy,yz,zz} (pass 2, `centroid` given).  absmax: the
    cloud's |x|,|y|,|z| bounds fixing the fx quantum (a sharded cloud passes
    the global ones).  With return_fx also the (3|6, 4) fx rows."""
    x = _xyz(xyz)
    L = N.load()
    count = x.shape[0] if idx is None else idx.numel()
    c = None if centroid is None else _c(centroid, np.float64)
    am = None if absmax is None else _c(absmax, np.float64)
    out = np.zeros(6, np.float64)
    fx = np.zeros((6, 4), np.int64)
    ws = N.workspace(int(L.o3dx_plane_moments_workspace_bytes(count)), x.device, "moments")
    ii = None if idx is None else idx.to(torch.int32).contiguous()
    N.check(L.o3dx_plane_moments(N.ptr(x), N.ptr(ii), count, _np_ptr(c), _np_ptr(am), _np_ptr(out), _np_ptr(fx),
                                 N.ptr(ws), ws.numel(), N.stream_ptr(x.device)), "plane_moments")
    k = 6 if centroid is not None else 3
    return (out[:k], fx[:k]) if return_fx else out[:k]


def plane_from_moments(sum_xyz, count, centred) -> np.ndarray:
    out = np.zeros(4, np.float64)
    N.check(N.load().o3dx_plane_from_moments(_np_ptr(_c(sum_xyz, np.float64)), int(count),
                                             _np_ptr(_c(centred, np.float64)), _np_ptr(out)), "plane_from_moments")
    return out


class ICPTarget:
    """Persistent target structure (grid of target points + normals) for ICP."""

    def __init__(self, tgt: torch.Tensor, tgt_normals: torch.Tensor, max_correspondence_distance: float):
        # float64 targets: a float64 grid (o3dx_icp_target_build_f64), float64 sources
        self.f64 = _is64(tgt)
        self.xyz = _xyz64(tgt, "target points") if self.f64 else _xyz(tgt, "target points")
        self.normals = _xyz(tgt_normals.to(self.xyz.device), "target normals")
        if self.normals.shape[0] != self.xyz.shape[0]:
            raise RuntimeError("target normals must match target points")
        L = N.load()
        nt = self.xyz.shape[0]
        self.max_corr = float(max_correspondence_distance)
        wsb = L.o3dx_icp_target_f64_workspace_bytes if self.f64 else L.o3dx_icp_target_workspace_bytes
        build = L.o3dx_icp_target_build_f64 if self.f64 else L.o3dx_icp_target_build
        self.ws = torch.empty(wsb(nt), dtype=torch.uint8, device=self.xyz.device)
        self.desc = np.zeros(N.ICP_DESC_LEN, np.float64)
        N.check(build(N.ptr(self.xyz), N.ptr(self.normals), nt, self.max_corr, N.ptr(self.ws), self.ws.numel(),
                      _np_ptr(self.desc), N.stream_ptr(self.xyz.device)), "icp_target_build")

    def accumulate(self, src: torch.Tensor, T: np.ndarray, want_corr: bool = False, absmax=None,
                   return_fx: bool = False):
        """Transform + 1-NN + point-to-plane moments: (sums[32], corr or None)
        (+ the (32, 4) int64 fx rows with return_fx).  `src` is (n,3) float32,
        or the (n,4) output of spatial_sort (faster).  absmax: |x|,|y|,|z|
        bounds of the WHOLE source (a sharded source passes the global ones);
        default: spatial_sort's record of them, else the library measures src."""
        if self.f64:
            raise RuntimeError("ICPTarget.accumulate: float64 targets run the device loop (register)")
        sorted4 = src.ndim == 2 and src.shape[1] == 4
        if sorted4:
            N.require_device(src, "source points")
            s = src.float().contiguous()
        else:
            s = _xyz(src.to(self.xyz.device), "source points")
        if absmax is None:
            absmax = getattr(src, "absmax", None)
            of = getattr(src, "absmax_of", None)
            if absmax is None and of is not None:  # spatial_sort's cloud, measured on first use only
                absmax = src.absmax = _absmax(of)
        L = N.load()
        ns = s.shape[0]
        TT = _c(T, np.float64).reshape(4, 4)
        am = None if absmax is None else _c(absmax, np.float64).reshape(3)
        sums = np.zeros(N.ICP_NSUMS, np.float64)
        fx = np.zeros((N.ICP_NSUMS, 4), np.int64)
        corr = torch.empty((max(ns, 1), 2), dtype=torch.int32, device=s.device) if want_corr else None
        nc = np.zeros(1, np.int64)
        ws = N.workspace(L.o3dx_icp_accumulate_workspace_bytes(ns), s.device, "icp_acc")
        N.check(L.o3dx_icp_accumulate(N.ptr(s), ns, 1 if sorted4 else 0, N.ptr(self.ws), _np_ptr(self.desc),
                                      _np_ptr(TT), self.max_corr, _np_ptr(am),
                                      _np_ptr(sums), _np_ptr(fx), N.ptr(corr), _np_ptr(nc), N.ptr(ws), ws.numel(),
                                      N.stream_ptr(s.device)), "icp_accumulate")
        out = (sums, (corr[: int(nc[0])] if want_corr else None))
        return out + (fx,) if return_fx else out

    def register(self, src: torch.Tensor, init=None, max_iteration: int = 30, relative_fitness: float = 1e-6,
                 relative_rmse: float = 1e-6, absmax=None, want_corr: bool = False):
        """Open3D registration_icp (point-to-plane) onto this target with the
        whole loop on the device (o3dx_icp_register): each iteration's fused
        correspondence + moments pass, the solve and the convergence test are
        queued at once and the host waits once.  `src` as in accumulate (the
        (n,4) spatial_sort output is faster).  -> dict(transformation,
        fitness, inlier_rmse[, correspondence_set])."""
        sorted4 = src.ndim == 2 and src.shape[1] == 4
        if sorted4:
            N.require_device(src, "source points")
            # the index column's encoding follows the dtype (spatial_sort:
            # int32 bits in a float32 column; spatial_sort_f64: the index as a
            # double), so a cast would corrupt it: the sorted form must match
            want = torch.float64 if self.f64 else torch.float32
            if src.dtype != want:
                raise RuntimeError(f"ICPTarget.register: a {'float64' if self.f64 else 'float32'} target takes the "
                                   f"({'spatial_sort_f64' if self.f64 else 'spatial_sort'}) sorted source, got "
                                   f"{src.dtype}")
            s = src.contiguous()
        elif self.f64:
            s = _xyz64(src.to(self.xyz.device), "source points")
        else:
            s = _xyz(src.to(self.xyz.device), "source points")
        if absmax is None:
            absmax = getattr(src, "absmax", None)
        L = N.load()
        ns = s.shape[0]
        T0 = _c(np.eye(4) if init is None else init, np.float64).reshape(4, 4)
        am = None if absmax is None else _c(absmax, np.float64).reshape(3)
        T = np.zeros((4, 4), np.float64)
        fit, rm = np.zeros(1), np.zeros(1)
        corr = torch.empty((max(ns, 1), 2), dtype=torch.int32, device=s.device) if want_corr else None
        nc = np.zeros(1, np.int64)
        ws = N.workspace(L.o3dx_icp_accumulate_workspace_bytes(ns), s.device, "icp_acc")
        reg = L.o3dx_icp_register_f64 if self.f64 else L.o3dx_icp_register
        N.check(reg(N.ptr(s), ns, 1 if sorted4 else 0, N.ptr(self.ws), _np_ptr(self.desc), _np_ptr(T0),
                    int(max_iteration), float(relative_fitness), float(relative_rmse), self.max_corr, _np_ptr(am),
                    _np_ptr(T), _np_ptr(fit), _np_ptr(rm), N.ptr(corr), _np_ptr(nc), N.ptr(ws), ws.numel(),
                    N.stream_ptr(s.device)), "icp_register")
        out = {"transformation": T, "fitness": float(fit[0]), "inlier_rmse": float(rm[0])}
        if want_corr:
            out["correspondence_set"] = corr[: int(nc[0])]
        return out


class ICPShardLoop:
    """One rank's side of the sharded device loop (o3dx_icp_shard_*,
    distributed.registration_icp_sharded): the state lives in the workspace;
    step() queues the rank's match + moments into a 64-int64 digit tensor,
    the caller all-reduces it, finish() queues the shared solve / update.
    Nothing here waits on the device except state() and resume()."""

    def __init__(self, src: torch.Tensor, absmax, max_correspondence_distance: float, init=None):
        sorted4 = src.ndim == 2 and src.shape[1] == 4
        if sorted4:
            N.require_device(src, "source points")
            if src.dtype != torch.float32:
                raise RuntimeError("ICPShardLoop: float32 sources (spatial_sort output or (n,3))")
            self.src = src.contiguous()
        else:
            self.src = _xyz(src, "source points")
        self.sorted4 = 1 if sorted4 else 0
        self.ns = int(self.src.shape[0])
        self.mc = float(max_correspondence_distance)
        self.dev = self.src.device
        L = N.load()
        self.L = L
        self.ws = torch.empty(int(L.o3dx_icp_accumulate_workspace_bytes(self.ns)), dtype=torch.uint8,
                              device=self.dev)
        T0 = _c(np.eye(4) if init is None else init, np.float64).reshape(4, 4)
        am = _c(absmax, np.float64).reshape(3)
        self.st = N.stream_ptr(self.dev)
        N.check(L.o3dx_icp_shard_begin(_np_ptr(T0), _np_ptr(am), self.mc, self.ns, N.ptr(self.ws), self.ws.numel(),
                                       self.st), "icp_shard_begin")

    def step(self, target, digits: torch.Tensor, use_prior: bool, widen: float = float("inf")):
        tws = None if target is None else N.ptr(target.ws)
        desc = None if target is None else _np_ptr(target.desc)
        N.check(self.L.o3dx_icp_shard_step(N.ptr(self.src), self.ns, self.sorted4, tws, desc, self.mc,
                                           1 if use_prior else 0, float(widen), N.ptr(digits), N.ptr(self.ws),
                                           self.ws.numel(), self.st), "icp_shard_step")

    def finish(self, digits: torch.Tensor, n_total: int, it: int, max_iteration: int, relative_fitness: float,
               relative_rmse: float, target=None, win: Optional[torch.Tensor] = None, widen: float = float("inf")):
        desc = None if target is None else _np_ptr(target.desc)
        world = 0 if win is None else int(win.shape[0])
        N.check(self.L.o3dx_icp_shard_finish(N.ptr(digits), int(n_total), int(it), int(max_iteration),
                                             float(relative_fitness), float(relative_rmse), self.mc, desc,
                                             None if win is None else N.ptr(win), world, float(widen), self.ns,
                                             N.ptr(self.ws), self.ws.numel(), self.st), "icp_shard_finish")

    def state(self):
        """(T, fitness, inlier_rmse, info {done, iterations applied, window stop}) — one host wait"""
        T = np.zeros((4, 4), np.float64)
        fit, rm = np.zeros(1), np.zeros(1)
        info = np.zeros(3, np.int32)
        N.check(self.L.o3dx_icp_shard_state(self.ns, N.ptr(self.ws), self.ws.numel(), _np_ptr(T), _np_ptr(fit),
                                            _np_ptr(rm), _np_ptr(info), self.st), "icp_shard_state")
        return T, float(fit[0]), float(rm[0]), info

    def resume(self):
        N.check(self.L.o3dx_icp_shard_resume(self.ns, N.ptr(self.ws), self.ws.numel(), self.st), "icp_shard_resume")


def spatial_sort_f64(xyz: torch.Tensor, target_occ: float = 8.0) -> torch.Tensor:
    """(n,4) float64 form of spatial_sort for float64 sources (x, y, z,
    original index), o3dx_spatial_sort_f64: ICPTarget.register's fast input
    on a float64 target."""
    x = _xyz64(xyz)
    L = N.load()
    n = x.shape[0]
    out = torch.empty((max(n, 1), 4), dtype=torch.float64, device=x.device)
    ws = N.workspace(L.o3dx_spatial_sort_f64_workspace_bytes(n), x.device, "sort")
    N.check(L.o3dx_spatial_sort_f64(N.ptr(x), n, float(target_occ), N.ptr(out), N.ptr(ws), ws.numel(),
                                    N.stream_ptr(x.device)), "spatial_sort_f64")
    return out[:n]


def spatial_sort(xyz: torch.Tensor, target_occ: float = 8.0) -> torch.Tensor:
    """(n,4) float32 copy of the cloud in a compact spatial order (8^3 blocks of
    grid cells, Morton order inside a block); column 3 holds the original
    int32 index bits (o3dx_spatial_sort_bounds).  The tensor carries
    `.absmax`, the cloud's |x|,|y|,|z| bounds from the sort's own bounds pass
    (the default fx quanta of ICPTarget.accumulate / register, which then
    skip their own measuring pass and host wait; a sharded source passes the
    global bounds instead), and `.absmax_of`, the cloud itself."""
    x = _xyz(xyz)
    L = N.load()
    n = x.shape[0]
    out = torch.empty((max(n, 1), 4), dtype=torch.float32, device=x.device)
    ws = N.workspace(L.o3dx_spatial_sort_workspace_bytes(n), x.device, "sort")
    am = np.zeros(3, np.float64)
    N.check(L.o3dx_spatial_sort_bounds(N.ptr(x), n, float(target_occ), N.ptr(out), _np_ptr(am), N.ptr(ws),
                                       ws.numel(), N.stream_ptr(x.device)), "spatial_sort")
    res = out[:n]
    res.absmax = am  # the sort's own bounds: ICP on it skips its absmax pass
    res.absmax_of = x
    return res


def icp_update(sums, T: np.ndarray) -> np.ndarray:
    """T <- solve(sums) * T in the library's own float64 order (o3dx_icp_update)."""
    TT = np.array(T, np.float64).reshape(4, 4).copy()
    rc = N.load().o3dx_icp_update(_np_ptr(_c(sums, np.float64)), _np_ptr(TT))
    if rc < 0:  # 1 solved, 0 singular (identity update, as Open3D), < 0 a library error
        N.check(rc, "icp_update")
    return TT


def icp_solve(sums) -> np.ndarray:
    upd = np.zeros((4, 4), np.float64)
    rc = N.load().o3dx_icp_solve_point_to_plane(_np_ptr(_c(sums, np.float64)), _np_ptr(upd))
    if rc < 0:
        N.check(rc, "icp_solve")
    return upd


def registration_icp(src: torch.Tensor, tgt: torch.Tensor, tgt_normals: torch.Tensor,
                     max_correspondence_distance: float, init=None, max_iteration: int = 30,
                     relative_fitness: float = 1e-6, relative_rmse: float = 1e-6, return_corr: bool = True):
    """Open3D registration_icp + TransformationEstimationPointToPlane on one device.
    A float64 source or target: both in float64 (o3dx_registration_icp_point_to_plane_f64)."""
    f64 = _is64(src) or _is64(tgt)
    cv = _xyz64 if f64 else _xyz
    s = cv(src, "source points")
    t = cv(tgt.to(s.device), "target points")
    tn = _xyz(tgt_normals.to(s.device), "target normals")
    L = N.load()
    ns, nt = s.shape[0], t.shape[0]
    T0 = np.eye(4) if init is None else _c(init, np.float64).reshape(4, 4)
    T0 = _c(T0, np.float64)
    T = np.zeros((4, 4), np.float64)
    fit = np.zeros(1)
    rm = np.zeros(1)
    corr = torch.empty((max(ns, 1), 2), dtype=torch.int32, device=s.device) if return_corr else None
    nc = np.zeros(1, np.int64)
    tws = N.workspace((L.o3dx_icp_target_f64_workspace_bytes if f64 else L.o3dx_icp_target_workspace_bytes)(nt),
                      s.device, "icp_target")
    ws = N.workspace((L.o3dx_registration_icp_f64_workspace_bytes if f64 else
                      L.o3dx_registration_icp_workspace_bytes)(ns), s.device, "icp")
    fn = L.o3dx_registration_icp_point_to_plane_f64 if f64 else L.o3dx_registration_icp_point_to_plane
    rc = fn(N.ptr(s), ns, N.ptr(t), N.ptr(tn), nt, float(max_correspondence_distance), _np_ptr(T0),
            int(max_iteration), float(relative_fitness), float(relative_rmse), _np_ptr(T), _np_ptr(fit),
            _np_ptr(rm), N.ptr(corr), _np_ptr(nc), N.ptr(tws), tws.numel(), N.ptr(ws), ws.numel(),
            N.stream_ptr(s.device))
    N.check(rc, "registration_icp")
    out = {"transformation": T, "fitness": float(fit[0]), "inlier_rmse": float(rm[0])}
    if return_corr:
        out["correspondence_set"] = corr[: int(nc[0])]
    return out


_absmax = absmax  # for ICPTarget.accumulate, whose parameter of that name shadows it
