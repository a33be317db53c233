"""oracle/oracle.py — ctypes front-end of the CPU restatement (o3d_restate.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker / CPU baseline.  The product path
(open3dpypro + libo3dx.so) never imports this module.

Parity status of the Open3D-path restatement: "parity unpinned" — see the
header of o3d_restate.cpp and DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libo3dref.so")
_lib = None

KNN, RADIUS, HYBRID = 0, 1, 2

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int
_D = ctypes.c_double


def build() -> str:
    """Compile the oracle with its Makefile (gcc).  Returns the .so path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oref_num_threads.restype = _I32
        L.oref_set_num_threads.argtypes = [_I32]
        L.oref_aabb.argtypes = [_P, _I64, _P]
        L.oref_voxel_down_sample.argtypes = [_P, _I64, _P, _P, _D, _P, _P, _P, _P]
        L.oref_voxel_down_sample.restype = _I32
        L.oref_voxel_reps_parallel.argtypes = [_P, _I64, _P, _P, _D, _P, _P]
        L.oref_voxel_reps_parallel.restype = _I32
        L.oref_estimate_normals.argtypes = [_P, _I64, _I32, _I32, _D, _P, _P]
        L.oref_knn_search.argtypes = [_P, _I64, _P, _I64, _I32, _I32, _D, _I32, _P, _P, _P]
        L.oref_fast_eigen3x3.argtypes = [_P, _I64, _P]
        L.oref_fast_eigen3x3_nudged.argtypes = [_P, _I64, _I32, _P]
        L.oref_ransac_samples.argtypes = [_I64, _I32, _I32, ctypes.c_uint64, _P]
        L.oref_segment_plane.argtypes = [_P, _I64, _D, _I32, _I32, _D, _P, _P, _P, _P, _P, _P, _P]
        L.oref_segment_plane.restype = _I32
        L.oref_plane_from_points.argtypes = [_P, _P, _I64, _P]
        L.oref_registration_icp.argtypes = [_P, _I64, _P, _P, _I64, _D, _P, _I32, _D, _D,
                                            _P, _P, _P, _P, _P]
        L.oref_registration_icp.restype = _I32
        L.oref_icp_accumulate.argtypes = [_P, _I64, _P, _P, _I64, _D, _P, _P]
        L.oref_icp_accumulate_fx.argtypes = [_P, _I64, _P, _P, _I64, _D, _P, _P, _P]
        L.oref_icp_solve.argtypes = [_P, _P]
        L.oref_icp_solve.restype = _I32
        _lib = L
    return _lib


def _f64(a):
    """(n,3) float64 coordinates as Open3D stores them (Vector3dVector): a
    float32 cloud is upcast exactly, a float64 cloud is taken as is."""
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, 3))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def num_threads() -> int:
    return lib().oref_num_threads()


def set_num_threads(n: int) -> None:
    lib().oref_set_num_threads(int(n))


def aabb(xyz):
    x = _f64(xyz)
    mm = np.zeros(6, np.float64)
    lib().oref_aabb(_ptr(x), len(x), _ptr(mm))
    return mm[:3].copy(), mm[3:].copy()


PARALLEL_REPS_AT = 20_000_000


def voxel_down_sample(xyz, voxel_size, min_bound=None, max_bound=None, trace=False, parallel=None):
    """Returns (rep_idx ascending int32, voxel_of_point, cubic_id (M,8)) — the
    latter two only when trace=True.  Without trace, clouds of
    PARALLEL_REPS_AT points or more (or parallel=True) take
    oref_voxel_reps_parallel, the same function computed over hashed buckets."""
    x = _f64(xyz)
    n = len(x)
    if min_bound is None or max_bound is None:
        mn, mx = aabb(x)
        min_bound = mn if min_bound is None else min_bound
        max_bound = mx if max_bound is None else max_bound
    mnb = np.ascontiguousarray(min_bound, np.float64)
    mxb = np.ascontiguousarray(max_bound, np.float64)
    rep = np.empty(max(n, 1), np.int32)
    m = np.zeros(1, np.int64)
    if parallel is None:
        parallel = n >= PARALLEL_REPS_AT
    if parallel and not trace:
        rc = lib().oref_voxel_reps_parallel(_ptr(x), n, _ptr(mnb), _ptr(mxb), float(voxel_size),
                                            _ptr(rep), _ptr(m))
        if rc != 0:
            raise RuntimeError("voxel_size is invalid or too small")
        return rep[: int(m[0])].copy()
    vop = np.empty(max(n, 1), np.int32) if trace else None
    cub = np.empty(max(8 * n, 8), np.int32) if trace else None
    rc = lib().oref_voxel_down_sample(_ptr(x), n, _ptr(mnb), _ptr(mxb), float(voxel_size),
                                      _ptr(rep), _ptr(m), _ptr(vop), _ptr(cub))
    if rc != 0:
        raise RuntimeError("voxel_size is invalid or too small")
    M = int(m[0])
    if trace:
        return rep[:M].copy(), vop[:n].copy(), cub[: 8 * M].reshape(M, 8).copy()
    return rep[:M].copy()


def estimate_normals(xyz, mode=KNN, knn=30, radius=0.0, prior=None):
    x = _f64(xyz)
    out = np.zeros((len(x), 3), np.float64)
    pr = None if prior is None else np.ascontiguousarray(prior, np.float64).reshape(-1, 3)
    lib().oref_estimate_normals(_ptr(x), len(x), mode, knn, float(radius), _ptr(pr), _ptr(out))
    return out


def knn_search(xyz, queries, mode=KNN, knn=30, radius=0.0, K=None):
    x = _f64(xyz)
    q = _f64(queries)
    if K is None:
        K = knn
    idx = np.empty((len(q), K), np.int32)
    d2 = np.empty((len(q), K), np.float64)
    cnt = np.empty(len(q), np.int32)
    lib().oref_knn_search(_ptr(x), len(x), _ptr(q), len(q), mode, knn, float(radius), K,
                          _ptr(idx), _ptr(d2), _ptr(cnt))
    return idx, d2, cnt


def fast_eigen3x3(cov6):
    c = np.ascontiguousarray(cov6, np.float64).reshape(-1, 6)
    out = np.empty((len(c), 3), np.float64)
    lib().oref_fast_eigen3x3(_ptr(c), len(c), _ptr(out))
    return out


def fast_eigen3x3_nudged(cov6, nudge):
    """FastEigen3x3 with acos / cos results moved by one ulp (nudge: base-3
    digits, see o3d_restate.cpp) — the conditioning certificate."""
    c = np.ascontiguousarray(cov6, np.float64).reshape(-1, 6)
    out = np.empty((len(c), 3), np.float64)
    lib().oref_fast_eigen3x3_nudged(_ptr(c), len(c), int(nudge), _ptr(out))
    return out


def covariance(xyz, idx, cnt=None):
    """Open3D ComputeCovariance over neighbour rows idx (m,K) (first cnt[i]
    entries, in the given order — the kNN result order): sequential float64
    raw moments, {xx,xy,xz,yy,yz,zz}.  <3 neighbours -> identity."""
    p = np.asarray(xyz, np.float64).reshape(-1, 3)
    idx = np.asarray(idx).reshape(len(idx), -1)
    cnt = np.full(len(idx), idx.shape[1]) if cnt is None else np.asarray(cnt)
    out = np.zeros((len(idx), 6))
    for r in range(len(idx)):
        k = int(cnt[r])
        if k < 3:
            out[r] = [1, 0, 0, 1, 0, 1]
            continue
        m = np.zeros(9)
        for j in range(k):
            x, y, z = p[idx[r, j]]
            m += [x, y, z, x * x, x * y, x * z, y * y, y * z, z * z]
        u = m / k
        out[r] = [u[3] - u[0] * u[0], u[4] - u[0] * u[1], u[5] - u[0] * u[2], u[6] - u[1] * u[1],
                  u[7] - u[1] * u[2], u[8] - u[2] * u[2]]
    return out


def ransac_samples(n, ransac_n, iters, seed):
    out = np.empty((iters, ransac_n), np.int32)
    lib().oref_ransac_samples(n, ransac_n, iters, seed, _ptr(out))
    return out


def segment_plane(xyz, distance_threshold, ransac_n, num_iterations, samples,
                  probability=0.99999999):
    """Returns (plane[4], inliers int64 ascending, counts per hypothesis (-1 =
    degenerate), abs sums per hypothesis, best hypothesis index)."""
    x = _f64(xyz)
    n = len(x)
    s = np.ascontiguousarray(samples, np.int32).reshape(num_iterations, ransac_n)
    plane = np.zeros(4, np.float64)
    inl = np.empty(max(n, 1), np.int64)
    ninl = np.zeros(1, np.int64)
    counts = np.empty(num_iterations, np.int64)
    sums = np.empty(num_iterations, np.float64)
    best = np.zeros(1, np.int32)
    rc = lib().oref_segment_plane(_ptr(x), n, float(distance_threshold), ransac_n, num_iterations,
                                  float(probability), _ptr(s), _ptr(plane), _ptr(inl), _ptr(ninl),
                                  _ptr(counts), _ptr(sums), _ptr(best))
    if rc != 0:
        raise RuntimeError("segment_plane: invalid arguments")
    return plane, inl[: int(ninl[0])].copy(), counts, sums, int(best[0])


def plane_from_points(xyz, idx):
    x = _f64(xyz)
    i = np.ascontiguousarray(idx, np.int64)
    out = np.zeros(4, np.float64)
    lib().oref_plane_from_points(_ptr(x), _ptr(i), len(i), _ptr(out))
    return out


def registration_icp(src, tgt, tgt_normals, max_dist, init=None, max_iteration=30,
                     relative_fitness=1e-6, relative_rmse=1e-6):
    s = _f64(src)
    t = _f64(tgt)
    tn = _f64(tgt_normals)
    T0 = np.eye(4) if init is None else np.asarray(init, np.float64)
    T0 = np.ascontiguousarray(T0, np.float64)
    T = np.zeros((4, 4), np.float64)
    fit = np.zeros(1)
    rm = np.zeros(1)
    corr = np.empty((max(len(s), 1), 2), np.int32)
    nc = np.zeros(1, np.int64)
    rc = lib().oref_registration_icp(_ptr(s), len(s), _ptr(t), _ptr(tn), len(t), float(max_dist),
                                     _ptr(T0), int(max_iteration), float(relative_fitness),
                                     float(relative_rmse), _ptr(T), _ptr(fit), _ptr(rm), _ptr(corr),
                                     _ptr(nc))
    if rc != 0:
        raise RuntimeError("registration_icp: invalid arguments")
    return T, float(fit[0]), float(rm[0]), corr[: int(nc[0])].copy()


def icp_accumulate(src, tgt, tgt_normals, max_dist, T):
    s = _f64(src)
    t = _f64(tgt)
    tn = _f64(tgt_normals)
    TT = np.ascontiguousarray(T, np.float64)
    sums = np.zeros(32, np.float64)
    lib().oref_icp_accumulate(_ptr(s), len(s), _ptr(t), _ptr(tn), len(t), float(max_dist),
                              _ptr(TT), _ptr(sums))
    return sums


def icp_accumulate_fx(src, tgt, tgt_normals, max_dist, T, absmax):
    """The same sums as exact fx rows (32, 4) int64 {lo, hi, q, 0} (the
    order-free form libo3dx uses; restated with 128-bit integers)."""
    s = _f64(src)
    t = _f64(tgt)
    tn = _f64(tgt_normals)
    TT = np.ascontiguousarray(T, np.float64)
    am = np.ascontiguousarray(absmax, np.float64).reshape(3)
    fx = np.zeros((32, 4), np.int64)
    lib().oref_icp_accumulate_fx(_ptr(s), len(s), _ptr(t), _ptr(tn), len(t), float(max_dist), _ptr(TT), _ptr(am),
                                 _ptr(fx))
    return fx


def icp_solve(sums):
    s = np.ascontiguousarray(sums, np.float64)
    upd = np.zeros((4, 4), np.float64)
    ok = lib().oref_icp_solve(_ptr(s), _ptr(upd))
    return upd, bool(ok)
