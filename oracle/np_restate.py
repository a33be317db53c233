"""oracle/np_restate.py — small-N numpy restatement of the same Open3D algorithms.

TEST INFRASTRUCTURE ONLY (see oracle/oracle.py).  A second, independent
transcription used to cross-check the C++ restatement on small inputs; it is
written with numpy vector ops / brute force so that the two share no code.
"""
from __future__ import annotations

import math

import numpy as np


def voxel_down_sample(xyz, voxel_size, min_bound=None):
    """Open3D VoxelDownSampleAndTrace + idxmat.max(1) + _select_by_idx
    (reference PointCloud.py:338-341, :185-204): representative = largest
    index per voxel, keys floor((p - min_bound)/vs) in float64; returns the
    ascending representative indices."""
    p = np.asarray(xyz, np.float64).reshape(-1, 3)
    if len(p) == 0:
        return np.zeros(0, np.int64)
    mn = p.min(0) if min_bound is None else np.asarray(min_bound, np.float64)
    keys = np.floor((p - mn) / voxel_size).astype(np.int64)
    # lexicographic group id; representative = max index in group
    _, inv = np.unique(keys, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    rep = np.full(inv.max() + 1, -1, np.int64)
    np.maximum.at(rep, inv, np.arange(len(p)))
    return np.sort(rep)


def nanoflann_d2(q, pts):
    d = pts - q
    r = d[:, 0] * d[:, 0]
    r = r + d[:, 1] * d[:, 1]
    r = r + d[:, 2] * d[:, 2]
    return r


def neighbours(pts, q, mode, knn, radius):
    """KDTreeFlann::Search by brute force; (d2, idx) lexicographic order."""
    d2 = nanoflann_d2(q, pts)
    order = np.lexsort((np.arange(len(pts)), d2))
    if mode == 1:  # radius
        order = order[d2[order] < radius * radius]
        return order
    order = order[:knn]
    if mode == 2:  # hybrid
        order = order[d2[order] < radius * radius]
    return order


def covariance(pts, idx):
    if len(idx) == 0:
        return np.eye(3)
    m = np.zeros(9)
    for i in idx:
        x, y, z = pts[i]
        m += [x, y, z, x * x, x * y, x * z, y * y, y * z, z * z]
    m /= len(idx)
    c = np.empty((3, 3))
    c[0, 0] = m[3] - m[0] * m[0]
    c[1, 1] = m[6] - m[1] * m[1]
    c[2, 2] = m[8] - m[2] * m[2]
    c[0, 1] = c[1, 0] = m[4] - m[0] * m[1]
    c[0, 2] = c[2, 0] = m[5] - m[0] * m[2]
    c[1, 2] = c[2, 1] = m[7] - m[1] * m[2]
    return c


def smallest_eigvec(c):
    """Reference answer up to sign (numpy eigh)."""
    w, v = np.linalg.eigh(c)
    return v[:, 0], w


def plane_dist(plane, pts):
    a, b, c, d = plane
    return np.abs((a * pts[:, 0] + c * pts[:, 2]) + (b * pts[:, 1] + d))


def triangle_plane(p0, p1, p2):
    e0 = p1 - p0
    e1 = p2 - p0
    abc = np.array([e0[1] * e1[2] - e0[2] * e1[1],
                    e0[2] * e1[0] - e0[0] * e1[2],
                    e0[0] * e1[1] - e0[1] * e1[0]])
    nrm = math.sqrt((abc[0] * abc[0] + abc[1] * abc[1]) + abc[2] * abc[2])
    if nrm == 0:
        return np.zeros(4)
    abc = abc / nrm
    d = -((abc[0] * p0[0] + abc[1] * p0[1]) + abc[2] * p0[2])
    return np.array([abc[0], abc[1], abc[2], d])


def segment_plane_counts(xyz, thr, samples):
    """Per-hypothesis exact inlier counts (ransac_n == 3) — EvaluateRANSACBasedOnDistance."""
    p = np.asarray(xyz, np.float64).reshape(-1, 3)
    out = []
    for s in np.asarray(samples).reshape(-1, 3):
        pl = triangle_plane(p[s[0]], p[s[1]], p[s[2]])
        if not pl.any():
            out.append(-1)
            continue
        out.append(int((plane_dist(pl, p) < thr).sum()))
    return np.array(out, np.int64)


def remove_statistical_outlier(xyz, nb_neighbors, std_ratio, knn_d2):
    """Open3D PointCloud::RemoveStatisticalOutliers (0.19, geometry/
    PointCloud.cpp; the reference calls it at PointCloud.py:370-372):
    mean of sqrt(d2) over the nb_neighbors nearest (self included; the
    kd-tree's ascending order, std::accumulate), cloud mean over the positive
    means (std::accumulate, index order), sum of squared deviations
    (std::inner_product, index order), std with n - 1, keep
    0 < mean < cloud_mean + std_ratio * std.  knn_d2: (n, k) float64 squared
    distances of the kNN search (oracle.knn_search)."""
    d2 = np.asarray(knn_d2, np.float64)
    n = d2.shape[0]
    if n == 0:
        return np.zeros(0, np.int64)
    k = min(nb_neighbors, n)
    d = np.sqrt(d2[:, :k])
    acc = np.zeros(n)
    for j in range(k):
        acc = acc + d[:, j]
    avg = acc / k
    pos = avg > 0
    m = np.add.accumulate(np.where(pos, avg, 0.0))[-1] / n
    sq = np.add.accumulate(np.where(pos, (avg - m) * (avg - m), 0.0))[-1]
    with np.errstate(divide="ignore", invalid="ignore"):
        std = np.sqrt(sq / np.float64(n - 1))
    thr = m + std_ratio * std
    return np.nonzero(pos & (avg < thr))[0].astype(np.int64)


# ---------------------------------------------------------------------------
# Restatements of the reference's own torch branches (pinned by
# tests/golden/ref_torch_branch.npz, generated from the reference itself).

def voxel_torch_hash(xyz, voxel_size):
    """Processors.VoxelDownsample cuda branch (reference processors.py:433-448):
    int32 keys floor(p/vs), hash x*73856093 + y*19349663 + z*83492791 (int32
    wrap), one representative per hash value, output in ascending (signed)
    hash order.  Which member represents a group is whatever the reference's
    unstable torch.sort puts first (the golden vector shows min, max and
    middle members): unspecified.  This restatement returns the lowest index;
    the fixture pins the group set and order, not the member."""
    p = np.asarray(xyz, np.float32)
    v = np.floor(p / np.float32(voxel_size)).astype(np.int32)
    with np.errstate(over="ignore"):
        key = (v[:, 0] * np.int32(73856093) + v[:, 1] * np.int32(19349663) + v[:, 2] * np.int32(83492791))
    key = key.astype(np.int32)
    order = np.lexsort((np.arange(len(p)), key))
    ks = key[order]
    first = np.ones(len(ks), bool)
    first[1:] = ks[1:] != ks[:-1]
    return order[first]


def torch_hash_keys(xyz, voxel_size):
    p = np.asarray(xyz, np.float32)
    v = np.floor(p / np.float32(voxel_size)).astype(np.int64)
    key = v[:, 0] * 73856093 + v[:, 1] * 19349663 + v[:, 2] * 83492791
    return ((key + 2 ** 31) % 2 ** 32 - 2 ** 31).astype(np.int32)


def ransac_batched_fp32(xyz, thr, samples, batch):
    """PlaneDetection.ransac_plane_detection_torch_batched (reference
    processors.py:561-627) given its sampled triples: float32 planes flipped
    to d >= 0, counts |p.n + d| < thr, first strict improvement over batches."""
    p = np.asarray(xyz, np.float32)
    best_c, best = 0, None
    for b0 in range(0, len(samples), batch):
        s = samples[b0:b0 + batch]
        p1, p2, p3 = p[s[:, 0]], p[s[:, 1]], p[s[:, 2]]
        nrm = np.cross(p2 - p1, p3 - p1).astype(np.float32)
        ln = np.linalg.norm(nrm, axis=1, keepdims=True).astype(np.float32)
        nrm = nrm / np.maximum(ln, np.float32(1e-6))
        d = -(nrm * p1).sum(1).astype(np.float32)
        flip = d < 0
        nrm[flip] = -nrm[flip]
        d[flip] = -d[flip]
        dist = np.abs(p @ nrm.T + d)
        cnt = (dist < np.float32(thr)).sum(0)
        j = int(np.argmax(cnt))
        if cnt[j] > best_c:
            best_c = int(cnt[j])
            best = np.concatenate([nrm[j], [d[j]]]).astype(np.float64)
    return best, best_c


# ---------------------------------------------------------------------------
# Exact order-free ("fx") sums — the form libo3dx gives every float sum that
# may cross GPUs (include/o3dx.h, o3dx_plane_moments note), restated in numpy:
# each term rounded to the nearest integer multiple of 2^q (ties to even),
# q = frexp-exponent(B) - 51 for a bound B of the terms, integers added.

def fx_exp(B):
    b = float(B) if (B > 0 and math.isfinite(B)) else 1.0
    return math.frexp(max(b, math.ldexp(1.0, -900)))[1] - 51


def fx_row(terms, q):
    """fx row {lo, hi, q, 0} of float64 terms at exponent q."""
    v = np.rint(np.ldexp(np.asarray(terms, np.float64), -q)).astype(np.int64)
    return np.array([int((v & 0xFFFFFFFF).sum()), int((v >> 32).sum()), q, 0], np.int64)


def fx_value(row):
    """float64 value of an fx row (Python's int -> float rounding: to nearest, ties to even)."""
    lo, hi, q = int(row[0]), int(row[1]), int(row[2])
    return math.ldexp(float((hi << 32) + lo), q)


def plane_abs_sum_fx(pts, plane, thr):
    """Sigma |d| over |d| < thr (EvaluateRANSACBasedOnDistance's error sum) as an fx row."""
    d = plane_dist(plane, np.asarray(pts, np.float64).reshape(-1, 3))
    return fx_row(d[d < thr], fx_exp(thr))


def plane_moments_fx(pts, A, centroid=None):
    """GetPlaneFromPoints' sums over pts as fx rows: {x, y, z} (q from A, the
    cloud's largest |coordinate|) or, with the centroid, centred {xx, xy, xz,
    yy, yz, zz} (q from 4 A^2 * 1.01)."""
    p = np.asarray(pts, np.float64).reshape(-1, 3)
    if centroid is None:
        q = fx_exp(A)
        return np.stack([fx_row(p[:, a], q) for a in range(3)])
    r = p - np.asarray(centroid, np.float64)
    q = fx_exp(4.0 * A * A * 1.01)
    pairs = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]
    return np.stack([fx_row(r[:, a] * r[:, b], q) for a, b in pairs])


# ---------------------------------------------------------------------------
# The reference's processor glue around the hot path, restated for value
# parity (reference open3dpypro/processors.py; these are its own formulas —
# numpy or torch, in the data's dtype — not Open3D's).

def rotation_matrix_from_vectors_ref(vec1, vec2, lib, device=None):
    """PlaneNormalize.rotation_matrix_from_vectors (processors.py:709-723)."""
    if lib == "torch":
        import torch
        norm, cross, eye, dot = torch.norm, (lambda a, b: torch.cross(a, b, dim=-1)), torch.eye, torch.dot
        mat = lambda l, dtype: torch.tensor(l, dtype=dtype, device=device)  # noqa: E731
        mm = torch.matmul
        eye_ = lambda n, dtype: torch.eye(n, dtype=dtype, device=device)  # noqa: E731
    else:
        norm, cross, dot = np.linalg.norm, (lambda a, b: np.cross(a, b, axis=-1)), np.dot
        mat = lambda l, dtype: np.array(l, dtype=dtype)  # noqa: E731
        mm = lambda a, b: a @ b  # noqa: E731
        eye_ = lambda n, dtype: np.eye(n, dtype=dtype)  # noqa: E731
    a = vec1 / norm(vec1)
    b = vec2 / norm(vec2)
    v = cross(a, b)
    if norm(v) < 1e-6:
        return eye_(3, a.dtype)
    c = dot(a, b)
    s = norm(v)
    kmat = mat([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]], a.dtype)
    return eye_(3, a.dtype) + kmat + mm(kmat, kmat) * ((1 - c) / (s ** 2))


def rotate_to_plane_ref(pcd, plane):
    """PlaneNormalize.rotate_to_plane (processors.py:725-744): T in the data's
    dtype, applied as (T @ [xyz | 1]^T)^T.  Returns (xyz', T)."""
    a, b, c, d = plane
    if hasattr(pcd, "device") and not isinstance(pcd, np.ndarray):
        import torch
        lib, dev = "torch", pcd.device
        mat = lambda l: torch.tensor(l, dtype=pcd.dtype, device=dev)  # noqa: E731
        normal, z = mat([a, b, c]), mat([0, 0, 1])
        R = rotation_matrix_from_vectors_ref(normal, z, lib, dev)
        pop = -d * normal / torch.dot(normal, normal)
        t = -torch.matmul(R, pop)
        T = torch.eye(4, dtype=pcd.dtype, device=dev)
        T[:3, :3] = R
        T[:3, 3] = t
        homo = torch.cat([pcd[:, :3], torch.ones((pcd.shape[0], 1), dtype=pcd.dtype, device=dev)], dim=1)
        return torch.matmul(T, homo.T).T[:, :3], T
    normal = np.array([a, b, c], dtype=pcd.dtype)
    z = np.array([0, 0, 1], dtype=pcd.dtype)
    R = rotation_matrix_from_vectors_ref(normal, z, "numpy")
    pop = -d * normal / np.dot(normal, normal)
    t = -(R @ pop)
    T = np.eye(4, dtype=pcd.dtype)
    T[:3, :3] = R
    T[:3, 3] = t
    homo = np.hstack([pcd[:, :3], np.ones((pcd.shape[0], 1), dtype=pcd.dtype)])
    return (T @ homo.T).T[:, :3], T


def plane_flip_ref(plane_model):
    """PlaneDetection.cpu_model's orientation (processors.py:640-650, 644-646): flip so
    the sensor origin lies on the normal's side."""
    plane_model = np.asarray(plane_model)
    n, d = plane_model[:3], plane_model[3]
    v = np.zeros(3) - (-d * n)
    return -plane_model if np.dot(n, v) < 0 else plane_model


def ema_ref(best, plane, alpha):
    """PlaneDetection.forward_raw's blend (processors.py:697)."""
    return (np.asarray(best) * (1.0 - alpha) + plane * alpha).tolist()
