"""Focused driver for rocprofv3 (kernel trace / PMC): normals on the C2 reps,
converged ICP accumulate, RANSAC, the RANSAC count alone, ICP's first
iteration; a few launches each.  GPU box only.
Usage: python tools/prof_kernels.py [all|normals|icp|icp_loop|ransac|ransac_upper|ransac_count|icp_first]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from open3dpypro import ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
N = int(os.environ.get("N", "10000000"))
what = sys.argv[1] if len(sys.argv) > 1 else "all"
if what in ("all", "normals"):
    pts = S.uniform_cube(N, 0, device=dev)
    vd = ops.voxel_down_sample(pts, S.voxel_size_for(N), keep_grid=True)
    reps, vg = vd["rep_xyz"], vd["voxel_grid"]
    for _ in range(3):
        ops.estimate_normals(reps, knn=30, voxel_grid=vg)
    torch.cuda.synchronize()
    del pts, reps, vd, vg
if what in ("all", "icp"):
    tgt = S.box_surface(N, 1, device=dev)
    src = S.apply_transform(S.box_surface(N, 2, device=dev), S.rigid_transform())
    tn = ops.estimate_normals(tgt, knn=30)
    target = ops.ICPTarget(tgt, tn, 0.02)
    src4 = ops.spatial_sort(src)
    T = np.linalg.inv(S.rigid_transform())
    for _ in range(3):
        sums, _ = target.accumulate(src4, T)
    torch.cuda.synchronize()
if what == "icp_loop":  # the device loop (o3dx_icp_register) from T = I: 30 steps, prior matches from step 2
    tgt = S.box_surface(N, 1, device=dev)
    src = S.apply_transform(S.box_surface(N, 2, device=dev), S.rigid_transform())
    tn = ops.estimate_normals(tgt, knn=30)
    target = ops.ICPTarget(tgt, tn, 0.02)
    src4 = ops.spatial_sort(src)
    target.register(src4, max_iteration=30, relative_fitness=0.0, relative_rmse=0.0)
    torch.cuda.synchronize()
if what in ("all", "ransac"):
    pts = S.planted_plane(N, 3, device=dev)
    samples = ops.ransac_samples(N, 3, 1000, seed=7)
    for _ in range(2):
        ops.segment_plane(pts, 0.01, 3, 1000, samples=samples)
    torch.cuda.synchronize()
if what == "ransac_upper":  # the upper-bound sweep alone (O3DX_RANSAC_UPPER picks it), three calls
    pts = S.planted_plane(N, 3, device=dev)
    idx = np.random.default_rng(0).integers(0, N, (1000, 3))
    p64 = pts.cpu().numpy().astype(np.float64)
    a, b, c = p64[idx[:, 0]], p64[idx[:, 1]], p64[idx[:, 2]]
    nrm = np.cross(b - a, c - a)
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-300)
    planes = np.concatenate([nrm, -np.sum(nrm * a, 1, keepdims=True)], 1)
    for _ in range(3):
        ops.plane_count_upper(pts, planes, 0.01)
    torch.cuda.synchronize()
if what == "ransac_count":
    pts = S.planted_plane(N, 3, device=dev)
    idx = np.random.default_rng(0).integers(0, N, (1000, 3))
    p64 = pts.cpu().numpy().astype(np.float64)
    a, b, c = p64[idx[:, 0]], p64[idx[:, 1]], p64[idx[:, 2]]
    nrm = np.cross(b - a, c - a)
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-300)
    planes = np.concatenate([nrm, -np.sum(nrm * a, 1, keepdims=True)], 1)
    for _ in range(3):
        ops.plane_count(pts, planes, 0.01)
    torch.cuda.synchronize()
if what == "icp_first":  # the T = I iteration of C3's ICP (source displaced by T_gt)
    tgt = S.box_surface(N, 1, device=dev)
    src = S.apply_transform(S.box_surface(N, 2, device=dev), S.rigid_transform())
    tn = ops.estimate_normals(tgt, knn=30)
    target = ops.ICPTarget(tgt, tn, 0.02)
    src4 = ops.spatial_sort(src)
    for _ in range(3):
        sums, _ = target.accumulate(src4, np.eye(4))
    torch.cuda.synchronize()
print("done")
