"""Focused driver for rocprofv3 (kernel trace / PMC): normals on the C2 reps
and converged ICP accumulate, a few launches each.  GPU box only."""
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
if what in ("all", "ransac"):
    pts = S.planted_plane(N, 3, device=dev)
    samples = ops.ransac_samples(N, 3, 1000, seed=7)
    for _ in range(2):
        ops.segment_plane(pts, 0.01, 3, 1000, samples=samples)
    torch.cuda.synchronize()
print("done")
