"""C2's voxel-table normals with the device search statistics on: stile
hand-offs (stats[4]), list overflows (stats[5]), beyond-range (stats[7]) and
the wave form's counters.  Usage (GPU box): python tools/stile_stats.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))

import torch  # noqa: E402

from open3dpypro import _native, ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
N = int(os.environ.get("N", "10000000"))
pts = S.uniform_cube(N, 0, device=dev)
vd = ops.voxel_down_sample(pts, S.voxel_size_for(N), keep_grid=True)
reps, vg = vd["rep_xyz"], vd["voxel_grid"]
ops.estimate_normals(reps, knn=30, voxel_grid=vg)
_native.search_stats(True)
ops.estimate_normals(reps, knn=30, voxel_grid=vg)
st = _native.search_stats()
_native.search_stats(False)
print(json.dumps({"reps": int(reps.shape[0]), "stats": st}))
