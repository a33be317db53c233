"""A/B of the float64 normals (a 10M-point LAS-like scan's 5 cm reps, KNN30):
wall time per call and the library timers.  O3DX_LIB selects a variant.
Usage: python tools/f64_normals_ab.py [n]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
las = S.las_scene(n, seed=0, device=dev)
reps = ops.voxel_down_sample(las, 0.05)["rep_xyz"].clone()
del las
a = ops.estimate_normals(reps, knn=30)
ts = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b = ops.estimate_normals(reps, knn=30)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
N.set_kernel_timing(True)
N.reset_kernel_timing()
ops.estimate_normals(reps, knn=30)
torch.cuda.synchronize()
kt = {k: round(N.kernel_timing(k)[0], 3) for k in ("normals_f64", "normals_tile64", "normals_wave64", "grid_count", "grid_sort")}
N.set_kernel_timing(False)
print(json.dumps({"lib": os.path.basename(os.environ.get("O3DX_LIB", "in-tree")),
                  "no_tiles": os.environ.get("O3DX_F64_NO_TILES"), "no_wave": os.environ.get("O3DX_F64_NO_WAVE"), "reps": int(reps.shape[0]),
                  "ms_min": round(min(ts), 3), "timers": kt, "same": bool(torch.equal(a, b))}), flush=True)
