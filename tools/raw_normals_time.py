"""estimate_normals(knn=30) on C3's raw planted-plane cloud (the sorted-grid
path): wall time and event-timed parts.  GPU box only.
Usage: python tools/raw_normals_time.py [n]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
dev = torch.device("cuda:0")
pts = S.planted_plane(n, seed=1, device=dev)
ops.estimate_normals(pts, knn=30)
torch.cuda.synchronize()
t0 = time.perf_counter()
ops.estimate_normals(pts, knn=30)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) * 1e3
N.set_kernel_timing(True)
N.reset_kernel_timing()
ops.estimate_normals(pts, knn=30)
torch.cuda.synchronize()
out = {"env": {k: v for k, v in os.environ.items() if k.startswith("O3DX_")}, "ms": round(el, 3)}
for name in ("grid_count", "grid_sort", "normals_nested", "normals_tile", "normals_wave", "normals_knn"):
    ms, c = N.kernel_timing(name)
    if c:
        out[name] = round(ms, 3)
N.search_stats(True)
ops.estimate_normals(pts, knn=30)
out["stats"] = N.search_stats()
N.search_stats(False)
print(json.dumps(out), flush=True)
