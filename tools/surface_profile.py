"""Surface-cloud normals (KNN30): where the time goes.  (a) C5's target:
voxel reps of a box surface at vs = 0.5 mm (N points, default 200M), (b) the
raw 10M box-surface cloud (C3's ICP target).  Per case: wall time, library
kernel timers, search stats (hand-offs).  GPU box only.
Usage: python tools/surface_profile.py [c5_n]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
NAMES = ("grid_count", "grid_sort", "grid_voxel", "normals_nested", "normals_tile", "normals_wave", "normals_knn",
         "normals_stile")


def profile(name, fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    out = {"case": name, "ms": round((time.perf_counter() - t0) * 1e3, 3)}
    N.set_kernel_timing(True)
    N.reset_kernel_timing()
    fn()
    torch.cuda.synchronize()
    for k in NAMES:
        ms, c = N.kernel_timing(k)
        if c:
            out[k] = round(ms, 3)
    N.set_kernel_timing(False)
    N.search_stats(True)
    fn()
    torch.cuda.synchronize()
    out["stats"] = N.search_stats()
    N.search_stats(False)
    print(json.dumps(out), flush=True)


c5n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
tgt = S.box_surface(c5n, seed=1, device=dev)
vt = ops.voxel_down_sample(tgt, 0.0005, keep_grid=True)
del tgt
treps = vt["rep_xyz"].clone()
print(json.dumps({"c5_reps": int(treps.shape[0]), "voxel_grid": vt.get("voxel_grid") is not None}), flush=True)
del vt
torch.cuda.empty_cache()
profile("c5_target_reps", lambda: ops.estimate_normals(treps, knn=30))
del treps
torch.cuda.empty_cache()
pts = S.box_surface(10_000_000, seed=1, device=dev)
profile("box_surface_10M", lambda: ops.estimate_normals(pts, knn=30))
