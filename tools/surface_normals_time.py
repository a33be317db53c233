"""estimate_normals(knn=30) on a 10M box-surface cloud (C3's ICP target): the
sorted-grid path with and without the nested grid (O3DX_NESTED_OFF), timed
parts and search stats.  GPU box only."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
pts = S.box_surface(10_000_000, seed=1, device=dev)
# argv: NAME=VAL[,NAME=VAL] configurations (default: nested on / off)
cfgs = [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[1:]] or [{}, {"O3DX_NESTED_OFF": "1"}]
keys = {k for c in cfgs for k in c}
for env in cfgs:
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update(env)
    a = ops.estimate_normals(pts, knn=30)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a = ops.estimate_normals(pts, knn=30)
    torch.cuda.synchronize()
    out = {"env": env, "ms": round((time.perf_counter() - t0) * 1e3, 3)}
    N.set_kernel_timing(True)
    N.reset_kernel_timing()
    ops.estimate_normals(pts, knn=30)
    torch.cuda.synchronize()
    for name in ("grid_count", "grid_sort", "normals_nested", "normals_tile", "normals_wave", "normals_knn"):
        ms, c = N.kernel_timing(name)
        if c:
            out[name] = round(ms, 3)
    N.set_kernel_timing(False)
    N.search_stats(True)
    ops.estimate_normals(pts, knn=30)
    out["stats"] = N.search_stats()
    N.search_stats(False)
    print(json.dumps(out), flush=True)
