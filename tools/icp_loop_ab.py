"""A/B of the device ICP loop (o3dx_icp_register) at C3: 10M box-surface
source / target, 30 iterations from T = I; per-step kernel times.  Run once
per library (O3DX_LIB selects a variant).  Usage: python tools/icp_loop_ab.py [n] [iters] [reps]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda:0")
tgt = S.box_surface(n, seed=1, device=dev)
src = S.apply_transform(S.box_surface(n, seed=2, device=dev), S.rigid_transform())
tn = ops.estimate_normals(tgt, knn=30)
target = ops.ICPTarget(tgt, tn, 0.02)
s4 = ops.spatial_sort(src)
target.register(s4, max_iteration=2, relative_fitness=0.0, relative_rmse=0.0)
times = []
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = target.register(s4, max_iteration=iters, relative_fitness=0.0, relative_rmse=0.0)
    torch.cuda.synchronize()
    times.append(time.perf_counter() - t0)
N.set_kernel_timing(True)
N.reset_kernel_timing()
target.register(s4, max_iteration=iters, relative_fitness=0.0, relative_rmse=0.0)
torch.cuda.synchronize()
m, nm = N.kernel_timing("icp_match")
N.set_kernel_timing(False)
el = min(times)
print(json.dumps({"lib": os.path.basename(os.environ.get("O3DX_LIB", "in-tree")), "iters_per_s": round(iters / el, 1),
                  "ms_per_iter": round(el / iters * 1e3, 4), "match_ms_avg": round(m / max(nm, 1), 4),
                  "T": np.asarray(res["transformation"]).round(14).tolist(), "fitness": res["fitness"]}), flush=True)
