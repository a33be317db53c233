"""C3's ICP loop (bench.py's ICP leg: 10M box surface, 30 iterations from
T = I, o3dx_icp_register) timed on a library given by O3DX_LIB (A/B of
builds).  GPU box tool.  Usage: O3DX_LIB=path python tools/icp_loop_time.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N  # noqa: E402

if os.environ.get("O3DX_LIB"):
    N.LIB_PATH = os.environ["O3DX_LIB"]
from open3dpypro import ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
n = 10_000_000
tgt = S.box_surface(n, seed=1, device=dev)
src = S.apply_transform(S.box_surface(n, seed=2, device=dev), S.rigid_transform())
tn = ops.estimate_normals(tgt, knn=30)
target = ops.ICPTarget(tgt, tn, 0.02)
src4 = ops.spatial_sort(src)
target.register(src4, max_iteration=1, relative_fitness=0.0, relative_rmse=0.0)
ts = []
for _ in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = target.register(src4, max_iteration=30, relative_fitness=0.0, relative_rmse=0.0)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
err = np.abs(res["transformation"] - np.linalg.inv(S.rigid_transform())).max()
print(f"{os.path.basename(N.LIB_PATH)} it/s={30 / min(ts):.1f} ms={[round(t * 1e3, 2) for t in ts]} T_err={err:.2e} "
      f"fit={res['fitness']:.6f}", flush=True)
