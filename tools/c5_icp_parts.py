"""C5's ICP stage in parts (GPU box only): target grid build (ICPTarget),
source spatial sort, the 30-iteration device loop — wall times after a
warm-up, and the library kernel timers of the loop.
Usage: python tools/c5_icp_parts.py [n] [source-sort occupancy targets, e.g. 8,16,32]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
occs = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [8.0]
vs = 0.0005
tgt = S.box_surface(n, seed=1, device=dev)
treps = ops.voxel_down_sample(tgt, vs)["rep_xyz"].clone()
del tgt
src = S.apply_transform(S.box_surface(n, seed=2, device=dev), S.rigid_transform())
sreps = ops.voxel_down_sample(src, vs)["rep_xyz"].clone()
del src
torch.cuda.empty_cache()
tn = ops.estimate_normals(treps, knn=30)


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, round((time.perf_counter() - t0) * 1e3, 3)


for rep, occ in [(r, o) for o in occs for r in range(2)]:
    target, t_build = wall(lambda: ops.ICPTarget(treps, tn, 0.02))
    s4, t_sort = wall(lambda: ops.spatial_sort(sreps, occ))
    N.set_kernel_timing(True)
    N.reset_kernel_timing()
    reg, t_loop = wall(lambda: target.register(s4, max_iteration=30, relative_fitness=0.0, relative_rmse=0.0))
    kt = {}
    for k in ("icp_loop", "icp_match", "icp_accumulate"):
        ms, c = N.kernel_timing(k)
        if c:
            kt[k] = [round(ms, 3), c]
    N.set_kernel_timing(False)
    print(json.dumps({"rep": rep, "sort_occ": occ, "n_tgt": int(treps.shape[0]), "n_src": int(sreps.shape[0]),
                      "target_build_ms": t_build, "source_sort_ms": t_sort, "loop_ms": t_loop, "timers": kt,
                      "fitness": reg["fitness"]}), flush=True)
