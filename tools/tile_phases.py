"""Phase budget of the sorted-grid tile kernel (k_normals_knn_tile) on surface
clouds: O3DX_TILE_DEBUG=1/2/3/4 stop after staging / histogram / list scan /
moments (profiling only: wrong normals).  Cases: the 10M box surface (C3's
ICP target) and C5's target reps (box surface, 200M points at vs 0.5 mm;
argv[1] = that N, 0 skips it).  GPU box only."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")


def phases(name, pts):
    out = {"case": name, "n": int(pts.shape[0])}
    for dbg in ("1", "2", "3", "4", ""):
        if dbg:
            os.environ["O3DX_TILE_DEBUG"] = dbg
        else:
            os.environ.pop("O3DX_TILE_DEBUG", None)
        ops.estimate_normals(pts, knn=30)
        torch.cuda.synchronize()
        N.set_kernel_timing(True)
        N.reset_kernel_timing()
        for _ in range(3):
            ops.estimate_normals(pts, knn=30)
        torch.cuda.synchronize()
        ms, c = N.kernel_timing("normals_tile")
        N.set_kernel_timing(False)
        out["tile_dbg" + (dbg or "off")] = round(ms / max(c, 1), 3)
    os.environ.pop("O3DX_TILE_DEBUG", None)
    print(json.dumps(out), flush=True)


pts = S.box_surface(10_000_000, seed=1, device=dev)
phases("box_surface_10M", pts)
del pts
c5n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
if c5n:
    tgt = S.box_surface(c5n, seed=1, device=dev)
    treps = ops.voxel_down_sample(tgt, 0.0005)["rep_xyz"].clone()
    del tgt
    torch.cuda.empty_cache()
    phases("c5_target_reps", treps)
