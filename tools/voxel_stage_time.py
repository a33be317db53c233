"""Voxel stage timing on the GPU box: C2 (10M uniform, dense one-pass
binning) and C5 (200M box surface at 0.5 mm, hash-binned), per variant of
the env switches given on the command line, checked equal to the first
variant's representatives.  Library HIP-event timers (voxel_assign =
binning + reduce, voxel_compact = flag compaction) plus the wall time of the
whole call.
Usage: python tools/voxel_stage_time.py c2|c4|c5 [VAR=a,b ...]
e.g.   python tools/voxel_stage_time.py c2 O3DX_VOXEL_COPIES=4,8"""
import itertools
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "c2"
axes = []
for a in sys.argv[2:]:
    k, v = a.split("=", 1)
    axes.append([(k, x) for x in v.split(",")])
dev = torch.device("cuda:0")
if which in ("c2", "c4"):
    n = 10_000_000 if which == "c2" else 50_000_000
    pts = S.uniform_cube(n, 0, device=dev)
    vs, keep = S.voxel_size_for(n), True
else:
    n = 200_000_000
    pts = S.box_surface(n, seed=1, device=dev)
    vs, keep = 0.0005, False
torch.cuda.synchronize()
ref = None
for combo in itertools.product(*axes) if axes else [()]:
    for k, v in combo:
        os.environ[k] = v
    for _ in range(3):
        out = ops.voxel_down_sample(pts, vs, keep_grid=keep)
    torch.cuda.synchronize()
    N.set_kernel_timing(True)
    N.reset_kernel_timing()
    reps = 10 if which != "c5" else 4
    t0 = time.perf_counter()
    for _ in range(reps):
        out = ops.voxel_down_sample(pts, vs, keep_grid=keep)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e3
    a_ms, a_n = N.kernel_timing("voxel_assign")
    c_ms, c_n = N.kernel_timing("voxel_compact")
    N.set_kernel_timing(False)
    rep = out["rep_idx"]
    if ref is None:
        ref = rep.clone()
    print(f"{which} {dict(combo)} m={rep.numel()} wall={wall:.3f} ms assign={a_ms / max(a_n, 1):.4f} "
          f"compact={c_ms / max(c_n, 1):.4f} equal={torch.equal(rep, ref)}", flush=True)
    del out
