"""Sparse-grid voxel down-sample timing (C5's box-surface scene at vs 0.5 mm):
hash-binned LDS reduction vs the global hash table.  GPU box tool."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open3d-py-extension_amd"))
from open3dpypro import ops, synthetic as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
dev = torch.device("cuda:0")
pts = S.box_surface(n, seed=1, device=dev)
torch.cuda.synchronize()
ref = None
for name, env in (("hbin", "0"), ("global_hash", "-1"), ("hbin", "0")):
    os.environ["O3DX_VOXEL_HBIN_MIN"] = env
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = ops.voxel_down_sample(pts, 0.0005)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    rep = out["rep_idx"]
    if ref is None:
        ref = rep
    print(f"{name:12s} n={n} m={rep.numel()} ms={['%.2f' % t for t in ts]} equal={torch.equal(rep, ref)}",
          flush=True)
    del out
