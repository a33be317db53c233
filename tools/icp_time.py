"""GPU timing of C3's converged ICP iterations (bench.py's ICP leg, alone):
10M box-surface source / target, 30 iterations from T = I; per-kernel times
from the library's HIP-event timers.  Usage: python tools/icp_time.py [n] [iters]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda:0")
    tgt = S.box_surface(n, seed=1, device=dev)
    src = S.apply_transform(S.box_surface(n, seed=2, device=dev), S.rigid_transform())
    tn = ops.estimate_normals(tgt, knn=30)
    target = ops.ICPTarget(tgt, tn, 0.02)
    src4 = ops.spatial_sort(src)
    T = np.eye(4)
    target.accumulate(src4, T)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        sums, _ = target.accumulate(src4, T)
        T = ops.icp_solve(sums) @ T
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    N.reset_kernel_timing()
    N.set_kernel_timing(True)
    T2 = np.eye(4)
    for _ in range(iters):
        s2, _ = target.accumulate(src4, T2)
        T2 = ops.icp_solve(s2) @ T2
    torch.cuda.synchronize()
    acc, na = N.kernel_timing("icp_accumulate")
    m, nm = N.kernel_timing("icp_match")
    N.set_kernel_timing(False)
    per_iter = []  # match time of each iteration from T = I (the first ones see the displaced source)
    T3 = np.eye(4)
    N.set_kernel_timing(True)
    for _ in range(iters):
        N.reset_kernel_timing()
        s3, _ = target.accumulate(src4, T3)
        torch.cuda.synchronize()
        per_iter.append(round(N.kernel_timing("icp_match")[0], 3))
        T3 = ops.icp_solve(s3) @ T3
    N.set_kernel_timing(False)
    err = float(np.abs(T - np.linalg.inv(S.rigid_transform())).max())
    print(json.dumps({"tag": os.environ.get("TAG", ""), "iters_per_s": round(iters / el, 2),
                      "ms_per_iter": round(el / iters * 1e3, 4), "accumulate_ms": round(acc / max(na, 1), 4),
                      "match_ms": round(m / max(nm, 1), 4), "T_err": err, "T": T.round(12).tolist(),
                      "fitness": float(sums[28]) / n, "match_ms_per_iteration": per_iter}), flush=True)


if __name__ == "__main__":
    main()
