"""ICP 1-NN work at T = I (C3's displaced source) and converged: search
counters (cells / candidates per query) and k_icp_match times over target
grid settings.  Usage (GPU box): python tools/icp_first_stats.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))

SETTINGS = [{}, {"O3DX_ICP_OCC": "4"}, {"O3DX_ICP_OCC": "1"}, {"O3DX_ICP_MINH_DIV": "8"},
            {"O3DX_ICP_MINH_DIV": "32"}, {"O3DX_ICP_CAP": "24"}]


def run_one():
    import numpy as np
    import torch
    from open3dpypro import _native, ops, synthetic as S
    dev = torch.device("cuda:0")
    N = 10_000_000
    tgt = S.box_surface(N, 1, device=dev)
    src = S.apply_transform(S.box_surface(N, 2, device=dev), S.rigid_transform())
    tn = ops.estimate_normals(tgt, knn=30)
    target = ops.ICPTarget(tgt, tn, 0.02)
    src4 = ops.spatial_sort(src)
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith("O3DX_")}}
    for name, T in (("first", np.eye(4)), ("converged", np.linalg.inv(S.rigid_transform()))):
        target.accumulate(src4, T)
        _native.search_stats(True)
        sums, _ = target.accumulate(src4, T)
        out[name + "_stats"] = _native.search_stats()
        _native.search_stats(False)
        _native.set_kernel_timing(True)
        _native.reset_kernel_timing()
        for _ in range(3):
            sums, _ = target.accumulate(src4, T)
        ms, c = _native.kernel_timing("icp_match")
        _native.set_kernel_timing(False)
        out[name + "_match_ms"] = ms / max(c, 1)
        out[name + "_fitness"] = float(sums[28]) / N
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        run_one()
    else:
        for s in SETTINGS:
            env = dict(os.environ, **s)
            subprocess.run([sys.executable, __file__, "one"], env=env, check=True, timeout=300)
