"""GPU timing of the RANSAC count kernels at C3 (10M points x 1000 hypotheses).

The exact count is timed with the library's own HIP-event timer
"plane_count" over a few calls; each upper-bound form of segment_plane's
sweep (O3DX_RANSAC_UPPER, read per call by ransac.hip) is timed and checked
to bound the exact counts.
Usage (GPU box): python tools/ransac_time.py [reps]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import _native as N, ops, synthetic as S  # noqa: E402

VARIANTS = [("count", {})]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    variants = VARIANTS if len(sys.argv) < 3 else [v for v in VARIANTS if v[0] in sys.argv[2].split(",")]
    dev = torch.device("cuda:0")
    n, H = 10_000_000, 1000
    x = S.planted_plane(n, 0, device=dev)
    pts = x.cpu().numpy().astype(np.float64)
    idx = np.random.default_rng(0).integers(0, n, (H, 3))
    a, b, c = pts[idx[:, 0]], pts[idx[:, 1]], pts[idx[:, 2]]
    nrm = np.cross(b - a, c - a)
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-300)
    planes = np.concatenate([nrm, -np.sum(nrm * a, 1, keepdims=True)], 1)
    ref = None
    out = {}
    for name, env in variants:
        os.environ.update(env)
        got = ops.plane_count(x, planes, 0.01)  # warm-up
        N.set_kernel_timing(True)
        N.reset_kernel_timing()
        for _ in range(reps):
            got = ops.plane_count(x, planes, 0.01)
        torch.cuda.synchronize()
        ms, cnt = N.kernel_timing("plane_count")
        N.set_kernel_timing(False)
        if ref is None:
            ref = got
        out[name] = {"ms": ms / max(cnt, 1), "equal": bool(np.array_equal(got, ref)),
                     "pairs_per_s": n * H / (ms / max(cnt, 1) * 1e-3)}
        print(json.dumps({name: out[name]}), flush=True)
    # the upper-bound count (segment_plane's sweep) and the whole segment_plane
    for name in (os.environ.get("UPPER", "cull,mfma2,valu")).split(","):
        os.environ["O3DX_RANSAC_UPPER"] = name
        ub = ops.plane_count_upper(x, planes, 0.01)
        N.set_kernel_timing(True)
        N.reset_kernel_timing()
        for _ in range(reps):
            ub = ops.plane_count_upper(x, planes, 0.01)
        torch.cuda.synchronize()
        ms, cnt = N.kernel_timing("plane_count_upper")
        N.set_kernel_timing(False)
        ok = bool(np.all(ub >= ref)) and bool(np.all((ub < 0) == (ref < 0)))
        out["upper_" + name] = {"ms": ms / max(cnt, 1), "upper_bound_ok": ok, "max_slack": int((ub - ref).max()),
                                "sum_slack": int((ub - ref).sum())}
        print(json.dumps({"upper_" + name: out["upper_" + name]}), flush=True)
    os.environ.pop("O3DX_RANSAC_UPPER", None)
    samples = ops.ransac_samples(n, 3, H, 0)
    ops.segment_plane(x, 0.01, 3, H, samples=samples)
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for _ in range(reps):
        plane, inl = ops.segment_plane(x, 0.01, 3, H, samples=samples)
    torch.cuda.synchronize()
    out["segment_plane_ms"] = (time.perf_counter() - t0) / reps * 1e3
    print(json.dumps({"segment_plane_ms": out["segment_plane_ms"], "inliers": int(inl.numel())}), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "ransac_time%s.json" % os.environ.get("TAG", "")), "w"),
              indent=1)


if __name__ == "__main__":
    main()
