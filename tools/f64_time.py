"""The float64 boundary's speed (GPU box only): a LAS-like scan (box surface
40 x 32 x 24 m at a ~5e5 m offset, full-mantissa float64) through the hot
path — voxel_down_sample (5 cm), KNN30 normals on the reps, segment_plane
(1000 hypotheses, 2 cm), point-to-plane ICP of a moved second scan's reps (30
iterations from T = I, in the recentred frame) — each stage timed after a
warm-up, against the same stages on the scan re-centred and rounded to
float32 (the float32 kernels).
Usage: python tools/f64_time.py [n]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
from open3dpypro import ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
VS = 0.05
T = S.rigid_transform(0.5, t=(0.02, -0.01, 0.015))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, round((time.perf_counter() - t0) * 1e3, 3)


def chain(tgt, src, tag):
    out = {"case": tag, "n": int(tgt.shape[0])}
    vt, out["voxel_ms"] = timed(lambda: ops.voxel_down_sample(tgt, VS))
    reps = vt["rep_xyz"]
    vsrc = ops.voxel_down_sample(src, VS)["rep_xyz"]
    out["reps"] = int(reps.shape[0])
    tn, out["normals_ms"] = timed(lambda: ops.estimate_normals(reps, knn=30))
    samples = ops.ransac_samples(reps.shape[0], 3, 1000, seed=7)
    (plane, inl), out["segment_plane_ms"] = timed(lambda: ops.segment_plane(reps, 0.02, 3, 1000, samples=samples))
    out["plane_inliers"] = int(inl.numel())
    # ICP in the frame users register such scans in (recentred: at a 5e5 m
    # offset point-to-plane's normal matrix is rounding noise, for Open3D too;
    # tests/test_gpu_f64.py test_f64_icp); the coordinates stay full-mantissa
    c = reps.mean(0)
    reg, out["icp_30_ms"] = timed(lambda: ops.registration_icp(vsrc - c, reps - c, tn, 0.2, max_iteration=30))
    out["icp_fitness"] = round(float(reg["fitness"]), 6)
    print(json.dumps(out), flush=True)


las = S.las_scene(n, seed=0, device=dev)
src = S.las_scene(n, seed=1, T=T, device=dev)
chain(las, src, "f64 LAS scan (float64 kernels)")
x0 = torch.tensor(S.LAS_OFFSET, dtype=torch.float64, device=dev)
chain((las - x0).float(), (src - x0).float(), "same scan re-centred in float32 (float32 kernels)")
