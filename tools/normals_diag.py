"""GPU diagnostic: where do the HIP normals differ from the oracle, and why?

For each case: normals error vs the oracle, the production kernels' selected
neighbour sets (o3dx_set_debug_neighbors) vs the oracle's kNN sets, and for
the rows whose sets agree but normals differ, the device FastEigen3x3 vs the
oracle's on the same covariance.  Also the device acos/cos vs the host libm.
Usage (GPU box): python tools/normals_diag.py [out.json]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
sys.path.insert(0, ROOT)
from open3dpypro import _native as N, ops, pcd_io, synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

dev = torch.device("cuda:0")
L = N.load()


def dev_fast_eigen(cov):
    c = torch.from_numpy(np.ascontiguousarray(cov, np.float64)).to(dev)
    o = torch.empty((len(cov), 3), dtype=torch.float64, device=dev)
    N.check(L.o3dx_fast_eigen3x3(N.ptr(c), len(cov), N.ptr(o), N.stream_ptr(dev)), "fast_eigen")
    return o.cpu().numpy()


def dev_libm(x, fn):
    t = torch.from_numpy(np.ascontiguousarray(x, np.float64)).to(dev)
    o = torch.empty_like(t)
    N.check(L.o3dx_libm_probe(N.ptr(t), len(x), fn, N.ptr(o), N.stream_ptr(dev)), "libm")
    return o.cpu().numpy()


def cov_seq(pts64, idx):
    """Open3D ComputeCovariance in the given index order (sequential f64)."""
    m = np.zeros((len(idx), 9))
    for j in range(idx.shape[1]):
        p = pts64[idx[:, j]]
        x, y, z = p[:, 0], p[:, 1], p[:, 2]
        m += np.stack([x, y, z, x * x, x * y, x * z, y * y, y * z, z * z], 1)
    u = m / idx.shape[1]
    return np.stack([u[:, 3] - u[:, 0] ** 2, u[:, 4] - u[:, 0] * u[:, 1], u[:, 5] - u[:, 0] * u[:, 2],
                     u[:, 6] - u[:, 1] ** 2, u[:, 7] - u[:, 1] * u[:, 2], u[:, 8] - u[:, 2] ** 2], 1)


def case(name, reps, voxel_grid=None, k=30):
    t0 = time.time()
    M = reps.shape[0]
    nbr = torch.full((M, k), -1, dtype=torch.int32, device=dev)
    N.check(L.o3dx_set_debug_neighbors(N.ptr(nbr), M, k), "dbg")
    got = ops.estimate_normals(reps, knn=k, voxel_grid=voxel_grid).cpu().numpy().astype(np.float64)
    N.check(L.o3dx_set_debug_neighbors(None, 0, 0), "dbg")
    gn = np.sort(nbr.cpu().numpy(), 1)
    r = reps.cpu().numpy()
    ref = O.estimate_normals(r, O.KNN, k)
    idx, d2, _ = O.knn_search(r, r, O.KNN, k)
    on = np.sort(idx, 1)
    set_bad = np.any(gn != on, 1)
    es = np.abs(got - ref).max(1)
    ea = np.minimum(es, np.abs(got + ref).max(1))
    bad = es > 1e-5
    out = {"case": name, "M": int(M), "set_mismatch_rows": int(set_bad.sum()),
           "unset_rows": int(np.any(gn < 0, 1).sum()),
           "err_signed_gt_1e-5": int(bad.sum()), "err_any_gt_1e-5": int((ea > 1e-5).sum()),
           "max_err_signed": float(es.max()), "max_err_any": float(ea.max()),
           "bad_with_set_mismatch": int((bad & set_bad).sum())}
    rows = np.nonzero(set_bad)[0][:20]
    ex = []
    for i in rows:
        g, o_ = set(gn[i].tolist()), set(on[i].tolist())
        ex.append({"row": int(i), "gpu_only": sorted(g - o_)[:5], "oracle_only": sorted(o_ - g)[:5],
                   "kth_d2": float(d2[i, k - 1]), "kp1": None})
    out["set_examples"] = ex
    # arithmetic-only mismatches: same set, different normal
    ar = np.nonzero(bad & ~set_bad)[0]
    out["bad_same_set"] = int(len(ar))
    if len(ar):
        pts64 = r.astype(np.float64)
        c = cov_seq(pts64, idx[ar])           # the oracle's order
        e_host = O.fast_eigen3x3(c)
        e_dev = dev_fast_eigen(c)
        out["host_eigen_reproduces_ref"] = int(np.all(np.abs(e_host - ref[ar]) == 0, 1).sum())
        out["dev_eigen_eq_host_eigen"] = int(np.all(e_dev == e_host, 1).sum())
        out["dev_eigen_close_gpu_normal"] = int((np.abs(e_dev - got[ar]).max(1) < 1e-6).sum())
        # order sensitivity: the covariance in the GPU's summation order
        gi = nbr.cpu().numpy()[ar]
        c2 = cov_seq(pts64, gi)
        out["cov_order_differs"] = int(np.any(c2 != c, 1).sum())
        out["bad_examples"] = [{"row": int(i), "err": float(es[i]), "got": got[i].tolist(), "ref": ref[i].tolist()}
                               for i in ar[:5]]
    out["secs"] = round(time.time() - t0, 2)
    print(json.dumps(out), flush=True)
    return out


def libm_check():
    rng = np.random.default_rng(0)
    res = {}
    x = np.concatenate([rng.uniform(-1, 1, 2_000_000), rng.uniform(0.999, 1.0, 200_000),
                        rng.uniform(-1.0, -0.999, 200_000)])
    a = dev_libm(x, 0)
    h = np.arccos(x)
    res["acos_diff"] = int((a != h).sum())
    res["acos_maxulp"] = int(np.max(np.abs(a.view(np.int64) - h.view(np.int64))))
    y = rng.uniform(0, np.pi, 2_000_000)
    a = dev_libm(y, 1)
    h = np.cos(y)
    res["cos_diff"] = int((a != h).sum())
    res["cos_maxulp"] = int(np.max(np.abs(a.view(np.int64) - h.view(np.int64))))
    z = rng.uniform(0, 10, 1_000_000)
    res["sqrt_diff"] = int((dev_libm(z, 2) != np.sqrt(z)).sum())
    # random covariances: device vs host FastEigen
    A = rng.normal(size=(500_000, 3, 3))
    C = A @ A.transpose(0, 2, 1)
    c6 = np.stack([C[:, 0, 0], C[:, 0, 1], C[:, 0, 2], C[:, 1, 1], C[:, 1, 2], C[:, 2, 2]], 1)
    res["eigen_random_diff"] = int(np.any(dev_fast_eigen(c6) != O.fast_eigen3x3(c6), 1).sum())
    print(json.dumps({"libm": res}), flush=True)
    return res


def main():
    outp = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "normals_diag.json")
    os.makedirs(os.path.dirname(outp), exist_ok=True)
    res = {"libm": libm_check(), "cases": []}
    f = pcd_io.read_pcd_arrays(os.path.join(ROOT, "tests", "golden", "bunny.pcd"))
    bunny = torch.from_numpy(np.stack([f["x"], f["y"], f["z"]], 1).astype(np.float32)).to(dev)
    o = ops.voxel_down_sample(bunny, 0.005, keep_grid=True)
    res["cases"].append(case("bunny_reps_sortedgrid", o["rep_xyz"]))
    res["cases"].append(case("bunny_raw_sortedgrid", bunny))
    n = 10_000_000
    cl = S.uniform_cube(n, seed=0, device=dev)
    o = ops.voxel_down_sample(cl, S.voxel_size_for(n), keep_grid=True)
    res["cases"].append(case("c2_voxel_table", o["rep_xyz"], o["voxel_grid"]))
    res["cases"].append(case("c2_sorted_grid", o["rep_xyz"]))
    del cl, o
    torch.cuda.empty_cache()
    cl = S.uniform_cube(1_000_000, seed=5, device=dev)
    res["cases"].append(case("cube1m_raw_sortedgrid", cl))
    surf = S.box_surface(1_000_000, 1, device=dev)
    res["cases"].append(case("surface1m_sortedgrid", surf))
    json.dump(res, open(outp, "w"), indent=1)


if __name__ == "__main__":
    main()
