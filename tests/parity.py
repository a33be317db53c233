"""Shared parity checks of the GPU normals against the oracle (tests only).

The bar (BASELINE.json north_star): every normal within 1e-5 of the oracle's,
signed, on every row — no fraction of rows is exempt.  The one allowance is
a row whose oracle normal itself moves beyond the tolerance when Open3D's
transcendental results (acos / cos inside FastEigen3x3) change by one ulp —
the latitude between two correct libms (glibc's acos is not correctly
rounded; the GPU's differs from it by one ulp on ~9 % of inputs, measured in
tools/normals_diag.py).  Such a row is "certified" only when the GPU normal
equals (to float32 rounding) the oracle's normal under one of the 26 one-ulp
nudges, computed from the oracle's own neighbour set in the oracle's order;
every certified row is counted in the report.  Neighbour sets of the
production kernels (o3dx_set_debug_neighbors) are compared bit-exactly.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from oracle import oracle as O

TOL = 1e-5


def _report(what, info):
    path = os.environ.get("O3DX_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"check": what, **info}) + "\n")


def assert_normals(got, ref, xyz=None, mode=O.KNN, k=30, radius=0.0, prior=None, what=""):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    e = np.abs(got - ref).max(1) if len(got) else np.zeros(0)
    bad = np.nonzero(e > TOL)[0]
    info = {"rows": int(len(got)), "max_err": float(e.max()) if len(e) else 0.0, "beyond_tol": int(len(bad)),
            "certified": 0}
    if len(bad):
        assert xyz is not None, (what, info)
        x = np.asarray(xyz).reshape(-1, 3)  # float32 clouds, or float64 ones kept as such
        if mode == O.RADIUS:  # every neighbour within the radius, sorted (capped rows would not certify)
            idx, _, cnt = O.knn_search(x, x[bad], mode, k, radius, K=1024)
            assert (cnt < 1024).all(), (what, "radius neighbourhoods beyond the certificate's cap")
        else:
            idx, _, cnt = O.knn_search(x, x[bad], mode, k, radius)
        cov = O.covariance(x, idx, cnt)
        ok = np.zeros(len(bad), bool)
        for nudge in range(1, 27):
            v = O.fast_eigen3x3_nudged(cov, nudge)
            zero = ~np.any(v != 0, 1)
            v[zero] = [0.0, 0.0, 1.0]
            if prior is not None:
                pr = np.asarray(prior, np.float64)[bad]
                v[zero] = pr[zero]
                v[np.sum(v * pr, 1) < 0] *= -1
            ok |= np.abs(v - got[bad]).max(1) < 1e-6
        info["certified"] = int(ok.sum())
        assert ok.all(), (what, info, bad[~ok][:10].tolist(), e[bad[~ok]][:10].tolist())
    _report(what, info)
    return info


def assert_neighbour_sets(nbr, xyz, k, what=""):
    """Sorted neighbour ids of every row == the oracle's kNN set (bit-exact)."""
    g = np.sort(np.asarray(nbr), 1)
    x = np.asarray(xyz).reshape(-1, 3)
    idx, _, _ = O.knn_search(x, x, O.KNN, k)
    o = np.sort(idx, 1)
    diff = np.any(g != o, 1)
    info = {"rows": int(len(g)), "set_mismatch": int(diff.sum())}
    _report(what + ":sets", info)
    assert not diff.any(), (what, info, np.nonzero(diff)[0][:10].tolist())
    return info


class DebugNeighbors:
    """Context manager: the production normals kernels record their selected
    neighbour ids (include/o3dx.h o3dx_set_debug_neighbors)."""

    def __init__(self, rows, k, device):
        from open3dpypro import _native as N
        self.N = N
        self.buf = torch.full((max(rows, 1), k), -1, dtype=torch.int32, device=device)
        self.rows, self.k = rows, k

    def __enter__(self):
        self.N.check(self.N.load().o3dx_set_debug_neighbors(self.N.ptr(self.buf), self.rows, self.k), "dbg")
        return self

    def __exit__(self, *a):
        torch.cuda.synchronize()
        self.N.check(self.N.load().o3dx_set_debug_neighbors(None, 0, 0), "dbg")

    def ids(self):
        return self.buf[: self.rows].cpu().numpy()
