"""Diagnostics for the normals on the voxel table: hand-off counts and kernel
times per setting.  GPU box only.  Usage: python tools/stile_probe.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))


def run_one():
    import torch
    from open3dpypro import _native, ops, synthetic as S

    dev = torch.device("cuda:0")
    N = int(os.environ.get("N", "10000000"))
    pts = S.uniform_cube(N, 0, device=dev)
    vd = ops.voxel_down_sample(pts, S.voxel_size_for(N), keep_grid=True)
    reps, vg = vd["rep_xyz"], vd["voxel_grid"]
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith("O3DX_") and k != "O3DX_PROBE_CHILD"}}
    ops.estimate_normals(reps, knn=30, voxel_grid=vg)
    _native.search_stats(True)
    ops.estimate_normals(reps, knn=30, voxel_grid=vg)
    out["stats"] = _native.search_stats()
    _native.search_stats(False)
    _native.set_kernel_timing(True)
    _native.reset_kernel_timing()
    for _ in range(5):
        ops.estimate_normals(reps, knn=30, voxel_grid=vg)
    for name in ("normals_knn", "normals_stile", "normals_tile", "normals_wave", "grid_voxel"):
        ms, c = _native.kernel_timing(name)
        if c:
            out[name + "_ms"] = round(ms / c, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if os.environ.get("O3DX_PROBE_CHILD"):
        run_one()
        sys.exit(0)
    sets = [{}, {"O3DX_NO_STILE": "1"}]
    for extra in sets:
        env = dict(os.environ, O3DX_PROBE_CHILD="1", **extra)
        subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, check=True, timeout=300)
