#!/bin/bash
# the float64 lane form (O3DX_F64_NO_TILES=1) and the tiles, with the tiles' hand-off statistics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O3DX_F64_NO_TILES=1 timeout -k 10 200 python tools/f64_normals_ab.py 2>/dev/null | tee -a gpurun_out/r06_f64_lane.txt || exit 1
timeout -k 10 200 python tools/f64_normals_ab.py 2>/dev/null | tee -a gpurun_out/r06_f64_lane.txt || exit 1
timeout -k 10 200 python - <<'PY' 2>/dev/null | tee -a gpurun_out/r06_f64_lane.txt
import os, sys, json, torch
sys.path.insert(0, "open3d-py-extension_amd")
from open3dpypro import _native as N, ops, synthetic as S
dev = torch.device("cuda:0")
las = S.las_scene(10_000_000, seed=0, device=dev)
reps = ops.voxel_down_sample(las, 0.05)["rep_xyz"].clone()
ops.estimate_normals(reps, knn=30)
N.search_stats(True)
ops.estimate_normals(reps, knn=30)
print(json.dumps({"f64_tile_stats": N.search_stats()}))
PY
