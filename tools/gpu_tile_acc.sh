#!/bin/bash
# tile kernel moments: anchored Fast2Sum (default) vs TwoSum (O3DX_TILE_DD=1) — bit-identity tests, then timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "normals or knn or c4 or c5 or sorted_grid or full_mantissa or statistical" > gpurun_out/tile_acc_tests.log 2>&1 || { tail -30 gpurun_out/tile_acc_tests.log; exit 1; }
tail -2 gpurun_out/tile_acc_tests.log
timeout -k 10 300 python tools/surface_normals_time.py "" O3DX_TILE_DD=1 > gpurun_out/tile_acc_time.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/raw_normals_time.py >> gpurun_out/tile_acc_time.jsonl 2>&1 || exit 1
O3DX_TILE_DD=1 timeout -k 10 200 python tools/raw_normals_time.py >> gpurun_out/tile_acc_time.jsonl 2>&1 || exit 1
cut -c1-200 gpurun_out/tile_acc_time.jsonl
bash tools/gpu_trace.sh > /dev/null && cat gpurun_out/trace_step.txt
