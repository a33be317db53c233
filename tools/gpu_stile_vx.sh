#!/bin/bash
# stile xy loads as ds_read_b64 (O3DX_STILE_VX=1) vs ds_read2_b64: parity tests, then the step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "dense_voxel_table or on_voxel_grid or fused or 10m_voxel_table" > gpurun_out/stile_tests.log 2>&1 || { tail -30 gpurun_out/stile_tests.log; exit 1; }
tail -2 gpurun_out/stile_tests.log
bash tools/gpu_ab_env.sh base O3DX_STILE_VX=0
