#!/bin/bash
# GPU box: sparse-grid voxel paths — parity tests, then the 200M timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "voxel" > gpurun_out/vs_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/voxel_sparse_time.py > gpurun_out/voxel_sparse_time.log 2>&1
