#!/bin/bash
# Round-2 evidence: ICP/voxel GPU tests, bench line, rocprofv3 stats of the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "icp or voxel" > gpurun_out/ri_tests.log 2>&1 &&
bash tools/gpu_r02_bench.sh
