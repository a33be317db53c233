#!/bin/bash
# GPU box: RANSAC + ICP kernel tests, RANSAC count timing, ICP first-iteration trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_api.py -k "icp or registration" > gpurun_out/ri_tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_icpfirst -o run --output-format csv -- python3 $R/tools/prof_kernels.py icp_first > $R/gpurun_out/prof_icpfirst.log 2>&1 &&
cd $R && bash tools/gpu_r02_bench.sh
