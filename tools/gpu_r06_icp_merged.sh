#!/bin/bash
# ICP device loop A/B: two launches per iteration (the state picks one) vs
# one merged launch (O3DX_ICP_MERGED=1); parity of the merged loop first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O3DX_ICP_MERGED=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "icp or skip" > gpurun_out/r06_merged_tests.log 2>&1 || { tail -30 gpurun_out/r06_merged_tests.log; exit 1; }
tail -2 gpurun_out/r06_merged_tests.log
for m in 0 1 0 1; do
  O3DX_ICP_MERGED=$m timeout -k 10 200 python tools/icp_loop_ab.py 10000000 30 5 2>/dev/null | sed "s/^/merged=$m /" | cut -c1-140 | tee -a gpurun_out/r06_icp_merged.txt || exit 1
done
