#!/bin/bash
# GPU box: per-kernel trace of the sparse-grid voxel timing tool
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_vsparse
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_vsparse -o run --output-format csv -- python3 $R/tools/voxel_sparse_time.py > $R/gpurun_out/prof_vsparse.log 2>&1
