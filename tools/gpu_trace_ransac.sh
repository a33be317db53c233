#!/bin/bash
# GPU box: kernel + copy timeline of segment_plane at C3 (tools/prof_kernels.py ransac)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/tr_ransac -o run -- python3 $R/tools/prof_kernels.py ransac > $R/gpurun_out/tr_ransac.log 2>&1
