#!/bin/bash
# GPU box: kernel trace of the RANSAC count variants (tools/ransac_time.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ransac -o run -- python3 $R/tools/ransac_time.py 5 > $R/gpurun_out/prof_ransac.log 2>&1
