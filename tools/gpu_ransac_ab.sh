#!/bin/bash
# GPU box: kernel-trace A/B of the RANSAC count — the in-tree library vs an
# earlier build in tools/_cmp (tools/ransac_time.py; $1 = variant list).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
V=${1:-s32x16x0}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_new -o run -- python3 $R/tools/ransac_time.py 5 $V > $R/gpurun_out/ab_new.log 2>&1 &&
O3DX_LIB_CMP=$R/tools/_cmp/libo3dx.so TAG=_old timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_old -o run -- python3 $R/tools/ransac_time.py 5 s32x16x0 > $R/gpurun_out/ab_old.log 2>&1
