#!/bin/bash
# RANSAC upper bounds on the matrix cores: parity tests, then timing vs the VALU sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "ransac or segment_plane or plane_count or seg_planes or plane_detection or c5" > gpurun_out/ransac_tests.log 2>&1 || { tail -30 gpurun_out/ransac_tests.log; exit 1; }
tail -2 gpurun_out/ransac_tests.log
timeout -k 10 300 python tools/ransac_time.py 5 s32x16x0x6 > gpurun_out/ransac_time.log 2>&1 || { tail -20 gpurun_out/ransac_time.log; exit 1; }
cat gpurun_out/ransac_time.log
