#!/bin/bash
# Round 4 RANSAC iteration: cull-path tests, sweep timings (cull vs mfma2), the
# segment_plane timeline (kernel trace) at C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$1" != notest ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "ransac or segment_plane or plane_count or culled or seg_planes or mfma2" > gpurun_out/ransac_tests.log 2>&1 \
    || { tail -30 gpurun_out/ransac_tests.log; exit 1; }
  tail -2 gpurun_out/ransac_tests.log
fi
UPPER=cull,mfma2 timeout -k 10 300 python -u tools/ransac_time.py 5 s32x16x0x6 > gpurun_out/ransac_time.log 2>&1 || { tail -20 gpurun_out/ransac_time.log; exit 1; }
cat gpurun_out/ransac_time.log
bash tools/gpu_trace_ransac.sh && python3 tools/timeline.py gpurun_out/tr_ransac 40 > gpurun_out/tr_ransac_tl.txt
