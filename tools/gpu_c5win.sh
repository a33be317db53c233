#!/bin/bash
# C5 sharded pipeline with the windowed ICP target: GPU distributed tests, then the 2-rank rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread \
  -k "c5 or icp" > gpurun_out/c5win_tests.log 2>&1 || { tail -30 gpurun_out/c5win_tests.log; exit 1; }
tail -2 gpurun_out/c5win_tests.log
bash tools/gpu_rehearsal.sh 2
