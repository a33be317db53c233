#!/bin/bash
# Nested-grid normals on raw mixed-density clouds: parity tests, then the
# raw C3 timing under a few settings (O3DX_NESTED_* env).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread \
  -k "nested or raw_planted or paths_agree" > gpurun_out/nested_tests.log 2>&1 || { tail -40 gpurun_out/nested_tests.log; exit 1; }
tail -3 gpurun_out/nested_tests.log
: > gpurun_out/nested_time.jsonl
for cfg in "" "O3DX_WAVE_DEFER=0"; do
  env $cfg timeout -k 10 120 python tools/raw_normals_time.py >> gpurun_out/nested_time.jsonl 2>> gpurun_out/nested_time.err || exit 1
done
cat gpurun_out/nested_time.jsonl
