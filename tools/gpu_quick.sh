#!/bin/bash
# Quick GPU iteration: the GPU tests matching $1 (pytest -k), then the bench.
# Usage (via gpurun): bash tools/gpu_quick.sh "icp" [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
K="$1"; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err
