#!/bin/bash
# The full -m gpu suite (optionally filtered: $1 = pytest -k expression), with
# the parity report of every normals check in gpurun_out/parity_report.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/parity_report.jsonl
export O3DX_PARITY_LOG=$PWD/gpurun_out/parity_report.jsonl
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
exit $rc
