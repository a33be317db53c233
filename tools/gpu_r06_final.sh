#!/bin/bash
# Round-end evidence in one call: the -m gpu suite + smoke, then the PMC
# passes, the bench line and the C2-only rocprofv3 kernel stats
# (tools/gpu_final.sh tests / bench without the full-bench rocprof pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu_final.sh tests || exit 1
NO_FULL_PROF=1 bash tools/gpu_final.sh bench || exit 1
