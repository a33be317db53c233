#!/bin/bash
# Full PMC set (tools/pmc.sh: 4 separate counter passes) over tools/prof_kernels.py
# (normals, ICP, RANSAC) -> gpurun_out/pmc_summary.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc
bash tools/pmc.sh gpurun_out/pmc -- python tools/prof_kernels.py ${1:-all} || exit $?
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_summary.json
