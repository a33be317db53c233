#!/bin/bash
# PMC passes over the ICP device loop (its skip-proof steps: MODE 2), then the
# full --gpus 2 launcher rehearsal on one GPU (tools/gpu_r06_rehearsal_full.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_icp
bash tools/pmc.sh gpurun_out/pmc_icp -- python tools/prof_kernels.py icp_loop > gpurun_out/pmc_icp.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_icp gpurun_out/pmc_icp_summary.json || exit 1
bash tools/gpu_r06_rehearsal_full.sh
