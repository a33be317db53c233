#!/bin/bash
# round-end GPU suite + smoke (tools/gpu_final.sh tests), then the float64 batching A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_final.sh tests || exit 1
bash tools/gpu_r06_f64_b.sh
