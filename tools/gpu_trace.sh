#!/bin/bash
# Kernel trace of the headline bench (no secondary legs) + one step's timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python bench.py --no-cpu --no-secondary "$@" > gpurun_out/trace_bench.log 2>&1 || exit $?
python tools/step_timeline.py gpurun_out/trace > gpurun_out/trace_step.txt
cat gpurun_out/trace_step.txt
