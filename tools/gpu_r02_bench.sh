#!/bin/bash
# Round-2 bench evidence: the default bench line (N=1) and the rocprofv3
# kernel trace + stats of the same command without the CPU legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || exit $?
cat gpurun_out/r02_bench.json
rm -rf gpurun_out/prof_r02
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o run --output-format csv -- \
  python bench.py --no-cpu > gpurun_out/r02_prof_bench.log 2>&1 || exit $?
