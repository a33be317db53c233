#!/bin/bash
# Round-2 closing evidence: smoke(), bench line + rocprofv3 stats, then the full -m gpu suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
bash tools/gpu_r02_bench.sh || exit $?
bash tools/gpu_tests.sh
