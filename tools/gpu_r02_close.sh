#!/bin/bash
# Round-2 closing evidence: full -m gpu suite, smoke(), bench line + rocprofv3 stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
bash tools/gpu_r02_bench.sh
