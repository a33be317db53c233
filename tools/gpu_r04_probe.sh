#!/bin/bash
# Round-4 first probe: the default bench line without the CPU legs, then the
# cumulative stile phase costs (O3DX_TILE_DEBUG 1..4, 0 = full kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/r04_probe_bench.json 2> gpurun_out/r04_probe_bench.err || exit $?
cat gpurun_out/r04_probe_bench.json | head -c 600; echo
bash tools/gpu_stile_phases.sh 3
