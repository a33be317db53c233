#!/bin/bash
# Development loop on the GPU box: a -k filtered slice of the -m gpu suite,
# then the headline bench line without the CPU and secondary legs.
# $1: pytest -k expression ("" = skip tests), $2: tag
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$1" ]; then bash tools/gpu_tests.sh "$1" || exit $?; fi
BENCH_ARGS="--no-cpu --no-secondary ${BENCH_EXTRA:-}" bash tools/gpu_bench.sh "${2:-iter}"
