#!/bin/bash
# Bench evidence: the default bench line (N=1) and, with PROF=1, the
# rocprofv3 kernel trace + stats of the same command without the CPU legs.
# $1: tag for the output names (default: cur)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-cur}
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit $?
cat gpurun_out/bench_$T.json
if [ "${PROF:-0}" = 1 ]; then
  rm -rf gpurun_out/prof_$T
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- \
    python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/prof_bench_$T.log 2>&1 || exit $?
fi
