#!/bin/bash
# A/B of the headline step under env switches: for each "NAME=VAL" argument
# (or "base"), bench.py --no-cpu --no-secondary, ms_per_step into gpurun_out/ab_env.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab_env.txt
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then e=""; else e="$v"; fi
    out=$(env $e timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps ${STEPS:-50} --warmup 20 2>/dev/null) || exit $?
    ms=$(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['extra']['kernels']; print(d['ms_per_step'], {n: v['avg_ms'] for n, v in k.items()})")
    echo "$round $v $ms" | tee -a gpurun_out/ab_env.txt
  done
done
