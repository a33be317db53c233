#!/bin/bash
# ICP target-grid sweep: bench's ICP leg under each setting of $1 (VAR=v1,v2,..).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
key=${1%%=*}; vals=${1#*=}
: > gpurun_out/icp_sweep.txt
for v in ${vals//,/ }; do
  env "$key=$v" timeout -k 10 120 python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/sweep_one.json 2> gpurun_out/sweep_one.err || exit $?
  python -c "
import json,sys; d=json.load(open('gpurun_out/sweep_one.json'))['extra']['icp']
print('$key=$v', d['iters_per_s'], d['match_kernel_ms'], d['accumulate_kernel_ms'], d['target_build_s'], d['fitness'], d['T_err_vs_gt_inverse'])" >> gpurun_out/icp_sweep.txt
done
cat gpurun_out/icp_sweep.txt
