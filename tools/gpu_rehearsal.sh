#!/bin/bash
# C4 slab step rehearsal with N ranks sharing cuda:0 (gloo) and the
# rank-0 host timeline of one step (bench.py extra.host_timeline_rank0_ms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${1:-2}
export O3DX_BENCH_SHARED_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$R" --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus "$R" --steps 10 --warmup 3 --c4-n ${C4N:-50000000} --no-secondary \
  > gpurun_out/rehearsal_$R.json 2> gpurun_out/rehearsal_$R.log || { tail -20 gpurun_out/rehearsal_$R.log; exit 1; }
python - "$R" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/rehearsal_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("ms_per_step", d["ms_per_step"], "value", d["value"])
print("breakdown", d["extra"]["step_breakdown"])
print("host_timeline", d["extra"]["host_timeline_rank0_ms"])
PY
