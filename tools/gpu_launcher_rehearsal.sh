#!/bin/bash
# The --gpus N launcher on a one-GPU box: every rank on cuda:0 (gloo),
# O3DX_BENCH_SHARED_GPU=1; the line must carry n_gpus N and an N-entry curve.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${1:-2}
O3DX_BENCH_SHARED_GPU=1 timeout -k 10 600 python bench.py --gpus "$R" --steps ${STEPS:-10} --warmup 3 \
  --no-secondary ${EXTRA:-} > gpurun_out/launcher_$R.json 2> gpurun_out/launcher_$R.log \
  || { tail -30 gpurun_out/launcher_$R.log; exit 1; }
python - "$R" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/launcher_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("n_gpus", d["n_gpus"], "value", d["value"], "ms_per_step", d["ms_per_step"])
print("curve", json.dumps(d["scaling_curve"]))
print("launcher", d["launcher"])
print("host_timeline", d["extra"].get("host_timeline_rank0_ms"))
print("breakdown", d["extra"].get("step_breakdown"))
PY
