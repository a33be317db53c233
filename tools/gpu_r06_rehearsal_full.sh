#!/bin/bash
# --gpus 2 launcher on one GPU (O3DX_BENCH_SHARED_GPU=1, gloo) with the N-rank
# secondary legs (sharded ICP on the device loop, the sharded C5 chain at 40M)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O3DX_BENCH_SHARED_GPU=1 timeout -k 10 900 python bench.py --gpus 2 --steps 10 --warmup 3 --c5-n 40000000 --no-cpu \
  > gpurun_out/r06_rehearsal_full.json 2> gpurun_out/r06_rehearsal_full.log || { tail -30 gpurun_out/r06_rehearsal_full.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_rehearsal_full.json").read().strip().splitlines()[-1])
print("n_gpus", d["n_gpus"], "value", d["value"], "ms", d["ms_per_step"])
print("curve", json.dumps(d["scaling_curve"]))
e = d["extra"]
print("icp_sharded", e.get("icp_sharded"), e.get("icp_sharded_error"))
c5 = e.get("c5_sharded") or {}
print("c5_sharded", {k: c5.get(k) for k in ("ms", "ranks", "target_reps", "icp_fitness", "T_err_vs_gt_inverse", "stages_ms_rank0")}, e.get("c5_error"))
PY
