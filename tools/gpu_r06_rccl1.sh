#!/bin/bash
# RCCL on hardware with one rank: torchrun, backend nccl, the bench's
# sharded ICP leg (--dist-icp: o3dx_icp_shard_* with the digit all-reduce in
# place on the device) beside the single-GPU legs (C4 / C5 / CPU skipped).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --dist-icp --no-cpu --c4-n 0 --c5-n 0 --steps 10 --warmup 5 \
  > gpurun_out/r06_rccl1.json 2> gpurun_out/r06_rccl1.log || { tail -30 gpurun_out/r06_rccl1.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_rccl1.json").read().strip().splitlines()[-1])
e = d["extra"]
print("value", d["value"], "icp", e.get("icp", {}).get("iters_per_s"))
print("icp_sharded", json.dumps(e.get("icp_sharded")), e.get("icp_sharded_error"))
PY
