#!/bin/bash
# Round-2 PMC evidence: counter passes (tools/pmc.sh, one group per run) over
# the normals, the RANSAC count and the converged ICP accumulate; summaries
# merged into profiles/pmc_traffic.json (bench.py reads its traffic figure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in normals ransac_count icp; do
  rm -rf gpurun_out/pmc_$m
  bash tools/pmc.sh gpurun_out/pmc_$m -- python tools/prof_kernels.py $m > gpurun_out/pmc_$m.log 2>&1 || exit $?
  python tools/pmc_summary.py gpurun_out/pmc_$m gpurun_out/pmc_summary_$m.json || exit $?
done
python - <<'PY' || exit $?
import json
old = json.load(open("profiles/pmc_traffic.json"))
for m in ("normals", "ransac_count", "icp"):
    new = json.load(open(f"gpurun_out/pmc_summary_{m}.json"))
    old["kernels"].update(new["kernels"])
old["source_round"] = "r02"
for p in ("profiles/pmc_traffic.json", "gpurun_out/pmc_traffic.json"):
    with open(p, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)
print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in old["kernels"].items()}))
PY
