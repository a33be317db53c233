#!/bin/bash
# PMC passes over the normals (C2), the voxel passes and RANSAC (C3): one
# counter group per rocprofv3 run (tools/pmc.sh), summarised into
# profiles/pmc_traffic.json (merged) and gpurun_out/pmc_all.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for what in normals ransac; do
  rm -rf gpurun_out/pmc_$what
  bash tools/pmc.sh gpurun_out/pmc_$what -- python tools/prof_kernels.py $what > gpurun_out/pmc_$what.log 2>&1 || exit 1
  python tools/pmc_summary.py gpurun_out/pmc_$what gpurun_out/pmc_$what.json > /dev/null || exit 1
done
python - <<'PY'
import json
out = json.load(open("profiles/pmc_traffic.json"))
for w in ("normals", "ransac"):
    out["kernels"].update(json.load(open(f"gpurun_out/pmc_{w}.json"))["kernels"])
json.dump(out, open("gpurun_out/pmc_all.json", "w"), indent=1, sort_keys=True)
for k in ("plane_count", "vbin_count", "vbin_scatter", "vbin_reduce", "gather_vox", "normals_stile"):
    e = out["kernels"].get(k, {})
    print(k, {c: round(e[c]) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "hbm_bytes_per_launch") if c in e})
PY
