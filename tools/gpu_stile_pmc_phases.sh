#!/bin/bash
# Per-phase instruction budget of k_normals_stile: SQ counters of the C2
# normals (tools/prof_kernels.py normals) with the kernel stopped after each
# phase (O3DX_TILE_DEBUG 1 staging, 2 +count, 3 +list, 4 +finish without the
# eigen solve, 0 full), two counter groups per level, each its own rocprofv3
# --pmc pass.  Output: gpurun_out/stile_pmc/summary.json (per-wave counts).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/stile_pmc
rm -rf $OUT; mkdir -p $OUT
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"
G2="SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES"
for dbg in 1 2 3 4 0; do
  if [ $dbg = 0 ]; then unset O3DX_TILE_DEBUG; else export O3DX_TILE_DEBUG=$dbg; fi
  for g in 1 2; do
    if [ $g = 1 ]; then C="$G1"; else C="$G2"; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $OUT/d$dbg/p$g -o run --output-format csv -- \
      python tools/prof_kernels.py normals > $OUT/d$dbg.p$g.log 2>&1 || { tail -5 $OUT/d$dbg.p$g.log; exit 1; }
  done
  python tools/pmc_summary.py $OUT/d$dbg $OUT/d$dbg.json > /dev/null || exit 1
done
python - <<'PY'
import json
rows = {}
for d in (1, 2, 3, 4, 0):
    e = json.load(open(f"gpurun_out/stile_pmc/d{d}.json"))["kernels"]["normals_stile"]
    w = e["SQ_WAVES"]
    rows[d] = {k: e[k] / w for k in e if k.startswith("SQ_") and k != "SQ_WAVES"}
json.dump(rows, open("gpurun_out/stile_pmc/summary.json", "w"), indent=1)
keys = sorted(rows[0])
print("per wave  " + " ".join(f"{k[3:]:>16}" for k in keys))
for d in (1, 2, 3, 4, 0):
    print(f"dbg {d}    " + " ".join(f"{rows[d][k]:16.0f}" for k in keys))
PY
