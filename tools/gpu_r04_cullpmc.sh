#!/bin/bash
# PMC passes over the culled RANSAC sweep (prof_kernels.py ransac_upper):
# instruction mix and busy/wait cycles of k_plane_upper_cull and the binning.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cullpmc
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY" \
         "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/cullpmc/p$i -o run --output-format csv -- \
    python tools/prof_kernels.py ransac_upper > gpurun_out/cullpmc/p$i.log 2>&1 || { tail -5 gpurun_out/cullpmc/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/cullpmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "cull" in k or "cbin" in k:
        print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
