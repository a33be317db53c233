#!/bin/bash
# PMC passes over the voxel stage of C2 (prof_kernels.py normals): per-kernel
# instruction mix, wave/busy cycles and HBM requests of the binning, reduce,
# compaction and gather kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/voxpmc
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/voxpmc/p$i -o run --output-format csv -- \
    python tools/prof_kernels.py normals > gpurun_out/voxpmc/p$i.log 2>&1 || { tail -5 gpurun_out/voxpmc/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob("gpurun_out/voxpmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if any(s in k for s in ("vbin", "gather_vox", "compact", "aabb", "tile_sums", "scan_part")):
        print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
