#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only; never
# combined with sys/runtime tracing).  Usage: tools/pmc.sh OUTDIR -- cmd...
# PMC_SET=traffic runs only the FETCH_SIZE / WRITE_SIZE passes.
set -e
export TMPDIR=/tmp
OUT=$1; shift; shift
mkdir -p "$OUT"
if [ "${PMC_SET:-all}" = "traffic" ]; then
  groups=("FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE")
else
  groups=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
          "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
          "FETCH_SIZE GRBM_GUI_ACTIVE"
          "WRITE_SIZE")
fi
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1
done
echo PMC_DONE
