#!/bin/bash
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcdbg
for d in 1 2 3 4 0; do
  O3DX_TILE_DEBUG=$d timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmcdbg/d$d -o run --output-format csv -- python tools/prof_kernels.py normals > $R/gpurun_out/pmcdbg/d$d.log 2>&1
done
echo DONE
