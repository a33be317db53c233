#!/bin/bash
# GPU box: kernel trace + two SQ counter passes over one prof_kernels.py mode.
# Usage: bash tools/gpu_pmc_mode.sh MODE
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
M=$1
O=$R/gpurun_out/pmc_$M
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/prof_kernels.py $M > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/p1 -o run --output-format csv -- python3 $R/tools/prof_kernels.py $M > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python3 $R/tools/prof_kernels.py $M > $O/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/p3 -o run --output-format csv -- python3 $R/tools/prof_kernels.py $M > $O/p3.log 2>&1
