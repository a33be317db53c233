#!/bin/bash
# One rocprofv3 PMC pass over the normals driver: tools/pmc_one.sh OUTDIR COUNTERS...
set -e
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT" -o run --output-format csv -- python tools/prof_kernels.py normals > "$OUT.log" 2>&1
echo PMC_DONE
