#!/bin/bash
# C2 step: one-call vs two-call structure, with and without the in-region kernel events.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r02e.txt
for rep in 1 2; do
for opt in "" "--no-kernel-events" "--two-call" "--two-call --no-kernel-events"; do
  timeout -k 10 200 python bench.py --no-cpu --no-secondary --c4-n 0 --c5-n 0 --steps 20 $opt \
    > gpurun_out/r02e_one.json 2> gpurun_out/r02e_one.err || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/r02e_one.json')); e=d['extra']
print('$opt' or 'default', d['ms_per_step'], e['stream_event_ms_per_step'], e.get('two_call_ms_per_step'), e.get('one_call_ms_per_step'), e['kernels'].get('normals_stile'))" >> gpurun_out/r02e.txt
done
done
cat gpurun_out/r02e.txt
