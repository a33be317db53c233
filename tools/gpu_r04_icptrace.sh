#!/bin/bash
# rocprofv3 kernel trace of the device ICP loop (prof_kernels.py icp_loop):
# per-launch durations of k_icp_step / k_icp_finish in launch order and the
# gaps between consecutive kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/icptrace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/icptrace -o run --output-format csv -- \
  python tools/prof_kernels.py icp_loop > gpurun_out/icptrace.log 2>&1 || { tail -20 gpurun_out/icptrace.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/icptrace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
sel = [r for r in rows if "k_icp_step" in r["Kernel_Name"] or "k_icp_finish" in r["Kernel_Name"]]
sel = sel[-62:]
prev_end = None
out = []
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    out.append(("step" if "step" in r["Kernel_Name"] else "finish", (e - s) / 1e3, gap))
    prev_end = e
for name, d, gap in out:
    print(f"{name:7s} {d:9.1f} us  gap {gap:6.1f} us")
steps = [d for n, d, g in out if n == "step"]
fins = [d for n, d, g in out if n == "finish"]
gaps = [g for n, d, g in out[1:]]
print("first step", steps[0], "steady step mean", sum(steps[1:]) / len(steps[1:]), "finish mean", sum(fins) / len(fins),
      "gap mean", sum(gaps) / len(gaps), "total", (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3)
PY
