"""One bench step's kernels in launch order, with the idle gap before each
(rocprofv3 kernel trace).  Usage: python tools/step_timeline.py PROF_DIR [marker] [k]
prints the kernels between the k-th and (k+1)-th launches whose name holds marker."""
import csv
import os
import sys


def main(src, marker="k_normals_stile", k=5):
    rows = list(csv.DictReader(open(os.path.join(src, "run_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[k], idx[k + 1]
    prev = int(rows[a]["End_Timestamp"])
    busy = gaps = 0.0
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gaps += max(s - prev, 0) / 1e3
        busy += (e - s) / 1e3
        grid = r.get("Grid_Size_X") or r.get("Grid_Size")
        print(f"gap {(s - prev) / 1e3:7.1f}  run {(e - s) / 1e3:7.1f} us  {r['Kernel_Name'][:80]}  grid={grid}")
        prev = e
    print(f"busy {busy:.1f} us, idle {gaps:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *(int(x) for x in sys.argv[3:4]))
