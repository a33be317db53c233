"""rocprofv3 kernel trace -> markdown summary grouped by (kernel, grid size),
so launches of one kernel on different workloads (e.g. the C2 normals vs the
ICP target normals inside one bench run) are averaged separately.
Usage: python tools/prof_summary.py PROF_DIR OUT_MD [title]"""
import collections
import csv
import os
import sys


def main(src, out, title):
    rows = list(csv.DictReader(open(os.path.join(src, "run_kernel_trace.csv"))))
    g = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        g[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in g.values())
    items = sorted(g.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w") as f:
        f.write(f"# {title}\n\nGrouped by (kernel, grid size); durations in microseconds from the kernel trace.\n\n")
        f.write("| kernel | grid | calls | avg | min | max | total | % |\n|---|---|---|---|---|---|---|---|\n")
        for (name, grid), v in items[:40]:
            short = name.split("(")[0].replace("void ", "")[:70]
            f.write(f"| {short} | {grid} | {len(v)} | {sum(v)/len(v):.1f} | {min(v):.1f} | {max(v):.1f} | "
                    f"{sum(v):.1f} | {100*sum(v)/tot:.2f} |\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "rocprofv3 kernel trace")
