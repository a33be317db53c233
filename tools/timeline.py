"""Print the last-N GPU ops (kernels + copies) of a rocprofv3 .db as a
timeline: start offset, duration, gap to the previous op (host-side time).
Usage: python tools/timeline.py <dir with .db> [last_n]"""
import glob
import sqlite3
import sys

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
f = glob.glob(f"{d}/**/*.db", recursive=True)[0]
c = sqlite3.connect(f)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
rows = []
if "kernels" in tabs:
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    nm = "name" if "name" in cols else "kernel_name"
    for r in c.execute(f"select {nm}, start, end from kernels"):
        rows.append((r[1], r[2], "K " + str(r[0])[:70]))
mt = [t for t in tabs if t in ("memory_copies", "memory_copy")]
if mt:
    cols = [r[1] for r in c.execute(f"pragma table_info({mt[0]})")]
    for r in c.execute(f"select * from {mt[0]}"):
        rec = dict(zip(cols, r))
        rows.append((rec.get("start"), rec.get("end"), "C " + str(rec.get("name", rec.get("kind", "copy")))[:40] +
                     " %s B" % rec.get("size", "?")))
rows.sort()
rows = rows[-last:]
t0 = rows[0][0]
prev = None
for s, e, n in rows:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f}  gap {gap:8.1f}  {n}")
    prev = e
