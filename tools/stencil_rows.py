"""Generates O3DX_S25_ROWS (csrc/grid.hip): the voxel rows of the dense-table
normals stencil.  A voxel (dx, dy, dz) belongs to it when its box comes closer
than R voxels to some query in [LO, 1)^3 of the centre voxel (the oriented
frame: the kernel mirrors each axis so the query lies in the upper half)."""
import itertools
import math

R, LO = 2.45, 0.49


def mind(d):
    s = 0.0
    for a in d:
        lo, hi = a, a + 1
        m = LO - hi if hi <= LO else (lo - 1.0 if lo >= 1.0 else 0.0)
        s += m * m
    return math.sqrt(s)


rows = {}
for d in itertools.product(range(-4, 5), repeat=3):
    if mind(d) < R:
        rows.setdefault((d[1], d[2]), []).append(d[0])
out = []
for (dy, dz), xs in sorted(rows.items(), key=lambda t: (t[0][1], t[0][0])):
    xs.sort()
    assert xs == list(range(xs[0], xs[-1] + 1))
    out.append(f"X({dy}, {dz}, {xs[0]}, {xs[-1]})")
print(f"{len(out)} rows, {sum(len(v) for v in rows.values())} voxels")
print(" ".join(out))
