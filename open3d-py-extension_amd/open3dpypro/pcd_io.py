"""PCD (Point Cloud Data v0.7) reader/writer without Open3D.

Replaces o3d.io.read_point_cloud / write_point_cloud for the `.pcd` format
behind PointCloudBase.read_pcd / save_pcd (reference
open3dpypro/PointCloud.py:165-170).  Like Open3D's legacy reader it maps
x/y/z -> points, normal_x/normal_y/normal_z -> normals and rgb/rgba (packed
0x00RRGGBB) -> colors in [0,1]; other fields are parsed and returned by
read_pcd_arrays but not attached to the cloud.  DATA ascii, binary and
binary_compressed (LZF) are supported.

read_pcd_device is the hot-path reader: the header is
parsed here, the raw DATA bytes go to HBM in one copy (binary_compressed is
LZF-decompressed on the host by the library first), and o3dx_pcd_unpack
decodes every field on the GPU straight into the device arrays the
PointCloud keeps.
"""
from __future__ import annotations

import numpy as np

_NP = {("F", 4): np.float32, ("F", 8): np.float64, ("U", 1): np.uint8, ("U", 2): np.uint16,
       ("U", 4): np.uint32, ("U", 8): np.uint64, ("I", 1): np.int8, ("I", 2): np.int16,
       ("I", 4): np.int32, ("I", 8): np.int64}


def _parse_header(f):
    hdr = {}
    while True:
        line = f.readline()
        if not line:
            raise RuntimeError("PCD header ended before DATA")
        s = line.decode("ascii", errors="replace").strip()
        if not s or s.startswith("#"):
            continue
        key, *vals = s.split()
        hdr[key.upper()] = vals
        if key.upper() == "DATA":
            return hdr


def lzf_decompress(src: bytes, out_len: int) -> bytes:
    """LZF (liblzf) decompression, the codec of DATA binary_compressed."""
    out = bytearray(out_len)
    ip = op = 0
    n = len(src)
    while ip < n:
        ctrl = src[ip]
        ip += 1
        if ctrl < 32:  # literal run of ctrl+1 bytes
            ln = ctrl + 1
            out[op:op + ln] = src[ip:ip + ln]
            ip += ln
            op += ln
        else:  # back reference
            ln = ctrl >> 5
            ref = op - ((ctrl & 0x1F) << 8) - 1
            if ln == 7:
                ln += src[ip]
                ip += 1
            ref -= src[ip]
            ip += 1
            ln += 2
            if ref < 0:
                raise RuntimeError("corrupt LZF stream")
            for k in range(ln):  # may overlap
                out[op + k] = out[ref + k]
            op += ln
    if op != out_len:
        raise RuntimeError("LZF length mismatch")
    return bytes(out)


def read_pcd_arrays(filename: str) -> dict:
    """All fields of a PCD file as numpy arrays (count>1 fields -> (n, count))."""
    with open(filename, "rb") as f:
        h = _parse_header(f)
        fields = h["FIELDS"]
        sizes = [int(v) for v in h.get("SIZE", ["4"] * len(fields))]
        types = h.get("TYPE", ["F"] * len(fields))
        counts = [int(v) for v in h.get("COUNT", ["1"] * len(fields))]
        npts = int(h["POINTS"][0]) if "POINTS" in h else int(h["WIDTH"][0]) * int(h.get("HEIGHT", ["1"])[0])
        mode = h["DATA"][0].lower()
        dtypes = [np.dtype(_NP[(t.upper(), s)]) for t, s in zip(types, sizes)]
        out = {}
        if mode == "ascii":
            rows = []
            for line in f:
                s = line.decode("ascii", errors="replace").split()
                if s:
                    rows.append(s)
                if len(rows) == npts:
                    break
            cols = np.array(rows, dtype=object).reshape(len(rows), -1) if rows else np.zeros((0, sum(counts)), object)
            c = 0
            for name, dt, cnt in zip(fields, dtypes, counts):
                a = cols[:, c:c + cnt].astype(np.float64).astype(dt)
                out[name] = a[:, 0] if cnt == 1 else a
                c += cnt
        elif mode == "binary":
            rec = np.dtype([(f"f{i}", dt, (cnt,)) for i, (dt, cnt) in enumerate(zip(dtypes, counts))])
            raw = np.frombuffer(f.read(rec.itemsize * npts), dtype=rec, count=npts)
            for i, (name, cnt) in enumerate(zip(fields, counts)):
                a = np.array(raw[f"f{i}"])
                out[name] = a[:, 0] if cnt == 1 else a
        elif mode == "binary_compressed":
            import struct

            csize, usize = struct.unpack("<II", f.read(8))
            data = lzf_decompress(f.read(csize), usize)
            off = 0
            for name, dt, cnt in zip(fields, dtypes, counts):  # column-major layout
                nb = dt.itemsize * cnt * npts
                a = np.frombuffer(data[off:off + nb], dtype=dt).reshape(npts, cnt).copy()
                out[name] = a[:, 0] if cnt == 1 else a
                off += nb
        else:
            raise RuntimeError(f"unsupported PCD DATA mode {mode!r}")
    return out


def _unpack_rgb(a: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(a).view(np.uint32) if a.dtype.itemsize == 4 else a.astype(np.uint32)
    r = (u >> 16) & 0xFF
    g = (u >> 8) & 0xFF
    b = u & 0xFF
    return np.stack([r, g, b], 1).astype(np.float64) / 255.0


def read_pcd(filename: str, remove_nan_points: bool = False, remove_infinite_points: bool = False):
    """-> (points (n,3) float64, normals or None, colors or None), Open3D's field mapping."""
    fl = read_pcd_arrays(filename)
    if not all(k in fl for k in ("x", "y", "z")):
        raise RuntimeError(f"{filename}: PCD has no x/y/z fields")
    pts = np.stack([fl["x"], fl["y"], fl["z"]], 1).astype(np.float64)
    nrm = None
    if all(k in fl for k in ("normal_x", "normal_y", "normal_z")):
        nrm = np.stack([fl["normal_x"], fl["normal_y"], fl["normal_z"]], 1).astype(np.float64)
    col = None
    for k in ("rgb", "rgba"):
        if k in fl:
            col = _unpack_rgb(fl[k])
            break
    keep = np.ones(len(pts), bool)
    if remove_nan_points:
        keep &= ~np.isnan(pts).any(1)
        if nrm is not None:
            keep &= ~np.isnan(nrm).any(1)
    if remove_infinite_points:
        keep &= ~np.isinf(pts).any(1)
        if nrm is not None:
            keep &= ~np.isinf(nrm).any(1)
    if not keep.all():
        pts = pts[keep]
        nrm = nrm[keep] if nrm is not None else None
        col = col[keep] if col is not None else None
    return pts, nrm, col


def write_pcd(filename: str, points: np.ndarray, normals=None, colors=None, write_ascii: bool = False) -> bool:
    pts = np.asarray(points, np.float32).reshape(-1, 3)
    cols = [("x", pts[:, 0]), ("y", pts[:, 1]), ("z", pts[:, 2])]
    if normals is not None:
        nr = np.asarray(normals, np.float32).reshape(-1, 3)
        cols += [("normal_x", nr[:, 0]), ("normal_y", nr[:, 1]), ("normal_z", nr[:, 2])]
    if colors is not None:
        c = np.clip(np.round(np.asarray(colors, np.float64).reshape(-1, 3) * 255.0), 0, 255).astype(np.uint32)
        cols.append(("rgb", ((c[:, 0] << 16) | (c[:, 1] << 8) | c[:, 2]).astype(np.uint32)))
    n = len(pts)
    names = [c[0] for c in cols]
    types = ["U" if nm == "rgb" else "F" for nm in names]
    head = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\n"
            f"FIELDS {' '.join(names)}\nSIZE {' '.join(['4'] * len(names))}\n"
            f"TYPE {' '.join(types)}\nCOUNT {' '.join(['1'] * len(names))}\n"
            f"WIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\n"
            f"DATA {'ascii' if write_ascii else 'binary'}\n")
    with open(filename, "wb") as f:
        f.write(head.encode("ascii"))
        if write_ascii:
            strs = [[str(int(v)) for v in a] if nm == "rgb" else [repr(float(v)) for v in a] for nm, a in cols]
            for row in zip(*strs):
                f.write((" ".join(row) + "\n").encode("ascii"))
        else:
            rec = np.empty(n, dtype=[(nm, np.uint32 if nm == "rgb" else np.float32) for nm in names])
            for nm, v in cols:
                rec[nm] = v
            f.write(rec.tobytes())
    return True


def read_pcd_device(filename: str, device, remove_nan_points: bool = False, remove_infinite_points: bool = False):
    """-> (points (n,3) float32, normals or None, colors or None) as tensors on
    `device`, decoded on the GPU (o3dx_pcd_unpack).  ascii DATA is parsed on
    the host (text) and copied."""
    import ctypes
    import struct

    import torch

    from . import _native as N

    dev = torch.device(device)
    with open(filename, "rb") as f:
        h = _parse_header(f)
        mode = h["DATA"][0].lower()
        fields = h["FIELDS"]
        sizes = [int(v) for v in h.get("SIZE", ["4"] * len(fields))]
        types = [t.upper() for t in h.get("TYPE", ["F"] * len(fields))]
        wide = any(k in fields and sizes[fields.index(k)] == 8 for k in ("x", "y", "z"))
        if mode == "ascii" or wide:
            # ASCII values and F8 coordinates are float64 data (Open3D reads
            # them into its float64 storage): host decode, float64 points —
            # PointCloud keeps them in float64 when float32 cannot hold them
            f.close()
            pts, nrm, col = read_pcd(filename, remove_nan_points, remove_infinite_points)
            tt = lambda a, dt=np.float32: None if a is None else torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)  # noqa: E731
            return tt(pts, np.float64), tt(nrm), tt(col)
        counts = [int(v) for v in h.get("COUNT", ["1"] * len(fields))]
        npts = int(h["POINTS"][0]) if "POINTS" in h else int(h["WIDTH"][0]) * int(h.get("HEIGHT", ["1"])[0])
        rec = sum(sz * c for sz, c in zip(sizes, counts))
        if mode == "binary":
            raw = np.fromfile(f, dtype=np.uint8, count=rec * npts)
            if raw.size != rec * npts:
                raise RuntimeError(f"{filename}: truncated PCD binary data")
        elif mode == "binary_compressed":
            csize, usize = struct.unpack("<II", f.read(8))
            comp = np.frombuffer(f.read(csize), dtype=np.uint8)
            raw = np.empty(usize, dtype=np.uint8)
            got = N.load().o3dx_lzf_decompress(comp.ctypes.data_as(ctypes.c_void_p), comp.size,
                                               raw.ctypes.data_as(ctypes.c_void_p), usize)
            if got != usize:
                N.check(-22 if got >= 0 else int(got), "read_pcd (LZF)")
        else:
            raise RuntimeError(f"unsupported PCD DATA mode {mode!r}")
    if not all(k in fields for k in ("x", "y", "z")):
        raise RuntimeError(f"{filename}: PCD has no x/y/z fields")
    columnar = mode == "binary_compressed"
    # byte offset of each field: inside a record, or of its column block
    off, o = {}, 0
    for name, sz, c in zip(fields, sizes, counts):
        off[name] = (o, sz)
        o += sz * c * (npts if columnar else 1)
    buf = torch.from_numpy(raw).to(dev)
    pts = torch.empty((npts, 3), dtype=torch.float32, device=dev)
    has_n = all(k in fields for k in ("normal_x", "normal_y", "normal_z"))
    nrm = torch.empty((npts, 3), dtype=torch.float32, device=dev) if has_n else None
    ckey = next((k for k in ("rgb", "rgba") if k in fields), None)
    col = torch.empty((npts, 3), dtype=torch.float32, device=dev) if ckey else None
    plan = [(k, pts, a) for a, k in enumerate(("x", "y", "z"))]
    if has_n:
        plan += [(k, nrm, a) for a, k in enumerate(("normal_x", "normal_y", "normal_z"))]
    tys, so, ss, dp, ds = [], [], [], [], []
    for name, out, a in plan:
        o, sz = off[name]
        t = N.PCD_TYPES.get((types[fields.index(name)], sz))
        if t is None:
            raise RuntimeError(f"{filename}: unsupported PCD field type for {name!r}")
        tys.append(t), so.append(o), ss.append(sz if columnar else rec), dp.append(out.data_ptr() + 4 * a), ds.append(3)
    if ckey:
        o, sz = off[ckey]
        if sz != 4:
            raise RuntimeError(f"{filename}: PCD colour field must be 4 bytes")
        tys.append(N.PCD_RGB), so.append(o), ss.append(sz if columnar else rec), dp.append(col.data_ptr()), ds.append(3)
    nf = len(tys)
    arr = lambda v, ty: (ty * nf)(*v)  # noqa: E731
    N.check(N.load().o3dx_pcd_unpack(ctypes.c_void_p(buf.data_ptr()), npts, nf, arr(tys, ctypes.c_int32),
                                     arr(so, ctypes.c_int64), arr(ss, ctypes.c_int64),
                                     arr(dp, ctypes.c_void_p), arr(ds, ctypes.c_int64), N.stream_ptr(dev)),
            "read_pcd")
    del buf
    if remove_nan_points or remove_infinite_points:
        keep = torch.ones(npts, dtype=torch.bool, device=dev)
        for a in ([pts] + ([nrm] if nrm is not None else [])):
            if remove_nan_points:
                keep &= ~torch.isnan(a).any(1)
            if remove_infinite_points:
                keep &= ~torch.isinf(a).any(1)
        if not bool(keep.all()):
            pts = pts[keep]
            nrm = nrm[keep] if nrm is not None else None
            col = col[keep] if col is not None else None
    return pts, nrm, col
