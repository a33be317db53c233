"""CPU: host-side logic of the drop-in, the C-ABI library surface, PCD I/O,
synthetic data.  No kernel is launched here (no GPU in this leg)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import open3dpypro as o3p
from open3dpypro import _native as N
from open3dpypro import pcd_io, synthetic as S
from open3dpypro.PointCloudMat import PointCloudMat, PointCloudMatInfo, ShapeType

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GPU = torch.cuda.is_available()


# ---------------------------------------------------------------- C-ABI
def header_functions():
    txt = open(N.HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(o3dx_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = N.load()  # loads only: no compute call without a GPU
    decl = header_functions()
    assert len(decl) >= 30
    for name in decl:
        assert hasattr(lib, name), name
    assert sorted(N.declared_symbols()) == decl
    assert lib.o3dx_abi_version() == 7


def test_library_host_only_entry_points():
    # pure host functions are callable without a GPU
    out = np.empty((50, 3), np.int32)
    rc = N.load().o3dx_ransac_samples(1000, 3, 50, 11, out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0 and all(len(set(r)) == 3 for r in out)
    from oracle import oracle as O
    assert np.array_equal(out, O.ransac_samples(1000, 3, 50, 11))
    pl = np.zeros(4)
    pts = np.array([[0, 0, 1.0], [1, 0, 1], [0, 1, 1]])
    assert N.load().o3dx_plane_from_points(pts.ctypes.data_as(ctypes.c_void_p), 3,
                                           pl.ctypes.data_as(ctypes.c_void_p)) == 0
    assert np.allclose(pl, [0, 0, 1, -1])
    bad = N.load().o3dx_ransac_samples(2, 3, 5, 0, out.ctypes.data_as(ctypes.c_void_p))
    assert bad == -22 and b"ransac_n" in N.load().o3dx_last_error()


def test_slab_entry_points_validate_before_touching_the_device():
    """ABI 6's slab entry points reject bad arguments with -EINVAL (or
    -ENOMEM for a short workspace) and a message, before any device call
    (so this runs without a GPU)."""
    L = N.load()
    v = ctypes.c_void_p(8)  # never dereferenced: the checks come first
    assert L.o3dx_slab_pack_workspace_bytes(1000) > 0
    rc = L.o3dx_slab_halo_pack(v, v, v, None, 10, 0.0, 0.1, 1, 2, 1, 1, v, v, 4, v, 1 << 30, None)
    assert rc == -22 and b"slab_halo_pack" in L.o3dx_last_error()
    rc = L.o3dx_slab_halo_pack(v, v, v, v, 1000, 0.0, 0.1, 1, 2, 1, 1, v, v, 4, v, 16, None)
    assert rc == -12 and b"workspace" in L.o3dx_last_error()
    rc = L.o3dx_slab_halo_merge(v, v, v, 10, v, 4, 4, v, 17, v, v, None)  # ux rows < cap + na + nb
    assert rc == -22 and b"slab_halo_merge" in L.o3dx_last_error()
    rc = L.o3dx_slab_verdict(v, None, v, 10, v, v, 0.0, 1.0, 1, 1, 0.3, v, v, v, v, None)
    assert rc == -22 and b"slab_verdict" in L.o3dx_last_error()
    lo, hi = np.zeros(3), np.ones(3)
    rc = L.o3dx_voxel_down_sample_window_deferred(v, 10, lo.ctypes.data_as(ctypes.c_void_p),
                                                  hi.ctypes.data_as(ctypes.c_void_p), 0.1, 0, 5, v, v, None, v,
                                                  1 << 30, None)
    assert rc == -22 and b"counts_dev" in L.o3dx_last_error()


def test_icp_solve_host():
    # JTJ = I, JTr = -x  ->  x; small rotation about z + translation
    x = np.array([0, 0, 0.01, 0.1, -0.2, 0.3])
    sums = np.zeros(32)
    t = 0
    for a in range(6):
        for b in range(a, 6):
            sums[t] = 1.0 if a == b else 0.0
            t += 1
    sums[21:27] = -x
    sums[28] = 10
    upd = o3p.ops.icp_solve(sums)
    c, s = np.cos(0.01), np.sin(0.01)
    assert np.allclose(upd[:3, :3], [[c, -s, 0], [s, c, 0], [0, 0, 1]])
    assert np.allclose(upd[:3, 3], x[3:])


def test_icp_solve_rotation_angles_host():
    """The update's rotation uses the library's own sin / cos (the same bits
    on the host and in the device loop, icp.hip det_sincos): within 2 ulp of
    numpy's Rz(c) Ry(b) Rx(a) for angles across several quadrants."""
    rng = np.random.default_rng(5)
    angles = np.concatenate([rng.uniform(-0.05, 0.05, (300, 3)), rng.uniform(-4, 4, (300, 3)),
                             np.array([[np.pi / 2, -np.pi, 3 * np.pi / 4], [1e-9, -1e-12, 0.0], [20.0, -33.0, 7.5]])])
    for x0, x1, x2 in angles:
        sums = np.zeros(32)
        t = 0
        for a in range(6):
            for b in range(a, 6):
                sums[t] = 1.0 if a == b else 0.0
                t += 1
        sums[21:27] = -np.array([x0, x1, x2, 0.5, -1.0, 2.0])
        sums[28] = 1
        upd = o3p.ops.icp_solve(sums)
        ca, sa, cb, sb, cg, sg = np.cos(x0), np.sin(x0), np.cos(x1), np.sin(x1), np.cos(x2), np.sin(x2)
        Rz = np.array([[cg, -sg, 0], [sg, cg, 0], [0, 0, 1]])
        Ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
        Rx = np.array([[1, 0, 0], [0, ca, -sa], [0, sa, ca]])
        assert np.abs(upd[:3, :3] - Rz @ Ry @ Rx).max() < 2e-15, (x0, x1, x2)
        assert np.array_equal(upd[:3, 3], [0.5, -1.0, 2.0]) and np.array_equal(upd[3], [0, 0, 0, 1])


def test_fx_to_double_correctly_rounded():
    """o3dx_fx_to_double (the one conversion of every exact fx sum) equals
    Python's correctly rounded int -> float on random digits, on values with
    more than 53 significant bits, on halfway cases (ties to even), negative
    and extreme exponents; and the numpy restatement's fx rows agree."""
    from oracle import np_restate as NPR
    rng = np.random.default_rng(3)
    rows = []
    for _ in range(2000):
        lo = int(rng.integers(0, 1 << 62))
        hi = int(rng.integers(-(1 << 62), 1 << 62))
        rows.append([lo, hi, int(rng.integers(-200, 100)), 0])
    for v in (2 ** 53 + 1, 2 ** 53 + 3, -(2 ** 54) - 2, 2 ** 80 + 2 ** 27, (1 << 90) - 1, 0, -1, 1):
        rows.append([v & 0xFFFFFFFF, v >> 32, -40, 0])
    fx = np.array(rows, np.int64)
    got = o3p.ops.fx_to_double(fx)
    exp = np.array([NPR.fx_value(r) for r in fx])
    assert np.array_equal(got, exp)
    # digit sums of split terms equal the row of all terms (any order, any split)
    t = rng.normal(0, 1e-3, 10000)
    q = NPR.fx_exp(0.01)
    a, b = NPR.fx_row(t[:3333], q), NPR.fx_row(t[3333:], q)
    whole = NPR.fx_row(t[::-1], q)
    assert NPR.fx_value(a + np.array([b[0], b[1], 0, 0])) == NPR.fx_value(whole)
    assert abs(NPR.fx_value(whole) - t.sum()) < 1e-15


def test_planes_from_samples_and_icp_update_host():
    from oracle import np_restate as NPR
    rng = np.random.default_rng(4)
    c = rng.random((20, 3, 3))
    c[5, 2] = c[5, 0]  # degenerate triple
    P = o3p.ops.planes_from_samples(c, 3)
    for h in range(20):
        assert np.array_equal(P[h], NPR.triangle_plane(*c[h]))
    sums = np.zeros(32)
    sums[[0, 6, 11, 15, 18, 20]] = 1.0
    sums[21:27] = [0, 0, -0.01, -0.1, 0.2, -0.3]
    sums[28] = 5
    T0 = S.rigid_transform(3.0)
    T1 = o3p.ops.icp_update(sums, T0)
    assert np.allclose(T1, o3p.ops.icp_solve(sums) @ T0, atol=1e-15)


def test_ransac_needed_rounds_select_like_exact_counts():
    """Selection on count upper bounds (o3dx_plane_count_upper) refined by
    o3dx_ransac_needed rounds: the tied set and the selected hypothesis equal
    those on the exact counts — random counts, zero planes, degenerate -1,
    ties, and small n so that Open3D's early break (probability) is active."""
    rng = np.random.default_rng(11)
    ops = o3p.ops
    for trial in range(300):
        H = int(rng.integers(1, 200))
        n = int(rng.choice([40, 60, 1000]))
        prob = float(rng.choice([0.5, 0.9, 0.99999999, 1.0]))
        exact = rng.integers(-1, min(n, 45), H)
        planes = rng.normal(size=(H, 4))
        planes[exact < 0] = 0.0
        planes[rng.random(H) < 0.05] = 0.0  # zero planes the replay skips
        ub = np.where(exact >= 0, exact + rng.integers(0, 4, H), exact)
        counts, known, rounds = ub.copy(), np.zeros(H, bool), 0
        while True:
            need = ops.ransac_needed(counts, known, planes, n, 3, prob)
            if not len(need):
                break
            assert not known[need].any()
            counts[need] = exact[need]
            known[need] = True
            rounds += 1
        assert rounds <= H
        tie_e = ops.ransac_tied(exact, planes, n, 3, prob)
        assert np.array_equal(ops.ransac_tied(counts, planes, n, 3, prob), tie_e)
        sums = np.full(H, np.nan)
        sums[tie_e] = rng.random(len(tie_e))
        assert ops.ransac_select(counts, sums, planes, n, 3, prob) == ops.ransac_select(exact, sums, planes, n, 3, prob)


@pytest.mark.skipif(GPU, reason="checks the no-GPU behaviour")
def test_compute_fails_loudly_without_gpu():
    pc = o3p.PointCloud(np.random.rand(100, 3))
    with pytest.raises(RuntimeError):
        pc.voxel_down_sample(0.1)
    with pytest.raises(RuntimeError):
        pc.estimate_normals()
    with pytest.raises(RuntimeError):
        o3p.ops.aabb(torch.rand(10, 3))


# ---------------------------------------------------------------- PCD I/O
def test_read_bunny_pcd():
    f = pcd_io.read_pcd_arrays(os.path.join(ROOT, "tests", "golden", "bunny.pcd"))
    assert set(f) >= {"Intensity", "x", "y", "z", "_"}
    assert len(f["x"]) == 35947
    pc = o3p.PointCloud().read_pcd(os.path.join(ROOT, "tests", "golden", "bunny.pcd"))
    assert pc.size() == 35947 and not pc.has_normals()
    p = pc.get_points()
    assert p.dtype == np.float64
    np.testing.assert_allclose(p.min(0), [-0.0947, -0.0619, 0.033], atol=1e-4)


@pytest.mark.parametrize("ascii_", [False, True])
def test_pcd_roundtrip(tmp_path, ascii_):
    rng = np.random.default_rng(0)
    pts = rng.normal(size=(200, 3)).astype(np.float32).astype(np.float64)
    nrm = rng.normal(size=(200, 3)).astype(np.float32).astype(np.float64)
    col = rng.integers(0, 256, (200, 3)) / 255.0
    fn = str(tmp_path / "c.pcd")
    pcd_io.write_pcd(fn, pts, nrm, col, write_ascii=ascii_)
    p2, n2, c2 = pcd_io.read_pcd(fn)
    assert np.array_equal(p2, pts) and np.array_equal(n2, nrm)
    np.testing.assert_allclose(c2, col, atol=1e-12)


def test_pcd_nan_removal(tmp_path):
    pts = np.array([[0, 0, 0], [np.nan, 1, 1], [np.inf, 0, 0], [1, 2, 3]], np.float64)
    fn = str(tmp_path / "n.pcd")
    pcd_io.write_pcd(fn, pts)
    assert len(pcd_io.read_pcd(fn)[0]) == 4
    assert len(pcd_io.read_pcd(fn, remove_nan_points=True)[0]) == 3
    assert len(pcd_io.read_pcd(fn, remove_nan_points=True, remove_infinite_points=True)[0]) == 2


def test_lzf_decompress():
    # literal run "abc" then back-reference copying "abcabc" (len 6, offset 3)
    stream = bytes([2]) + b"abc" + bytes([(4 << 5) | 0, 2])
    assert pcd_io.lzf_decompress(stream, 9) == b"abcabcabc"


def test_read_other_formats(tmp_path):
    a = np.random.rand(20, 3)
    np.save(tmp_path / "a.npy", a)
    assert np.allclose(o3p.PointCloud().read_pcd(str(tmp_path / "a.npy")).get_points(), a)
    np.savetxt(tmp_path / "a.xyzn", np.hstack([a, a]))
    pc = o3p.PointCloud().read_pcd(str(tmp_path / "a.xyzn"))
    assert pc.has_normals() and np.allclose(pc.get_normals(), a.astype(np.float32))
    with pytest.raises(RuntimeError):
        o3p.PointCloud().read_pcd(str(tmp_path / "a.unknownfmt"))


# ---------------------------------------------------------- PointCloud host
def test_pointcloud_basics():
    xyz = np.random.rand(50, 3)
    rgb = np.random.rand(50, 3) * 255
    pc = o3p.PointCloud(xyz, rgb=rgb, intensity=np.arange(50).reshape(-1, 1),
                        labels=np.arange(50).reshape(-1, 1) % 3)
    assert pc.size() == 50 and pc.has_rgb() and pc.has_intensity() and pc.has_labels()
    assert np.array_equal(pc.get_points(), xyz)  # exact float64 round trip
    c = pc.get_colors()
    assert abs(c.min()) < 1e-6 and abs(c.max() - 1) < 1e-6  # reference PointCloud.py:36-40 rescale
    with pytest.raises(AssertionError):
        pc.set_points(np.zeros((3, 2)))
    with pytest.raises(AssertionError):
        pc.set_intensity(np.zeros((3, 2)))


def test_select_by_idx_order_and_attributes():
    xyz = np.random.rand(30, 3)
    pc = o3p.PointCloud(xyz, intensity=np.arange(30).reshape(-1, 1), labels=np.arange(30).reshape(-1, 1))
    s = pc._select_by_idx([7, 2, 2, 29])  # mask semantics: ascending, de-duplicated
    assert np.array_equal(s.get_points(), xyz[[2, 7, 29]])
    assert np.array_equal(s.intensity.ravel(), [2, 7, 29])
    inv = pc._select_by_idx([7, 2], invert=True)
    assert inv.size() == 28 and 2 not in inv.intensity.ravel()
    t = pc._select_by_idx(torch.tensor([3, 1]))
    assert np.array_equal(t.get_points(), xyz[[1, 3]])
    assert pc.clone().size() == 30 and pc.clone(invert=True).size() == 0


def test_selections_and_planes():
    xyz = np.array([[0, 0, 0.0], [0, 0, 0.5], [0, 0, 1.0], [3, 0, 0]])
    pc = o3p.PointCloud(xyz)
    assert list(pc.get_index_by_radius(1.0)) == [0, 1, 2]
    assert pc.select_by_aabb([-1, -1, -1], [1, 1, 0.7]).size() == 2
    assert pc.select_by_topN(2).size() == 2
    # plane selection / distance2plane run on the GPU: tests/test_gpu_api.py::test_plane_selection_*


def test_split_pcd_index_partitions():
    pc = o3p.PointCloud(np.random.rand(103, 3))
    parts = pc.split_pcd_index(10)
    assert sum(len(p) for p in parts) == 103 and len(parts) == 10
    assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(103))


def test_transform_translate():
    xyz = np.random.rand(10, 3)
    pc = o3p.PointCloud(xyz, normals=np.tile([[0, 0, 1.0]], (10, 1)))
    T = S.rigid_transform(30, (0, 0, 1), (1, 2, 3))
    pc.transform(T)
    np.testing.assert_allclose(pc.get_points(), xyz @ T[:3, :3].T + T[:3, 3], atol=1e-12)
    np.testing.assert_allclose(pc.get_normals(), np.tile([[0, 0, 1.0]], (10, 1)), atol=1e-6)
    pc.translate([1, 0, 0])
    np.testing.assert_allclose(pc.get_points()[:, 0], (xyz @ T[:3, :3].T + T[:3, 3])[:, 0] + 1, atol=1e-12)


def test_kdtree_params():
    from open3dpypro.params import resolve
    assert resolve(o3p.KDTreeSearchParamKNN(12)) == (N.SEARCH_KNN, 12, 0.0)
    assert resolve(o3p.KDTreeSearchParamRadius(0.5)) == (N.SEARCH_RADIUS, 0, 0.5)
    assert resolve(o3p.KDTreeSearchParamHybrid(0.01, 30)) == (N.SEARCH_HYBRID, 30, 0.01)


# --------------------------------------------------------- PointCloudMat
def test_pointcloudmat_validation():
    m = PointCloudMat(shape_type=ShapeType.XYZRGB).build(np.zeros((5, 6), np.float32))
    assert m.info.N == 5 and m.info.device == "cpu" and m.info.raw_shape == [5, 6]
    with pytest.raises(ValueError):
        PointCloudMat(shape_type=ShapeType.XYZ).build(np.zeros((5, 4), np.float32))
    with pytest.raises(ValueError):
        PointCloudMat(shape_type=ShapeType.XYZ).build(np.zeros(5, np.float32))
    with pytest.raises(TypeError):
        PointCloudMat(shape_type=ShapeType.XYZ).build([[0, 0, 0]])
    with pytest.raises(TypeError):
        m.require_torch_tensor()
    t = PointCloudMat(shape_type=ShapeType.XYZ).build(torch.zeros((4, 3), dtype=torch.float64))
    with pytest.raises(TypeError):
        t.require_torch_float()
    assert ShapeType.XYZ.add_normals() == ShapeType.XYZN and ShapeType.XYZRGBiN.contains_normals()
    assert PointCloudMat.random("XYZN", 7).data().shape == (7, 6)


def test_build_out_mats_rules():
    p = o3p.Processors.DoingNothing()
    a = PointCloudMat(shape_type=ShapeType.XYZ).build(np.zeros((3, 3), np.float32))
    b = PointCloudMat(shape_type=ShapeType.XYZN).build(np.zeros((3, 6), np.float32))
    assert len(p.build_out_mats([a], [np.zeros((2, 3)), np.zeros((1, 3))])) == 2
    assert p.build_out_mats([a, a], [np.zeros((2, 3))])[0].info.shape_type == ShapeType.XYZ
    with pytest.raises(ValueError):
        p.build_out_mats([a, b], [np.zeros((2, 3))])
    with pytest.raises(ValueError):
        p.build_out_mats([a, a, a], [np.zeros((2, 3)), np.zeros((2, 3))])


def test_pipeline_json_roundtrip():
    pipes = [o3p.Processors.RandomSample(n_samples=5), o3p.Processors.VoxelDownsample(voxel_size=0.2),
             o3p.Processors.PlaneDetection(distance_threshold=0.02, alpha=0.1),
             o3p.Processors.ICP(max_correspondence_distance=0.05)]
    js = o3p.PointCloudMatProcessors.dumps(pipes)
    back = o3p.PointCloudMatProcessors.loads(js)
    assert [type(p) for p in back] == [type(p) for p in pipes]
    assert back[2].alpha == 0.1 and back[1].voxel_size == 0.2
    assert back[0].uuid == pipes[0].uuid


def test_host_processors_run():
    data = np.random.rand(100, 3).astype(np.float32)
    m = PointCloudMat(shape_type=ShapeType.XYZ).build(data)
    meta = {}
    pipes = [o3p.Processors.RandomSample(n_samples=40), o3p.Processors.RadiusSelection(radius=1.0)]
    out, meta = o3p.PointCloudMatProcessors.run_once([m], meta, pipes, validate=True)
    assert out[0].data().shape[0] <= 40
    # PlaneNormalize maps the plane z = 0.5 onto z = 0
    pn = o3p.Processors.PlaneNormalize(detection_uuid="det")
    pts = np.c_[np.random.rand(10, 2), np.full(10, 0.5)].astype(np.float32)
    mm = PointCloudMat(shape_type=ShapeType.XYZ).build(pts)
    res, _ = pn.validate([mm], {"det": [[0, 0, 1, -0.5]]})
    np.testing.assert_allclose(res[0].data()[:, 2], 0, atol=1e-6)


# ------------------------------------------------------------- synthetic
def test_synthetic_deterministic_and_sharded():
    a = S.uniform_cube(1000, 3)
    b = torch.cat([S.uniform_cube(400, 3), S.uniform_cube(600, 3, offset=400)])
    assert torch.equal(a, b)
    assert a.min() >= 0 and a.max() < 1
    p = S.planted_plane(20000, 1)
    assert 0.15 < ((p[:, 2] - 0.5).abs() < 0.01).float().mean() < 0.3
    s = S.box_surface(5000, 2)
    on_face = ((s == 0) | (s == torch.tensor([1.0, 0.8, 0.6]))).any(1)
    assert bool(on_face.all())


def _lzf_compress(data: bytes) -> bytes:
    """Small greedy liblzf-format compressor (test helper): back references
    (>= 3 bytes, offset <= 8192) found by a hash of 3-byte prefixes."""
    out = bytearray()
    lit = bytearray()
    table = {}
    i, n = 0, len(data)

    def flush():
        while lit:
            chunk = lit[:32]
            out.append(len(chunk) - 1)
            out.extend(chunk)
            del lit[:32]

    while i < n:
        ref = table.get(data[i:i + 3]) if i + 3 <= n else None
        if i + 3 <= n:
            table[data[i:i + 3]] = i
        if ref is not None and 0 < i - ref <= 8192:
            ln = 0
            while i + ln < n and ln < 264 and data[ref + ln] == data[i + ln]:
                ln += 1
            if ln >= 3:
                flush()
                off = i - ref - 1
                l2 = ln - 2
                if l2 < 7:
                    out.append((l2 << 5) | (off >> 8))
                else:
                    out.append((7 << 5) | (off >> 8))
                    out.append(l2 - 7)
                out.append(off & 0xFF)
                i += ln
                continue
        lit.append(data[i])
        i += 1
    flush()
    return bytes(out)


def write_pcd_compressed(path, pts, normals=None, rgb_u32=None):
    cols = [("x", pts[:, 0]), ("y", pts[:, 1]), ("z", pts[:, 2])]
    if normals is not None:
        cols += [("normal_x", normals[:, 0]), ("normal_y", normals[:, 1]), ("normal_z", normals[:, 2])]
    if rgb_u32 is not None:
        cols.append(("rgb", rgb_u32))
    n = len(pts)
    body = b"".join(np.ascontiguousarray(c, np.uint32 if k == "rgb" else np.float32).tobytes() for k, c in cols)
    comp = _lzf_compress(body)
    head = ("VERSION 0.7\nFIELDS " + " ".join(k for k, _ in cols) + "\nSIZE " + " ".join("4" for _ in cols) +
            "\nTYPE " + " ".join("U" if k == "rgb" else "F" for k, _ in cols) + "\nCOUNT " +
            " ".join("1" for _ in cols) + f"\nWIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\n"
            "DATA binary_compressed\n")
    import struct
    with open(path, "wb") as f:
        f.write(head.encode() + struct.pack("<II", len(comp), len(body)) + comp)
    return body


def test_lzf_library_matches_python(tmp_path):
    """o3dx_lzf_decompress (host code in libo3dx.so) vs the Python decoder,
    on a stream with literal runs and overlapping back references."""
    import ctypes

    from open3dpypro import _native as N
    from open3dpypro import pcd_io

    rng = np.random.default_rng(3)
    data = bytes(rng.integers(0, 4, 5000, dtype=np.uint8)) + b"abcabcabcabc" * 50 + bytes(range(256)) * 3
    comp = _lzf_compress(data)
    assert pcd_io.lzf_decompress(comp, len(data)) == data
    src = np.frombuffer(comp, np.uint8)
    dst = np.zeros(len(data), np.uint8)
    got = N.load().o3dx_lzf_decompress(src.ctypes.data_as(ctypes.c_void_p), src.size,
                                       dst.ctypes.data_as(ctypes.c_void_p), dst.size)
    assert got == len(data) and dst.tobytes() == data
    bad = N.load().o3dx_lzf_decompress(src.ctypes.data_as(ctypes.c_void_p), src.size,
                                       dst.ctypes.data_as(ctypes.c_void_p), 10)
    assert bad < 0


def test_pcd_binary_compressed_host_reader(tmp_path):
    from open3dpypro import pcd_io

    rng = np.random.default_rng(4)
    pts = rng.random((3000, 3)).astype(np.float32)
    nrm = rng.standard_normal((3000, 3)).astype(np.float32)
    rgb = rng.integers(0, 1 << 24, 3000).astype(np.uint32)
    p = str(tmp_path / "c.pcd")
    write_pcd_compressed(p, pts, nrm, rgb)
    P, Nn, C = pcd_io.read_pcd(p)
    assert np.array_equal(P, pts.astype(np.float64)) and np.array_equal(Nn, nrm.astype(np.float64))
    assert np.allclose(C * 255.0, np.stack([(rgb >> 16) & 255, (rgb >> 8) & 255, rgb & 255], 1))


def test_anchored_moment_sums_are_correctly_rounded():
    """grid.hip MomAccA (the sorted-grid tile kernel's moments): anchored
    Fast2Sum per moment, restated in numpy float64 with the kernel's operation
    order, equals math.fsum (the correctly rounded exact sum) on every moment
    of random neighbourhoods — offsets, scales and mixed signs included — so
    its bits equal the double-double (TwoSum) accumulator's."""
    import math
    rng = np.random.default_rng(7)
    for trial in range(400):
        k = int(rng.integers(1, 65))
        scale = 10.0 ** rng.uniform(-3, 2)
        q = (rng.uniform(-1, 1, 3) * scale * rng.choice([1, 10, 100])).astype(np.float32)
        r = scale * rng.uniform(0.01, 0.5)
        p = (q.astype(np.float64) + rng.uniform(-1, 1, (k, 3)) * r / np.sqrt(3)).astype(np.float32)
        d2 = ((p.astype(np.float64) - q) ** 2).sum(1)
        r2 = np.float32(d2.max() * (1 + 2 * 2.0 ** -20))
        rr = math.sqrt(float(r2)) * (1.0 + 1e-6) + 1e-30
        X, Y, Z = (abs(float(c)) + rr for c in q)
        b = [X, Y, Z, X * X, X * Y, X * Z, Y * Y, Y * Z, Z * Z]
        a = [math.ldexp(1.0, math.frexp(k * bj)[1] - 1 + 3) for bj in b]  # ilogb(v) = frexp exponent - 1
        m, l = list(a), [0.0] * 9
        for x, y, z in p.astype(np.float64):
            for j, t in enumerate((x, y, z, x * x, x * y, x * z, y * y, y * z, z * z)):
                s = m[j] + t
                l[j] += t - (s - m[j])
                m[j] = s
        got = [(m[j] - a[j]) + l[j] for j in range(9)]
        pp = p.astype(np.float64)
        cols = [pp[:, 0], pp[:, 1], pp[:, 2], pp[:, 0] * pp[:, 0], pp[:, 0] * pp[:, 1], pp[:, 0] * pp[:, 2],
                pp[:, 1] * pp[:, 1], pp[:, 1] * pp[:, 2], pp[:, 2] * pp[:, 2]]
        exp = [math.fsum(c.tolist()) for c in cols]
        assert got == exp, (trial, k, got, exp)


def test_f32_exact_check():
    """PointCloud's float64 boundary test: float32-representable float64
    values (NaN included) take the float32 kernels, anything else float64."""
    from open3dpypro.PointCloud import _f32_exact

    a = np.array([[0.5, 1.25, np.nan], [3.0, -2.0, 1e30]])
    assert not _f32_exact(a)  # 1e30 is not a float32 value
    a[1, 2] = np.float32(1e30)
    assert _f32_exact(a) and _f32_exact(torch.from_numpy(a))
    b = a.copy()
    b[0, 0] = 0.1
    assert not _f32_exact(b) and not _f32_exact(torch.from_numpy(b))
    las = S.las_scene(1000).numpy()
    assert not _f32_exact(las) and _f32_exact(las.astype(np.float32).astype(np.float64))
