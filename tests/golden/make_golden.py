"""Generate tests/golden/ref_torch_branch.npz and tests/golden/ref_glue.npz
from the reference's OWN code.

Run here (the survey container), never on the GPU box:
    python tests/golden/make_golden.py          # ref_torch_branch.npz
    python tests/golden/make_golden.py glue     # ref_glue.npz (see glue())

The reference (/root/reference/open3dpypro) is imported with `open3d` and
`cv2` replaced by MagicMock (neither is installed).  Only its
pure-torch paths run, on CPU, and their outputs are stored as data:
  * TorchNormals.estimate_normals_torch (processors.py:267-303), k = 16
  * VoxelDownsample cuda branch (processors.py:433-448): origin-anchored int32
    hash, representative = first of each hash group, hash-sorted order
  * PlaneDetection.ransac_plane_detection_torch_batched (processors.py:561-627)
    under torch.manual_seed: best plane + inlier count, and the sampled triples
    (re-drawn with the same seed) so the counts can be re-scored.
Inputs are synthetic and stored alongside (x_normals, x_voxel, x_plane).
The Open3D-backed path has no reference output anywhere (open3d absent): the
oracle's Open3D restatement stays "parity unpinned" (oracle/o3d_restate.cpp).
"""
import os
import sys
import unittest.mock as mock

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.modules["open3d"] = mock.MagicMock()
    sys.modules["cv2"] = mock.MagicMock()
    sys.path.insert(0, "/root/reference")
    from open3dpypro.processors import Processors  # noqa: E402  (the reference package)
    from open3dpypro.PointCloudMat import PointCloudMat, ShapeType  # noqa: E402

    rng = np.random.default_rng(2024)
    out = {}

    # TorchNormals: structured cloud (noisy sphere patch + plane) so normals are well conditioned
    n = 2000
    th = rng.uniform(0, np.pi / 2, n)
    ph = rng.uniform(0, np.pi / 2, n)
    sph = np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)], 1)
    xn = (sph * (1.0 + rng.normal(0, 1e-4, (n, 1)))).astype(np.float32)
    tn = Processors.TorchNormals()
    nrm = tn.estimate_normals_torch(torch.from_numpy(xn), k=16).numpy()
    out["x_normals"] = xn
    out["torch_normals_k16"] = nrm

    # VoxelDownsample cuda branch, executed on CPU tensors
    xv = rng.uniform(-1.0, 1.0, (5000, 3)).astype(np.float32)
    m = PointCloudMat(shape_type=ShapeType.XYZ).build(torch.from_numpy(xv))
    m.info.device = "cuda:0"
    vd = Processors.VoxelDownsample(voxel_size=0.1)
    vd.num_gpus = 1
    vd.num_devices = ["cpu"]
    vd.input_mats = [m]
    vd._models = []
    vd.build()
    rep_pts = vd._models[0](torch.from_numpy(xv)).numpy()
    # recover indices of the selected rows
    lut = {tuple(r): i for i, r in enumerate(xv.tolist())}
    out["x_voxel"] = xv
    out["torch_voxel_rep_idx"] = np.array([lut[tuple(r)] for r in rep_pts.tolist()], np.int64)
    out["torch_voxel_size"] = np.float64(0.1)

    # batched RANSAC
    k = 6000
    xp = rng.uniform(0, 1, (k, 3)).astype(np.float32)
    on = rng.uniform(0, 1, k) < 0.3
    xp[on, 2] = (0.4 + rng.normal(0, 0.002, on.sum())).astype(np.float32)
    pd = Processors.PlaneDetection(distance_threshold=0.01)
    torch.manual_seed(7)
    plane, mask = pd.ransac_plane_detection_torch_batched(torch.from_numpy(xp), 0.01, 512, 256)
    torch.manual_seed(7)
    samples = np.concatenate([torch.randint(0, k, (256, 3)).numpy() for _ in range(2)], 0)
    out["x_plane"] = xp
    out["torch_ransac_plane"] = np.asarray(plane, np.float64)
    out["torch_ransac_inliers"] = int(mask.sum().item())
    out["torch_ransac_samples"] = samples.astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "ref_torch_branch.npz"), **out)
    print("wrote", os.path.join(HERE, "ref_torch_branch.npz"), {k: np.shape(v) for k, v in out.items()})


def _point_storage_stand_in():
    """Open3D's point storage only (o3d.geometry.PointCloud().points holding a
    float64 copy of the array — Vector3dVector is a float64 copy, SURVEY.md
    §1): lets the reference's numpy selection code (PointCloud.py:185-276)
    run; no Open3D algorithm is stood in for."""
    def pointcloud(*_a, **_k):
        m = mock.MagicMock()
        m.points = np.zeros((0, 3))
        m.has_points.side_effect = lambda: len(np.asarray(m.points)) > 0
        m.has_colors.return_value = False
        m.has_normals.return_value = False
        return m
    o3d = sys.modules["open3d"]
    o3d.geometry.PointCloud = pointcloud
    o3d.utility.Vector3dVector = lambda a: np.array(a, dtype=np.float64)


def glue():
    """The reference's glue around the hot path, recorded as data
    (VERDICT r3 "What's missing" 1):
      * PlaneNormalize.forward_raw (processors.py:701-759): output and T for
        numpy f32 / f64 (3 and 6 columns), torch-CPU f32 / f64, a normal
        parallel and one anti-parallel to z (the 1e-6 identity quirk);
      * PlaneDetection, CPU branch (processors.py:633-650, 688-699): the
        reference's own d-sign flip and EMA over 3 frames at alpha 0.1 (and
        the default alpha 0), with PointCloud.segment_plane — Open3D's
        SegmentPlane, absent here — replaced by the injected planes
        `pd_planes` (their inliers are not read by the processor);
      * PlaneDetection, torch branch (processors.py:561-627, 655-666,
        688-699): batched torch RANSAC on CPU tensors under
        torch.manual_seed(11), meta after each of 3 frames at alpha 0.1, and
        each frame's plane (the same draws, alpha 1);
      * RandomSample (processors.py:320-365): numpy branch under
        np.random.seed(5), torch branch under torch.manual_seed(5);
      * RadiusSelection (processors.py:367-416): torch branch (pure torch)
        and numpy branch (PointCloud.select_by_radius on the float64 points,
        Open3D's point storage stood in by _point_storage_stand_in)."""
    sys.modules["open3d"] = mock.MagicMock()
    sys.modules["cv2"] = mock.MagicMock()
    _point_storage_stand_in()
    sys.path.insert(0, "/root/reference")
    import importlib

    RPC = importlib.import_module("open3dpypro.PointCloud")  # the reference package's module
    from open3dpypro.processors import Processors  # noqa: E402
    from open3dpypro.PointCloudMat import PointCloudMat, ShapeType  # noqa: E402

    rng = np.random.default_rng(77)
    out = {}

    # --- PlaneNormalize
    base = rng.uniform(-2, 2, (400, 6))
    pn_cases = [
        ("np_f32", base[:, :3].astype(np.float32), [0.12, -0.31, 0.94, 0.37]),
        ("np_f64", base[:, :3].astype(np.float64), [0.12, -0.31, 0.94, 0.37]),
        ("np_f32_6col", base.astype(np.float32), [-0.4, 0.2, 0.89, -1.1]),
        ("torch_f32", base[:, :3].astype(np.float32), [0.02, 0.7, -0.71, 0.25]),
        ("torch_f64", base[:, :3].astype(np.float64), [0.02, 0.7, -0.71, 0.25]),
        ("np_f32_antiparallel", base[:, :3].astype(np.float32), [0.0, 0.0, -1.0, 0.3]),
        ("np_f64_parallel", base[:, :3].astype(np.float64), [0.0, 0.0, 1.0, -0.2]),
        ("torch_f32_unnormalised", base[:, :3].astype(np.float32), [0.5, 0.5, 2.0, 0.8]),
    ]
    for name, x, plane in pn_cases:
        is_np = not name.startswith("torch")
        pn = Processors.PlaneNormalize(detection_uuid="det")
        pn.init_common_utility_methods(0, is_np)
        data = x if is_np else torch.from_numpy(x)
        res = pn.forward_raw([data], [], {"det": [plane]})[0]
        out[f"pn_{name}_x"] = x
        out[f"pn_{name}_plane"] = np.asarray(plane, np.float64)
        out[f"pn_{name}_out"] = res if is_np else res.numpy()
        out[f"pn_{name}_T"] = np.asarray(pn.forward_T[0], np.float64)

    # --- PlaneDetection, CPU branch: injected segment_plane results
    frames = [rng.uniform(0, 1, (300, 3)).astype(np.float32) for _ in range(3)]
    planes = np.array([[0.1, 0.2, 0.97, -0.5], [-0.1, -0.2, -0.97, 0.45], [0.0, 0.6, 0.8, 0.3]])
    out["pd_frames"] = np.stack(frames)
    out["pd_planes"] = planes
    for alpha in (0.1, 0.0):
        it = iter(planes)
        orig = RPC.PointCloudBase.segment_plane
        RPC.PointCloudBase.segment_plane = lambda self, *a, **k: (list(next(it)), [])
        try:
            m = PointCloudMat(shape_type=ShapeType.XYZ).build(frames[0].copy())
            pd = Processors.PlaneDetection(distance_threshold=0.01, alpha=alpha, input_mats=[m])
            pd._models = []
            pd.build()
            pd.best_planes = [[0.0, 0.0, 0.0, 0.0]]
            metas = []
            for f in frames:
                meta = {}
                pd.forward_raw([f], [], meta)
                metas.append(np.asarray(meta[pd.uuid][0], np.float64))
        finally:
            RPC.PointCloudBase.segment_plane = orig
        out[f"pd_cpu_meta_alpha{alpha}"] = np.stack(metas)

    # --- PlaneDetection, torch branch (batched torch RANSAC on CPU tensors)
    tframes = []
    for i in range(3):
        k = 3000
        xp = rng.uniform(0, 1, (k, 3)).astype(np.float32)
        on = rng.uniform(0, 1, k) < 0.4
        xp[on, 2] = (0.3 + 0.1 * i + rng.normal(0, 0.002, on.sum())).astype(np.float32)
        tframes.append(xp)
    out["pdt_frames"] = np.stack(tframes)
    for alpha, key in ((0.1, "pdt_meta_alpha0.1"), (1.0, "pdt_planes")):
        m = PointCloudMat(shape_type=ShapeType.XYZ).build(torch.from_numpy(tframes[0].copy()))
        m.info.device = "cuda:0"
        pd = Processors.PlaneDetection(distance_threshold=0.01, alpha=alpha, num_gpus=1, num_devices=["cpu"],
                                       input_mats=[m])
        pd._models = []
        pd.build()
        pd.best_planes = [[0.0, 0.0, 0.0, 0.0]]
        torch.manual_seed(11)
        metas = []
        for f in tframes:
            meta = {}
            pd.forward_raw([torch.from_numpy(f)], [], meta)
            metas.append(np.asarray(meta[pd.uuid][0], np.float64))
        out[key] = np.stack(metas)

    # --- RandomSample / RadiusSelection
    xr = rng.uniform(-1.5, 1.5, (5000, 4)).astype(np.float32)
    out["rs_x"] = xr
    m = PointCloudMat(shape_type=ShapeType.XYZ).build(xr[:, :3].copy())
    rs = Processors.RandomSample(n_samples=1000, input_mats=[m])
    rs._models = []
    rs.build()
    np.random.seed(5)
    out["rs_np_out"] = rs._models[0](xr)
    mt = PointCloudMat(shape_type=ShapeType.XYZ).build(torch.from_numpy(xr[:, :3].copy()))
    mt.info.device = "cuda:0"
    rst = Processors.RandomSample(n_samples=1000, num_gpus=1, num_devices=["cpu"], input_mats=[mt])
    rst._models = []
    rst.build()
    torch.manual_seed(5)
    out["rs_torch_out"] = rst._models[0](torch.from_numpy(xr)).numpy()
    sel = Processors.RadiusSelection(radius=1.2, input_mats=[m])
    sel._models = []
    sel.build()
    out["rsel_np_out"] = np.asarray(sel._models[0](xr))
    selt = Processors.RadiusSelection(radius=1.2, num_gpus=1, num_devices=["cpu"], input_mats=[mt])
    selt._models = []
    selt.build()
    out["rsel_torch_out"] = selt._models[0](torch.from_numpy(xr)).numpy()
    out["rsel_radius"] = np.float64(1.2)

    np.savez_compressed(os.path.join(HERE, "ref_glue.npz"), **out)
    print("wrote", os.path.join(HERE, "ref_glue.npz"), {k: np.shape(v) for k, v in out.items()})


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "glue":
        glue()
    else:
        main()
