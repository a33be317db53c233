"""Generate tests/golden/ref_torch_branch.npz from the reference's OWN code.

Run here (the survey container), never on the GPU box:
    python tests/golden/make_golden.py

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


if __name__ == "__main__":
    main()
