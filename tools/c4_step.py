"""C4's size on one GPU: five one-call voxel + KNN30 normal steps on 50M
uniform points (for a rocprofv3 kernel trace).  GPU box only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))

import torch  # noqa: E402

from open3dpypro import ops, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
n = int(os.environ.get("N", "50000000"))
pts = S.uniform_cube(n, 0, device=dev)
vs = S.voxel_size_for(n)
for _ in range(5):
    ops.voxel_down_sample_normals(pts, vs, knn=30)
torch.cuda.synchronize()
print("done")
