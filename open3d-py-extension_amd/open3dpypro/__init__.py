"""open3dpypro — MI355X-native drop-in for the qinhy/Open3D-py-extension hot path.

Import surface mirrors the reference (/root/reference/open3dpypro/__init__.py:1-4):
PointCloud, processors.Processors, PointCloudMat, ShapeType, ...  The compute
behind voxel_down_sample / estimate_normals / segment_plane / registration_icp
runs in libo3dx.so (hand-written HIP for gfx950); Open3D is not required.
"""
from . import _native, ops, synthetic  # noqa: F401

__version__ = "0.1.0"
