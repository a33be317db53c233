"""open3dpypro — MI355X-native drop-in for the qinhy/Open3D-py-extension hot path.

Import surface mirrors the reference (/root/reference/open3dpypro/__init__.py:1-4):
PointCloud, processors.Processors, PointCloudMat, ShapeType, ...  The compute
behind voxel_down_sample / estimate_normals / segment_plane / registration_icp
runs in libo3dx.so (hand-written HIP for gfx950); Open3D is not required.
"""
from . import _native, ops, synthetic  # noqa: F401
from .params import KDTreeSearchParamHybrid, KDTreeSearchParamKNN, KDTreeSearchParamRadius  # noqa: F401
from .PointCloud import (KDTreeGrid, PointCloud, PointCloudBase, PointCloudSelections,  # noqa: F401
                         PointCloudUtility, RegistrationResult, set_random_seed)
from .PointCloudMat import *  # noqa: F401,F403
from .processors import PointCloudMatProcessors, Processors  # noqa: F401
from . import processors  # noqa: F401

__version__ = "0.1.0"
