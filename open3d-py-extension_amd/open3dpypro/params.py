"""Search-parameter shims for estimate_normals / KD-tree queries.

The reference defaults to o3d.geometry.KDTreeSearchParamKNN(30)
(/root/reference/open3dpypro/PointCloud.py:68) and test_mesh.py:18 uses
KDTreeSearchParamHybrid(radius, max_nn).  Parameters are duck-typed on
.knn / .radius / .max_nn, so genuine open3d.geometry objects work too.
"""
from __future__ import annotations

from . import _native as N


class KDTreeSearchParamKNN:
    def __init__(self, knn: int = 30):
        self.knn = int(knn)

    def __repr__(self):
        return f"KDTreeSearchParamKNN(knn={self.knn})"


class KDTreeSearchParamRadius:
    def __init__(self, radius: float):
        self.radius = float(radius)

    def __repr__(self):
        return f"KDTreeSearchParamRadius(radius={self.radius})"


class KDTreeSearchParamHybrid:
    def __init__(self, radius: float, max_nn: int):
        self.radius = float(radius)
        self.max_nn = int(max_nn)

    def __repr__(self):
        return f"KDTreeSearchParamHybrid(radius={self.radius}, max_nn={self.max_nn})"


def resolve(param):
    """-> (mode, knn, radius) for the C-ABI."""
    if param is None:
        return N.SEARCH_KNN, 30, 0.0
    has_r = hasattr(param, "radius")
    if has_r and hasattr(param, "max_nn"):
        return N.SEARCH_HYBRID, int(param.max_nn), float(param.radius)
    if has_r:
        return N.SEARCH_RADIUS, 0, float(param.radius)
    if hasattr(param, "knn"):
        return N.SEARCH_KNN, int(param.knn), 0.0
    raise TypeError(f"unsupported search parameter {param!r}")
