"""PointCloud — drop-in for open3dpypro.PointCloud (reference
/root/reference/open3dpypro/PointCloud.py), without Open3D.

Storage: points / normals / colors live on the GPU as float32 (N,3) torch
tensors (the kernels' input layout); a float64 host copy of the points is kept
when the caller supplied host data, so get_points() round-trips the caller's
values exactly, as Open3D's float64 storage does.  A float64 cloud that
float32 cannot hold (a LAS / E57 scan at a georeferenced offset; the check
runs once per set_points) also keeps a float64 device copy, and the hot-path
methods run the float64 kernels on it (ops / include/o3dx.h "float64
boundary"): voxel keys, kNN distances, normals' moments, RANSAC distances and
ICP are then computed from the float64 values, as Open3D computes them.
intensity / labels / row / column indices are plain numpy attributes, as in
the reference.

The hot-path methods call libo3dx.so (ops.py); there is no CPU fallback —
without an MI355X they raise RuntimeError.  Host-only helpers (selections by
numpy predicate, splitting, I/O) run anywhere.  Out of scope (SURVEY.md §2
rows 2 and 5) and not mirrored: DBSCAN, to_2D_Img, the colour-cosine
selections.
"""
from __future__ import annotations

import os
import uuid
from typing import Callable, List, Tuple

import numpy as np
import torch

from . import ops, pcd_io
from . import _native as N
from .params import KDTreeSearchParamKNN, resolve

_SEED = [None]


def _sor_keep_sequential(avg: np.ndarray, nv: int, std_ratio: float) -> np.ndarray:
    """RemoveStatisticalOutliers' cloud statistics in Open3D's order:
    std::accumulate of the positive means, std::inner_product of their
    squared deviations (both sequential over the index), then the decision."""
    pos = avg > 0
    S = np.add.accumulate(np.where(pos, avg, 0.0))[-1]
    m = S / nv
    t = np.where(pos, (avg - m) * (avg - m), 0.0)
    sq = np.add.accumulate(t)[-1]
    with np.errstate(divide="ignore", invalid="ignore"):
        std = np.sqrt(sq / np.float64(nv - 1))
    thr = m + std_ratio * std
    return np.nonzero(pos & (avg < thr))[0].astype(np.int64)


def set_random_seed(seed: int):
    """Counterpart of o3d.utility.random.seed: seeds segment_plane's sampler."""
    _SEED[0] = int(seed)


def _next_seed() -> int:
    if _SEED[0] is None:
        return int(np.random.SeedSequence().entropy) & 0xFFFFFFFF
    s = _SEED[0]
    _SEED[0] = (s * 6364136223846793005 + 1442695040888963407) & 0xFFFFFFFFFFFFFFFF
    return s & 0xFFFFFFFF


def _device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def _as_np(a) -> np.ndarray:
    if isinstance(a, torch.Tensor):
        return a.detach().cpu().numpy()
    return np.asarray(a)


def _f32_exact(a) -> bool:
    """Every value of the float64 array / tensor is a float32 value (NaN
    included): the float32 kernels then see exactly Open3D's float64 inputs."""
    if isinstance(a, torch.Tensor):
        t = a.detach()
        return bool(((t.float().double() == t) | torch.isnan(t)).all().item())
    with np.errstate(over="ignore", invalid="ignore"):
        return bool(np.array_equal(a.astype(np.float32).astype(np.float64), a, equal_nan=True))


def _check3(a, what):
    if a.ndim != 2 or a.shape[1] != 3:
        raise AssertionError(f"{what} shape must be (n,3)")


class RegistrationResult:
    """Mirror of o3d.pipelines.registration.RegistrationResult."""

    def __init__(self, transformation, fitness, inlier_rmse, correspondence_set):
        self.transformation = transformation
        self.fitness = fitness
        self.inlier_rmse = inlier_rmse
        self.correspondence_set = correspondence_set

    def __repr__(self):
        return (f"RegistrationResult with fitness={self.fitness:e}, inlier_rmse={self.inlier_rmse:e}, "
                f"and correspondence_set size of {len(self.correspondence_set)}")


class KDTreeGrid:
    """Stand-in for o3d.geometry.KDTreeFlann (reference PointCloud.py:148-163):
    the same search_* methods and return shapes (k, IntVector-like int64
    indices, DoubleVector-like float64 d^2).  Each call is one device query of
    any size (o3dx_search_one: a float64 d^2 pass over the cloud, the
    candidates compacted and radix-sorted by (d^2, index)) — the reference's
    get_points_by_knn asks for up to 10^6 neighbours."""

    def __init__(self, cloud: "PointCloudBase"):
        self._x = cloud._hot_points()

    def _one(self, query, mode, knn, radius):
        k, idx, d2 = ops.search_one(self._x, np.asarray(query, np.float64).reshape(3), mode=mode, knn=knn,
                                    radius=radius)
        return k, idx.cpu().numpy().astype(np.int64), d2.cpu().numpy()

    def search_knn_vector_3d(self, query, knn: int):
        return self._one(query, N.SEARCH_KNN, knn, 0.0)

    def search_hybrid_vector_3d(self, query, radius: float, max_nn: int):
        return self._one(query, N.SEARCH_HYBRID, max_nn, radius)

    def search_radius_vector_3d(self, query, radius: float):
        return self._one(query, N.SEARCH_RADIUS, 0, radius)


def _warn_offset_icp(src: "PointCloudBase", tgt: "PointCloudBase"):
    """Point-to-plane ICP forms J = p x n on the raw coordinates, so its 6x6
    normal matrix has entries ~|p|^2 against ~1: far from the origin relative
    to its extent (georeferenced LAS / E57 scans, ~5e5 m) the system is
    rounding noise in float64 — for Open3D as well (tests/test_oracle.py
    test_icp_offset_conditioning).  Warn; the remedy is to register in a
    re-centred frame (subtract a common origin from both clouds)."""
    import warnings

    mn, mx = src.get_aabb() if hasattr(src, "get_aabb") else (None, None)
    tmn, tmx = tgt.get_aabb() if hasattr(tgt, "get_aabb") else (None, None)
    if mn is None or tmn is None:
        return
    far = max(np.abs(np.asarray(mn)).max(), np.abs(np.asarray(mx)).max(), np.abs(np.asarray(tmn)).max(),
              np.abs(np.asarray(tmx)).max())
    ext = max(float(np.max(np.asarray(mx) - np.asarray(mn))), float(np.max(np.asarray(tmx) - np.asarray(tmn))), 1e-12)
    if far / ext > 1e3:
        warnings.warn(f"registration_icp: the clouds lie {far:.3g} from the origin at an extent of {ext:.3g}; "
                      "point-to-plane ICP on raw coordinates that far out is ill-conditioned in float64 (Open3D's "
                      "too): register in a re-centred frame", RuntimeWarning, stacklevel=3)


class PointCloudBase:
    COLOR_CHART = np.asarray([[230, 0, 18], [243, 152, 0], [252, 200, 0], [143, 195, 31], [0, 153, 68],
                              [0, 160, 233], [29, 32, 136], [146, 7, 131], [228, 0, 127]])

    def __init__(self, xyz=None, rgb=None, normals=None, intensity=None, labels=None, row_index=None,
                 column_index=None, e57=None):
        self.e57 = None
        self.intensity = []
        self.labels = []
        self.row_index = []
        self.column_index = []
        self._pts = None        # (N,3) float32 tensor on the device
        self._pts_host = None   # (N,3) float64 exact host copy (when supplied from host)
        self._pts64 = None      # device float64 copy of _pts_host (plane selections), made on demand
        # _wide: SOME float64 value is not float32-representable, so every hot
        # op runs its float64 kernels (o3dx_*_f64) to keep Open3D's float64
        # arithmetic on the exact values.  This is not limited to georeferenced
        # scans: np.random float64 arrays and a cloud after transform() with a
        # general rotation (transform() re-calls set_points) qualify too.  The
        # float64 path is slower (normals ~2-4x) and keeps no
        # voxel table for the normals.  Pass float32 values (or
        # points.astype(np.float32)) to opt into the float32 kernels: Open3D's
        # result on those values is the same either way.
        self._wide = False
        self._normals = None    # (N,3) float32 tensor
        self._colors = None     # (N,3) float32 tensor in [0,1]
        self.pcd_tree = None
        self.scan_No = -1
        self.uuid = uuid.uuid4()

        if isinstance(xyz, PointCloudBase):
            self._copy_from(xyz)
            return
        if xyz is not None and hasattr(xyz, "points") and not isinstance(xyz, (np.ndarray, torch.Tensor)):
            # an open3d.geometry.PointCloud (or anything shaped like one)
            pts = np.asarray(xyz.points)
            normals = np.asarray(xyz.normals) if len(getattr(xyz, "normals", [])) else normals
            rgb = np.asarray(xyz.colors) if len(getattr(xyz, "colors", [])) else rgb
            xyz = pts

        def ok(a):
            return a is not None and len(a) > 0 and np.prod(a.shape) > 0

        if ok(intensity):
            self.set_intensity(intensity)
        if ok(labels):  # accepted but silently dropped by the reference's __init__
            self.set_labels(labels)
        if ok(row_index):
            self.row_index = row_index
        if ok(column_index):
            self.column_index = column_index
        if ok(xyz):
            self.set_points(xyz)
        if ok(normals):
            self.set_normals(normals)
        if ok(rgb):
            rgb = _as_np(rgb)
            if rgb.max() > 1.0 or rgb.min() < 0.0:   # reference PointCloud.py:36-40
                rgb = rgb * 1.0
                rgb = (rgb - rgb.min()) / (rgb.max() - rgb.min())
            self.set_rgb(rgb)

    # ----------------------------------------------------------- storage
    def _copy_from(self, other: "PointCloudBase"):
        self._pts = other._pts
        self._pts_host = other._pts_host
        self._pts64 = other._pts64
        self._wide = other._wide
        self._normals = other._normals
        self._colors = other._colors
        self.intensity = other.intensity
        self.labels = other.labels
        self.row_index = other.row_index
        self.column_index = other.column_index

    def _dev_points(self) -> torch.Tensor:
        """float32 (N,3) device tensor — the kernels' input."""
        if self._pts is None:
            return torch.zeros((0, 3), dtype=torch.float32, device=_device())
        if self._pts.device.type != "cuda" and torch.cuda.is_available():
            self._pts = self._pts.to(_device())
        return self._pts

    def _plane_points(self) -> torch.Tensor:
        """The coordinates the plane selections evaluate: the caller's exact
        float64 values when the cloud came from float64 data (the reference
        computes distance2plane on get_points(), float64: PointCloud.py:
        400-404), else the float32 device points."""
        if self._pts_host is None and self._pts64 is None:
            return self._dev_points()
        if self._pts64 is None or self._pts64.device.type != "cuda":
            src = self._pts_host if self._pts_host is not None else self._pts64
            self._pts64 = torch.as_tensor(src, dtype=torch.float64, device=N.default_device())
        return self._pts64

    def _hot_points(self) -> torch.Tensor:
        """The hot-path kernels' input: the float64 device copy when float32
        cannot hold the cloud's values (the o3dx_*_f64 entry points, Open3D's
        float64 arithmetic), else the float32 device points (identical
        inputs: every float64 value is a float32 value)."""
        return self._plane_points() if self._wide else self._dev_points()

    @staticmethod
    def _to_dev(a, dtype=torch.float32) -> torch.Tensor:
        if isinstance(a, torch.Tensor):
            t = a.detach()
            if t.device.type == "cpu" and torch.cuda.is_available():
                t = t.to(_device())
            return t.to(dtype).contiguous()
        return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=_device())

    def clear(self):
        self.__init__()
        return self

    def size(self) -> int:
        return 0 if self._pts is None else int(self._pts.shape[0])

    def has_points(self) -> bool:
        return self.size() > 0

    def is_empty(self) -> bool:
        return not self.has_points()

    def has_colors(self) -> bool:
        return self._colors is not None and len(self._colors) > 0

    def get_center(self) -> np.ndarray:
        return self.get_points().mean(0) if self.has_points() else np.zeros(3)

    def transform(self, T: np.ndarray):
        """p <- (T @ [p;1])[:3] / w ; normals <- R n (Open3D Geometry3D::Transform)."""
        T = np.asarray(T, np.float64).reshape(4, 4)
        if self.has_points():
            if self._pts_host is not None:
                h = self._pts_host @ T[:3, :3].T + T[:3, 3]  # set_points drops _pts64
                w = self._pts_host @ T[3, :3] + T[3, 3]
                self.set_points(h / w[:, None])
            elif self._pts64 is not None:
                Tt = torch.as_tensor(T, dtype=torch.float64, device=self._pts64.device)
                h = self._pts64 @ Tt[:3, :3].T + Tt[:3, 3]
                w = self._pts64 @ Tt[3, :3] + Tt[3, 3]
                self.set_points(h / w[:, None])
            else:
                Tt = torch.as_tensor(T, dtype=torch.float64, device=self._pts.device)
                p = self._pts.double()
                h = p @ Tt[:3, :3].T + Tt[:3, 3]
                w = p @ Tt[3, :3] + Tt[3, 3]
                self._pts = (h / w[:, None]).float().contiguous()
        if self._normals is not None:
            R = torch.as_tensor(T[:3, :3], dtype=torch.float64, device=self._normals.device)
            self._normals = (self._normals.double() @ R.T).float().contiguous()
        self.pcd_tree = None
        return self

    def translate(self, t: np.ndarray, relative: bool = True):
        t = np.asarray(t, np.float64).reshape(3)
        if not relative:
            t = t - self.get_center()
        T = np.eye(4)
        T[:3, 3] = t
        return self.transform(T)

    def rotate(self, R: np.ndarray, center=None):
        R = np.asarray(R, np.float64).reshape(3, 3)
        c = self.get_center() if center is None else np.asarray(center, np.float64)
        T = np.eye(4)
        T[:3, :3] = R
        T[:3, 3] = c - R @ c
        return self.transform(T)

    # ------------------------------------------------------------ hot path
    def estimate_normals(self, method="default", param=KDTreeSearchParamKNN(30)):
        """Open3D EstimateNormals(param, fast_normal_computation=True) on the GPU
        (reference PointCloud.py:68-73).  Existing normals orient the result."""
        if method == "poisson":
            raise NotImplementedError("orient_normals_consistent_tangent_plane is outside the GPU hot path")
        mode, knn, radius = resolve(param)
        x = self._hot_points()
        prior = self._normals if self.has_normals() else None
        self._normals = ops.estimate_normals(x, mode=mode, knn=knn, radius=radius, prior=prior,
                                             voxel_grid=None if self._wide else self._kept_voxel_grid(x))
        return self

    def _kept_voxel_grid(self, x):
        """The voxel table of the voxel_down_sample that made this cloud, while
        its points are unchanged (same tensor, no in-place writes)."""
        kept = getattr(self, "_voxel_grid", None)
        if kept is None:
            return None
        vg, pts, version = kept
        if x is not pts or pts._version != version or vg.m != x.shape[0]:
            self._voxel_grid = None
            return None
        return vg

    def segment_plane(self, thickness: float = 0.01, ransac_n: int = 3, num_iterations: int = 450,
                      probability: float = 0.99999999, seed=None, samples=None) -> Tuple[List, List[int]]:
        """Open3D SegmentPlane (reference PointCloud.py:75-77) -> ([a,b,c,d], inlier indices)."""
        plane, inl = self._segment_plane_dev(thickness, ransac_n, num_iterations, probability, seed, samples)
        return plane, inl.cpu().numpy().astype(np.int64).tolist()

    def _segment_plane_dev(self, thickness=0.01, ransac_n=3, num_iterations=450, probability=0.99999999, seed=None,
                           samples=None):
        """segment_plane with the inlier indices left on the device (int32)."""
        x = self._hot_points()
        n = x.shape[0]
        if samples is None and n >= ransac_n >= 3 and 0 < probability <= 1:
            samples = ops.ransac_samples(n, ransac_n, num_iterations, _next_seed() if seed is None else seed)
        plane, inl = ops.segment_plane(x, thickness, ransac_n, num_iterations, probability, samples=samples)
        return [float(v) for v in plane], inl

    def get_aabb(self):
        if not self.has_points():
            return np.zeros(3), np.zeros(3)
        if self._pts_host is not None and not torch.cuda.is_available():
            raise RuntimeError("get_aabb needs the ROCm GPU (no CPU path)")
        return ops.aabb(self._hot_points())

    # ---------------------------------------------------------------- has
    def has_rgb(self) -> bool:
        return self.has_points() and self._colors is not None and self.size() == len(self._colors)

    def has_normals(self) -> bool:
        return self.has_points() and self._normals is not None and self.size() == len(self._normals)

    def has_intensity(self) -> bool:
        return self.has_points() and self.size() == len(self.intensity)

    def has_labels(self) -> bool:
        return self.has_points() and self.size() == len(self.labels)

    def has_col_row(self) -> bool:
        return self.has_points() and self.size() == len(self.column_index) == len(self.row_index)

    # ---------------------------------------------------------- set / get
    def set_rgb(self, colors):
        c = colors if isinstance(colors, torch.Tensor) else np.asarray(colors)
        _check3(c, "colors")
        self._colors = self._to_dev(c)
        return self

    def set_points(self, points):
        if isinstance(points, torch.Tensor):
            _check3(points, "points")
            self._pts_host = None
            self._pts64 = None
            self._wide = points.dtype == torch.float64 and not _f32_exact(points)
            if self._wide:  # kept in float64 on the device (get_points returns it)
                self._pts64 = self._to_dev(points, torch.float64)
            self._pts = self._to_dev(points)
        else:
            p = np.asarray(points)
            _check3(p, "points")
            self._pts_host = np.ascontiguousarray(p, dtype=np.float64)
            self._pts64 = None
            self._wide = not _f32_exact(self._pts_host)
            self._pts = self._to_dev(self._pts_host.astype(np.float32))
        self.pcd_tree = None
        return self

    def set_normals(self, normals):
        nrm = normals if isinstance(normals, torch.Tensor) else np.asarray(normals)
        _check3(nrm, "normals")
        self._normals = self._to_dev(nrm)
        return self

    def set_intensity(self, intensity: np.ndarray):
        assert intensity.shape[1] == 1, "intensity shape must be (n,1)"
        self.intensity = intensity
        return self

    def set_labels(self, labels: np.ndarray):
        assert labels.shape[1] == 1, "labels shape must be (n,1)"
        self.labels = labels
        return self

    def get_points(self) -> np.ndarray:
        if self._pts_host is not None:
            return self._pts_host.copy()
        if self._pts64 is not None:
            return self._pts64.detach().cpu().numpy().copy()
        if self._pts is None:
            return np.zeros((0, 3))
        return self._pts.detach().cpu().numpy().astype(np.float64)

    def get_colors(self) -> np.ndarray:
        return np.zeros((0, 3)) if self._colors is None else self._colors.cpu().numpy().astype(np.float64)

    def get_normals(self) -> np.ndarray:
        return np.zeros((0, 3)) if self._normals is None else self._normals.cpu().numpy().astype(np.float64)

    def get_intensity(self):
        return self.intensity

    def get_labels(self):
        return self.labels

    def get_col_row(self):
        return (self.column_index, self.row_index)

    def set_uniform_label(self, label: int):
        self.labels = np.ones((self.size(), 1), dtype=int) * label
        return self

    def set_uniform_intensity(self, intensity: float):
        self.set_intensity(np.ones((self.size(), 1), dtype=int) * intensity)
        return self

    # ------------------------------------------------------------- KD-tree
    def calc_KDtree(self):
        self.pcd_tree = KDTreeGrid(self)
        return self.pcd_tree

    def get_KDtree(self):
        if self.pcd_tree is None:
            self.calc_KDtree()
        return self.pcd_tree

    def get_points_by_knn(self, point_idx: int, max_nn: int = 1000000):
        q = self.get_points()[point_idx]
        return self.get_KDtree().search_knn_vector_3d(q, max_nn)

    def get_points_radius(self, point_idx: int, search_radius: float = 30.0):
        q = self.get_points()[point_idx]
        return self.get_KDtree().search_radius_vector_3d(q, search_radius)

    # ------------------------------------------------------------------ IO
    def read_pcd(self, filename: str, format: str = "auto", remove_nan_points: bool = False,
                 remove_infinite_points: bool = False, print_progress: bool = False):
        ext = (os.path.splitext(filename)[1].lstrip(".") if format == "auto" else format).lower()
        nrm = col = None
        if ext == "pcd" and torch.cuda.is_available():
            # decoded on the GPU into the device arrays the cloud keeps
            pts, nrm, col = pcd_io.read_pcd_device(filename, _device(), remove_nan_points, remove_infinite_points)
        elif ext == "pcd":
            pts, nrm, col = pcd_io.read_pcd(filename, remove_nan_points, remove_infinite_points)
        elif ext == "npy":
            pts = np.load(filename, allow_pickle=False).reshape(-1, 3).astype(np.float64)
        elif ext in ("xyz", "xyzn", "xyzrgb", "pts", "txt"):
            a = np.loadtxt(filename, ndmin=2)
            pts = a[:, :3]
            if ext == "xyzn" and a.shape[1] >= 6:
                nrm = a[:, 3:6]
            if ext == "xyzrgb" and a.shape[1] >= 6:
                col = a[:, 3:6]
        else:
            raise RuntimeError(f"read_pcd: unsupported format {ext!r}")
        if ext != "pcd" and (remove_nan_points or remove_infinite_points):
            keep = np.ones(len(pts), bool)
            if remove_nan_points:
                keep &= ~np.isnan(pts).any(1)
            if remove_infinite_points:
                keep &= ~np.isinf(pts).any(1)
            pts = pts[keep]
            nrm = nrm[keep] if nrm is not None else None
            col = col[keep] if col is not None else None
        return self.__class__(pts, rgb=col, normals=nrm)

    def save_pcd(self, filename: str, write_ascii: bool = False, compressed: bool = False,
                 print_progress: bool = False):
        return pcd_io.write_pcd(filename, self.get_points(), self.get_normals() if self.has_normals() else None,
                                self.get_colors() if self.has_rgb() else None, write_ascii=write_ascii)

    def draw(self, geos=[], point_size: int = 1, centralize: bool = False):
        raise NotImplementedError("visualisation is outside the GPU hot path (reference PointCloud.py:172-178)")


class PointCloudSelections(PointCloudBase):

    def clone(self, invert: bool = False):
        return self._select_by_idx(np.arange(self.size()), invert=invert)

    def _select_by_idx(self, indices, invert: bool = False):
        """Boolean-mask gather of every per-point attribute; output keeps ascending
        original index order (reference PointCloud.py:185-204)."""
        res = self.__class__()
        n = self.size()
        if isinstance(indices, torch.Tensor):
            dev = self._pts.device if self._pts is not None else indices.device
            mask = torch.zeros(n, dtype=torch.bool, device=dev)
            if indices.numel():
                mask[indices.to(dev).long()] = True
        else:
            idx = np.asarray(indices, dtype=np.int64).reshape(-1)
            mask = torch.zeros(n, dtype=torch.bool, device=self._pts.device if self._pts is not None else "cpu")
            if idx.size:
                mask[torch.as_tensor(idx, device=mask.device)] = True
        if invert:
            mask = ~mask
        sel = torch.nonzero(mask).reshape(-1)
        if self.has_points():
            res._pts = self._pts.index_select(0, sel).contiguous()
            res._wide = self._wide
            if self._pts_host is not None:
                res._pts_host = self._pts_host[sel.cpu().numpy()]
            elif self._pts64 is not None:
                res._pts64 = self._pts64.index_select(0, sel.to(self._pts64.device)).contiguous()
        if self.has_rgb():
            res._colors = self._colors.index_select(0, sel.to(self._colors.device)).contiguous()
        if self.has_normals():
            res._normals = self._normals.index_select(0, sel.to(self._normals.device)).contiguous()
        hm = None
        if self.has_intensity() or self.has_labels():
            hm = mask.cpu().numpy()
        if self.has_intensity():
            res.intensity = self.intensity[hm].copy()
        if self.has_labels():
            res.labels = self.labels[hm].copy()
        return res

    def select_by_box(self, center, x_direction, y_direction, z_direction, invert: bool = False):
        dirs = [np.asarray(d, np.float64) / np.linalg.norm(d) for d in (x_direction, y_direction, z_direction)]
        half = [np.linalg.norm(d) ** 2 for d in dirs]
        v = self.get_points() - np.asarray(center)
        inside = np.logical_and.reduce([np.square(v @ d) < h for d, h in zip(dirs, half)])
        return self.select_by_bool(inside, invert=invert)

    def _bool2index(self, bools, invert: bool = False) -> np.ndarray:
        b = np.asarray(bools)
        if invert:
            b = np.logical_not(b)
        return np.where(b)[0]

    def select_by_bool(self, bools, invert: bool = False):
        return self._select_by_idx(self._bool2index(bools), invert=invert)

    def get_index_by_normals(self, comfunc: Callable = lambda ns: np.ones(len(ns), dtype=bool), invert=False):
        if not self.has_normals():
            self.estimate_normals()
        return self._bool2index(comfunc(self.get_normals()), invert=invert)

    def select_by_normals(self, comfunc: Callable = lambda ns: np.ones(len(ns), dtype=bool), invert=False):
        return self._select_by_idx(self.get_index_by_normals(comfunc=comfunc), invert=invert)

    @staticmethod
    def _cosine(model, similarity):
        m = np.asarray(model, np.float64)[:3]
        return lambda v: (v @ m) / (np.linalg.norm(v, axis=1) * np.linalg.norm(m)) >= similarity

    def get_index_by_normals_cosine(self, model, similarity: float = 0.99, invert: bool = False):
        return self.get_index_by_normals(comfunc=self._cosine(model, similarity), invert=invert)

    def select_by_normals_cosine(self, model, similarity: float = 0.99, invert: bool = False):
        return self._select_by_idx(self.get_index_by_normals_cosine(model, similarity), invert=invert)

    def get_index_by_colors(self, comfunc: Callable = lambda rgb: np.ones(len(rgb), dtype=bool), invert=False):
        return self._bool2index(comfunc(self.get_colors()), invert=invert)

    def get_index_by_XYZ(self, comfunc: Callable = lambda X, Y, Z: np.ones(len(X), dtype=bool), invert=False):
        p = self.get_points()
        return self._bool2index(comfunc(p[:, 0], p[:, 1], p[:, 2]), invert=invert)

    def select_by_XYZ(self, comfunc: Callable = lambda X, Y, Z: np.ones(len(X), dtype=bool), invert=False):
        return self._select_by_idx(self.get_index_by_XYZ(comfunc), invert=invert)

    def get_index_by_radius(self, r: float, invert: bool = False):
        return self.get_index_by_XYZ(lambda X, Y, Z: (X ** 2 + Y ** 2 + Z ** 2) ** 0.5 <= r, invert=invert)

    def select_by_radius(self, r: float, invert: bool = False):
        return self._select_by_idx(self.get_index_by_radius(r), invert=invert)

    def get_index_by_plane(self, model, thickness=0.03, invert: bool = False):
        """|s| < thickness (strict), or a (lo, hi) signed band, s the point's
        signed distance to the plane (reference PointCloud.py:278-290), decided
        on the GPU (o3dx_plane_select) in float64; ascending numpy indices."""
        return self._plane_index_dev(model, thickness, invert).cpu().numpy().astype(np.int64)

    def _plane_index_dev(self, model, thickness, invert: bool = False) -> torch.Tensor:
        if not self.has_points():
            return torch.zeros(0, dtype=torch.int32, device=_device())
        return ops.plane_select(self._plane_points(), np.asarray(model, np.float64).reshape(4), thickness, invert)

    def select_by_plane(self, model, thickness=0.03, invert: bool = False):
        # indices stay on the device (reference PointCloud.py:289-290)
        return self._select_by_idx(self._plane_index_dev(model, thickness), invert=invert)

    def get_index_by_aabb(self, aabb_min, aabb_max, invert: bool = False):
        p = self.get_points()
        inside = np.all((p >= np.asarray(aabb_min)) & (p <= np.asarray(aabb_max)), axis=1)
        return self._bool2index(inside, invert=invert)

    def select_by_aabb(self, aabb_min, aabb_max, invert: bool = False):
        return self._select_by_idx(self.get_index_by_aabb(aabb_min, aabb_max), invert=invert)

    def get_index_by_aabb_list(self, aabb_min_max_list, invert: bool = False):
        p = self.get_points()
        inside = np.zeros(len(p), bool)
        for lo, hi in aabb_min_max_list:
            inside |= np.all((p >= np.asarray(lo)) & (p <= np.asarray(hi)), axis=1)
        return self._bool2index(inside, invert=invert)

    def select_by_aabb_list(self, aabb_min_max_list, invert: bool = False):
        return self._select_by_idx(self.get_index_by_aabb_list(aabb_min_max_list), invert=invert)

    def select_by_topN(self, n: int):
        return self._select_by_idx(np.arange(self.size())[:n])


class PointCloudUtility(PointCloudSelections):

    def paint_uniform_color(self, color=(1.0, 0.0, 0.0)):
        self._colors = self._to_dev(np.tile(np.asarray(color, np.float32).reshape(1, 3), (self.size(), 1)))
        return self

    def split_by_labels(self):
        ul = np.unique(self.labels)
        return [self.select_by_bool((self.labels == j).reshape(-1)) for j in ul], ul

    def centralize(self):
        return self.translate(-self.get_center())

    def voxel_down_sample_and_trace(self, voxel_size: float):
        """Open3D VoxelDownSampleAndTrace(vs, AABB min, AABB max) + idxmat.max(1) +
        _select_by_idx (reference PointCloud.py:338-341) on the GPU.

        Returns (cloud of the representatives in ascending index order,
        idxmat (M,8) int32 cubic-id matrix, vec: list of M int arrays).  Row r
        of idxmat / vec is the voxel of representative r; Open3D emits rows in
        its hash-map order instead, which no implementation can reproduce."""
        x = self._hot_points()
        mn, mx = self.get_aabb()
        out = ops.voxel_down_sample(x, voxel_size, mn, mx, with_xyz=False, trace=True)
        rep = out["rep_idx"]
        idxmat = out["cubic_id"].cpu().numpy()
        vop = out["voxel_of_point"].long()
        order = torch.argsort(vop, stable=True)
        counts = torch.bincount(vop, minlength=rep.numel()).cpu().numpy()
        flat = order.to(torch.int32).cpu().numpy()
        vec = np.split(flat, np.cumsum(counts)[:-1]) if rep.numel() else []
        return self._select_by_idx(rep), idxmat, vec

    def voxel_down_sample(self, voxel_size: float):
        """Representatives only (no trace) — the fast path."""
        x = self._hot_points()
        mn, mx = self.get_aabb()
        out = ops.voxel_down_sample(x, voxel_size, mn, mx, with_xyz=False, keep_grid=True)
        res = self._select_by_idx(out["rep_idx"])
        if out["voxel_grid"] is not None and res._pts is not None:
            # estimate_normals on the result reads its search grid off the voxel table
            res._voxel_grid = (out["voxel_grid"], res._pts, res._pts._version)
        return res

    def random_down_sample(self, down_sample_ratio: float = 0.1):
        if down_sample_ratio <= 0 or down_sample_ratio > 1:
            return self.__class__()
        idx = np.arange(self.size())
        np.random.shuffle(idx)
        return self._select_by_idx(idx[: int(len(idx) * down_sample_ratio)])

    def uniform_down_sample(self, down_sample_ratio: float = 0.1):
        if down_sample_ratio <= 0 or down_sample_ratio > 1:
            return self.__class__()
        return self._select_by_idx(np.arange(self.size())[:: int(1 / down_sample_ratio)])

    # scale of the rounding band around the outlier threshold (tests raise it
    # to force the exact sequential re-decision on every call)
    _SOR_BAND_SCALE = 8.0

    def remove_statistical_outlier(self, nb_neighbors: int = 20, std_ratio: float = 2.0,
                                   print_progress: bool = False):
        """Open3D RemoveStatisticalOutliers (reference PointCloud.py:370-372),
        index-exact: per point the mean of sqrt(d2) over its nb_neighbors
        nearest (self included), summed sequentially in ascending-distance
        order on the GPU (float64, the kernel's exact d2); keep points with
        0 < mean < cloud_mean + std_ratio * std (Bessel-corrected).

        Open3D forms cloud_mean and std with sequential std::accumulate /
        std::inner_product over all points in index order.  The GPU reduces
        them in a different order; their difference is bounded (a rounding
        band around the threshold).  When no point's mean lies inside that
        band the GPU decision is Open3D's; otherwise the two statistics are
        re-formed in Open3D's sequential order on the host (np.add.accumulate)
        and every point is decided against that threshold."""
        if nb_neighbors < 1 or std_ratio <= 0:
            raise RuntimeError("Illegal input parameters, the number of neighbors and standard deviation "
                               "ratio must be positive.")
        if not self.has_points():
            return self.__class__(), []
        x = self._hot_points()
        idx, d2, cnt = ops.knn_search(x, x, mode=N.SEARCH_KNN, knn=nb_neighbors)
        n = x.shape[0]
        col = torch.arange(d2.shape[1], device=d2.device)
        d = torch.where(col[None, :] < cnt[:, None].long(), torch.sqrt(d2.clamp_min(0)), torch.zeros_like(d2))
        acc = torch.zeros(n, dtype=torch.float64, device=d2.device)
        for j in range(d.shape[1]):  # std::accumulate order: ascending distance
            acc = acc + d[:, j]
        valid = cnt > 0
        avg = torch.where(valid, acc / cnt.clamp_min(1).double(), torch.full_like(acc, -1.0))
        nv = int(valid.sum().item())
        if nv == 0:
            return self.__class__(), []
        pos = avg > 0
        S = float(torch.where(pos, avg, torch.zeros_like(avg)).sum().item())
        m = S / nv
        sq = float(torch.where(pos, (avg - m) * (avg - m), torch.zeros_like(avg)).sum().item())
        std = float(np.sqrt(sq / (nv - 1))) if nv > 1 else float("nan")
        thr = m + std_ratio * std
        # |GPU order - sequential order| bounds (first order, n-term sums)
        E = (n + 4) * np.ldexp(1.0, -53)
        dm = 2.0 * E * m
        dsq = 2.0 * E * sq + 2.0 * dm * np.sqrt(max(n, 1) * sq)
        dstd = (std * (dsq / (2.0 * sq) + E)) if sq > 0 and np.isfinite(std) else 2.0 * np.sqrt(dsq / max(nv - 1, 1))
        band = self._SOR_BAND_SCALE * (dm + std_ratio * dstd) + abs(thr) * np.ldexp(1.0, -50)
        near = int((pos & ((avg - thr).abs() <= band)).sum().item()) if np.isfinite(thr) else 0
        if near == 0:
            keep = torch.nonzero(pos & (avg < thr)).reshape(-1)
        else:
            a = avg.cpu().numpy()
            keep = torch.from_numpy(_sor_keep_sequential(a, nv, std_ratio)).to(x.device)
        kept = keep.cpu().numpy().tolist()
        return self._select_by_idx(keep), kept

    def merge_pcds(self, raw_pcds, rgb: bool = False, intensity: bool = False, normals: bool = False,
                   labels: bool = False):
        pcds = [p if isinstance(p, PointCloudBase) else self.__class__(p) for p in raw_pcds]
        res = self.__class__(np.vstack([p.get_points() for p in pcds]))
        if rgb:
            res.set_rgb(np.vstack([p.get_colors() if p.has_colors() else np.ones((p.size(), 3)) for p in pcds]))
        if normals:
            for p in pcds:
                if not p.has_normals():
                    p.estimate_normals()
            res.set_normals(np.vstack([p.get_normals() for p in pcds]))
        if intensity:
            res.set_intensity(np.vstack([p.get_intensity() if p.has_intensity()
                                         else p.set_uniform_intensity(0).get_intensity() for p in pcds]))
        if labels:
            res.labels = np.vstack([p.get_labels() if p.has_labels() else p.set_uniform_label(0).get_labels()
                                    for p in pcds])
        return res

    def append_pcd(self, pcd, rgb=False, intensity=False, normals=False, labels=False):
        return self.merge_pcds([self, pcd], rgb=rgb, intensity=intensity, normals=normals, labels=labels)

    def distance2plane(self, plane) -> np.ndarray:
        """Signed float64 distance to the plane (reference PointCloud.py:400-404),
        computed on the GPU in numpy's order ((x*a + y*b) + z*c + d) / |abc|, on
        the caller's float64 coordinates when the cloud holds them."""
        if not self.has_points():
            return np.zeros(0)
        return ops.plane_distance(self._plane_points(), np.asarray(plane, np.float64).reshape(4)).cpu().numpy()

    def remove_plane_outlier(self, plane_model, thickness: float = 0.03, similarity: float = 0.999,
                             invert: bool = False):
        cand = self.get_index_by_normals_cosine(plane_model, similarity)
        sub = self._select_by_idx(cand)
        on = sub._plane_index_dev(plane_model, thickness).long()
        floor_idx = torch.as_tensor(np.asarray(cand, np.int64), device=on.device)[on]
        return self._select_by_idx(floor_idx), floor_idx.cpu().numpy()

    def project2plane(self, plane):
        plane = np.asarray(plane, np.float64)
        dis = self.distance2plane(plane).reshape(-1, 1) * plane[:3].reshape(1, 3)
        return self.__class__(self.get_points() - dis)

    def seg_plane_by_svd(self):
        p = self.get_points()
        c = p.mean(0)
        _, _, v = np.linalg.svd(p - c)
        a, b, cc = v[-1]
        return a, b, cc, -float((c * v[-1]).sum())


class PointCloud(PointCloudUtility):

    def split_pcd_index(self, nn: int, random: bool = False):
        n = self.size()
        if n <= nn:
            return [np.arange(n)]
        parts = n // nn
        sizes = np.full(parts, nn) + np.asarray([len(a) for a in np.array_split(np.ones(n % nn), parts)])
        r = np.arange(n)
        if random:
            np.random.shuffle(r)
        starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
        return [r[s:s + k] for s, k in zip(starts, sizes)]

    def split_pcd(self, nn: int, random: bool = False):
        if self.size() <= nn:
            return [self]
        return [self._select_by_idx(i) for i in self.split_pcd_index(nn=nn, random=random)]

    def split_by_voxel(self, voxel_size: float = 0.01, random: bool = True, top_n: int = 10):
        """Round-robin one point per voxel into up to top_n clouds (reference
        PointCloud.py:735-757), using the GPU voxel trace."""
        lists = [np.asarray(v).tolist() for v in self.voxel_down_sample_and_trace(voxel_size)[2]]
        if random:
            for v in lists:
                np.random.shuffle(v)
        pcds, taken = [], []
        while True:
            pick = [v.pop() for v in lists if len(v) > 0]
            if not pick:
                break
            taken += pick
            pcds.append(self._select_by_idx(pick))
            if len(pcds) >= top_n:
                break
        return pcds, self._select_by_idx(taken, True)

    def rotation_matrix_from_vectors(self, vec1, vec2) -> np.ndarray:
        a = (np.asarray(vec1, np.float64) / np.linalg.norm(vec1)).reshape(3)
        b = (np.asarray(vec2, np.float64) / np.linalg.norm(vec2)).reshape(3)
        v = np.cross(a, b)
        if not any(v):
            return np.eye(3)
        c = np.dot(a, b)
        s = np.linalg.norm(v)
        K = np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])
        return np.eye(3) + K + K @ K * ((1 - c) / s ** 2)

    def rotate_by_normal(self, plane):
        a, b, c, d = plane
        T = np.eye(4)
        T[2, 3] = d
        T[:3, :3] = self.rotation_matrix_from_vectors(np.array([a, b, c]) / np.linalg.norm([a, b, c]), (0, 0, 1))
        self.transform(T)
        return self, T

    rotate_to_plane = rotate_by_normal

    def seg_planes(self, thickness: float = 0.01, ransac_n: int = 3, num_iterations: int = 450,
                   top_n: float = 10e9, minPointsRatio: float = 0.1):
        """Repeated GPU segment_plane on the remaining outliers (reference
        PointCloud.py:941-985) -> (planes, pcds (inliers..., outliers), aabbs)."""
        rest, planes, pcds, aabbs = self, [], [], []
        raw = self.size()
        if raw < ransac_n:
            return planes, pcds, aabbs
        while rest.size() / raw > minPointsRatio:
            try:
                # the inliers stay on the device between the rounds
                plane, inl = rest._segment_plane_dev(thickness, ransac_n, num_iterations)
            except RuntimeError as e:
                print(e)
                break
            planes.append(plane)
            inliers = rest._select_by_idx(inl)
            pcds.append(inliers)
            aabbs.append(inliers.get_aabb())
            rest = rest._select_by_idx(inl, True)
            if len(planes) > top_n:
                break
        pcds.append(rest)
        aabbs.append(rest.get_aabb())
        return planes, pcds, aabbs

    def registration_icp(self, target: "PointCloudBase", max_correspondence_distance: float, init=None,
                         max_iteration: int = 30, relative_fitness: float = 1e-6, relative_rmse: float = 1e-6):
        """Point-to-plane ICP of self onto target (Open3D registration_icp with
        TransformationEstimationPointToPlane), on the GPU.  North-star op; the
        reference has no ICP."""
        if not target.has_normals():
            raise RuntimeError("TransformationEstimationPointToPlane and TransformationEstimationColoredICP "
                               "require pre-computed normal vectors for target PointCloud.")
        if max_correspondence_distance <= 0.0:
            raise RuntimeError("Invalid max_correspondence_distance.")
        wide = self._wide or target._wide
        src = self._plane_points() if wide else self._dev_points()
        tgt = target._plane_points() if wide else target._dev_points()
        if wide:
            _warn_offset_icp(self, target)
        r = ops.registration_icp(src, tgt, target._normals,
                                 max_correspondence_distance, init, max_iteration, relative_fitness, relative_rmse)
        return RegistrationResult(r["transformation"], r["fitness"], r["inlier_rmse"],
                                  r["correspondence_set"].cpu().numpy().astype(np.int64))
