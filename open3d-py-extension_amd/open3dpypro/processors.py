"""Processors — drop-in for /root/reference/open3dpypro/processors.py (hot-path
operators + the glue that feeds them), and the pipeline runner.

Device dispatch keeps the reference's rule: a mat whose info.device is 'cpu'
takes the numpy branch, 'cuda' in device takes the tensor branch (ROCm torch
reports 'cuda:N').  Both branches run the same MI355X kernels (Open3D
semantics); the numpy branch uploads, computes and downloads.  There is no
CPU compute path.  uuid prefixes equal class names so dumps/loads round-trip
(reference processors.py:1045-1052).
"""
from __future__ import annotations

import json
import multiprocessing
from typing import Any, Callable, List, Optional, Union

import numpy as np
import torch

from . import ops
from . import _native as N
from .PointCloud import PointCloud, PointCloudBase, _f32_exact, _next_seed
from .PointCloudMat import PointCloudMat, PointCloudMatInfo, PointCloudMatProcessor, ShapeType

logger = print


def _gpu() -> torch.device:
    return N.default_device()


def _to_gpu(a) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a if a.device.type == "cuda" else a.to(_gpu())
    return torch.from_numpy(np.ascontiguousarray(a)).to(_gpu())


def _xyz(a) -> torch.Tensor:
    """The mat's coordinates for the kernels: float32, or float64 when the
    mat holds float64 values float32 cannot represent (the float64 boundary:
    the reference's CPU models hand those to Open3D's float64 storage)."""
    t = _to_gpu(a)[:, :3]
    if t.dtype == torch.float64 and not _f32_exact(t):
        return t.contiguous()
    return t.float().contiguous()


class Processors:
    class DoingNothing(PointCloudMatProcessor):
        title: str = "doing_nothing"

        def validate_pcd(self, pcd_idx, pcd):
            pass

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            return pcds_data

    class BackUp(PointCloudMatProcessor):
        title: str = "output_backup"
        device: str = ""
        save_results_to_meta: bool = True
        _backup_mats: List[Any] = []

        def validate_pcd(self, idx, pcd):
            self.init_common_utility_methods(idx, pcd.is_ndarray())

        def get_backup_mats(self) -> List[PointCloudMat]:
            return [PointCloudMat(shape_type=m.info.shape_type).build(d)
                    for d, m in zip(self._backup_mats, self.input_mats)]

        def forward_raw(self, pcds_data, pcds_info=None, meta=None):
            self._backup_mats = []
            for i, p in enumerate(pcds_data):
                c = self._mat_funcs[i].copy_mat(p)
                if self.device == "cpu":
                    c = self._mat_funcs[i].to_numpy(c)
                self._backup_mats.append(c)
            return pcds_data

    class NumpyToTorch(PointCloudMatProcessor):
        """H2D with round-robin device placement (reference processors.py:188-209)."""
        title: str = "numpy_to_torch"

        def model_post_init(self, context):
            self.devices_info(gpu=True, multi_gpu=-1)
            return super().model_post_init(context)

        def validate_pcd(self, pcd_idx, pcd: PointCloudMat):
            pcd.require_ndarray()

        def forward_raw(self, pcds_data, pcds_info=None, meta=None):
            if self.num_gpus == 0:
                raise RuntimeError("NumpyToTorch: no ROCm GPU visible")
            return [torch.from_numpy(np.ascontiguousarray(p)).to(self.num_devices[i % self.num_gpus])
                    .type(PointCloudMatInfo.torch_pcd_dtype()) for i, p in enumerate(pcds_data)]

    class TorchToNumpy(PointCloudMatProcessor):
        title: str = "torch_to_numpy"

        def validate_pcd(self, pcd_idx, pcd: PointCloudMat):
            pcd.require_torch_float()

        def forward_raw(self, pcds_data, pcds_info=None, meta=None):
            return [p.detach().cpu().numpy() for p in pcds_data]

    class CPUNormals(PointCloudMatProcessor):
        """numpy in/out normals (reference processors.py:228-249): Open3D
        EstimateNormals(KNN 30) — computed on the GPU — hstacked as float64
        (the reference's np.hstack promotes to float64), ShapeType + 'N'."""
        title: str = "cpu_calc_normals"
        knn: int = 30
        input_shape_types: List[ShapeType] = []

        def validate_pcd(self, pcd_idx, pcd: PointCloudMat):
            pcd.require_ndarray()
            if pcd_idx == 0:
                self.input_shape_types = []
            self.input_shape_types.append(pcd.info.shape_type)

        def build_out_mats(self, validated_pcds, converted_raw_pcds):
            self.out_mats = [PointCloudMat(shape_type=o.info.shape_type.add_normals()).build(p)
                             for o, p in zip(validated_pcds, converted_raw_pcds)]
            return self.out_mats

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            res = []
            for i, p in enumerate(pcds_data):
                if self.input_shape_types[i].contains_normals():
                    res.append(p)  # already has normals (the reference drops such inputs)
                    continue
                ns = ops.estimate_normals(_xyz(p), knn=self.knn).cpu().numpy().astype(np.float64)
                res.append(np.hstack([p, ns]))
            return res

    class TorchNormals(PointCloudMatProcessor):
        """tensor in/out normals (reference processors.py:251-318; k=16).  The
        reference's cdist+SVD is O(N^2); here the grid kNN + FastEigen3x3
        kernel gives the same axis (sign: Open3D's convention, the reference
        SVD sign is arbitrary).  N < 3 raises ValueError as in the reference."""
        title: str = "torch_calc_normals"
        k: int = 16
        input_shape_types: List[ShapeType] = []

        def validate_pcd(self, pcd_idx, pcd: PointCloudMat):
            pcd.require_torch_float()
            if pcd_idx == 0:
                self.input_shape_types = []
            self.input_shape_types.append(pcd.info.shape_type)

        def build_out_mats(self, validated_pcds, converted_raw_pcds):
            self.out_mats = [PointCloudMat(shape_type=o.info.shape_type.add_normals()).build(p)
                             for o, p in zip(validated_pcds, converted_raw_pcds)]
            return self.out_mats

        def estimate_normals_torch(self, pcd: torch.Tensor, k: int = 16) -> torch.Tensor:
            k = min(k, pcd.shape[0])
            if k < 3:
                raise ValueError(f"Cannot compute normals with k={k}. Need at least 3 neighbors.")
            return ops.estimate_normals(_xyz(pcd), knn=k).to(pcd.device)

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            res = []
            for i, p in enumerate(pcds_data):
                if len(p) == 0:
                    res.append(p.reshape(-1, p.shape[1] + 3))
                    continue
                if self.input_shape_types[i].contains_normals():
                    res.append(p)
                    continue
                res.append(torch.hstack([p, self.estimate_normals_torch(p, self.k).to(p.dtype)]))
            return res

    class RandomSample(PointCloudMatProcessor):
        title: str = "rand_sample"
        n_samples: int = 1000
        copy_pcd: bool = False

        def validate_pcd(self, pcd_idx, pcd):
            if pcd.is_torch_tensor():
                pcd.require_torch_float()
                self.devices_info()
            else:
                pcd.require_ndarray()

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            res = []
            for p in pcds_data:
                if len(p) > self.n_samples:
                    if isinstance(p, torch.Tensor):
                        p = p[torch.randint(0, len(p), (self.n_samples,), device=p.device)]
                        p = p.clone() if self.copy_pcd else p
                    else:
                        p = p[np.random.randint(0, len(p), (self.n_samples,))]
                        p = p.copy() if self.copy_pcd else p
                res.append(p)
            return res

    class RadiusSelection(PointCloudMatProcessor):
        title: str = "radius_selection"
        radius: float = 5.0

        def validate_pcd(self, pcd_idx, pcd):
            if pcd.is_torch_tensor():
                pcd.require_torch_float()
            else:
                pcd.require_ndarray()

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            res = []
            for p in pcds_data:
                if isinstance(p, torch.Tensor):
                    res.append(p[p[:, :3].norm(dim=1) <= self.radius])
                else:  # reference: PointCloud(xyz).select_by_radius(r).get_points() -> float64 xyz
                    q = np.asarray(p[:, :3], np.float64)
                    res.append(q[(q[:, 0] ** 2 + q[:, 1] ** 2 + q[:, 2] ** 2) ** 0.5 <= self.radius])
            return res

    class VoxelDownsample(PointCloudMatProcessor):
        """Open3D voxel_down_sample_and_trace + idxmat.max(1) semantics on both
        branches (reference processors.py:418-474): grid anchored at the
        cloud's min bound, representative = largest index per voxel, rows in
        ascending index order, every column of the input kept."""
        title: str = "voxel_sample"
        voxel_size: float = 0.1

        def validate_pcd(self, pcd_idx, pcd):
            if pcd.is_torch_tensor():
                pcd.require_torch_float()
                self.devices_info()
            else:
                pcd.require_ndarray()

        def downsample(self, p):
            rep = ops.voxel_down_sample(_xyz(p), self.voxel_size, with_xyz=False)["rep_idx"]
            if isinstance(p, torch.Tensor):
                return p.index_select(0, rep.to(p.device).long())
            return p[rep.cpu().numpy()]

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            return [self.downsample(p) for p in pcds_data]

    class RemoveStatisticalOutlier(PointCloudMatProcessor):
        title: str = "remove_statistical_outlier"
        nb_neighbors: int = 20
        std_ratio: float = 2.0
        print_progress: bool = False

        def validate_pcd(self, pcd_idx, pcd):
            if not pcd.is_torch_tensor():
                pcd.require_ndarray()

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            res = []
            for p in pcds_data:
                _, keep = PointCloud(_xyz(p)).remove_statistical_outlier(self.nb_neighbors, self.std_ratio)
                res.append(p[torch.as_tensor(keep, device=p.device).long()] if isinstance(p, torch.Tensor)
                           else p[np.asarray(keep, np.int64)])
            return res

    class PlaneDetection(PointCloudMatProcessor):
        """RANSAC plane per cloud (reference processors.py:502-699) with Open3D
        SegmentPlane semantics on both branches; the plane is flipped so that
        d >= 0 (the reference's 'towards the sensor' flip) and blended into
        best_planes by EMA(alpha); meta[uuid] = best_planes."""
        title: str = "plane_detection"
        distance_threshold: float = 0.01
        arange: bool = False
        best_planes: List[List[float]] = []
        alpha: float = 0.0
        num_iterations: int = 512
        num_iteration_batch: int = 256
        voxel_size: float = 0.0
        z_lower: Optional[float] = None
        z_upper: Optional[float] = None
        seed: Optional[int] = None
        _vd: Any = None

        def model_post_init(self, context):
            if self.voxel_size > 0.0:
                self._vd = Processors.VoxelDownsample(voxel_size=self.voxel_size)
            return super().model_post_init(context)

        def validate_pcd(self, pcd_idx, pcd):
            if pcd.is_torch_tensor():
                pcd.require_torch_float()
                self.devices_info()
            else:
                pcd.require_ndarray()
            if pcd_idx == 0:
                self.best_planes = []
            self.best_planes.append([0.0, 0.0, 0.0, 0.0])

        def validate(self, pcds, meta={}, run=True):
            if self._vd:
                self._vd.validate(pcds, meta, run=False)
            return super().validate(pcds, meta, run)

        def detect(self, p) -> np.ndarray:
            x = _xyz(p)
            if self.z_lower is not None and self.z_upper is not None:
                x = x[(x[:, 2] > self.z_lower) & (x[:, 2] < self.z_upper)].contiguous()
            n = x.shape[0]
            seed = _next_seed() if self.seed is None else self.seed
            samples = ops.ransac_samples(n, 3, self.num_iterations, seed) if n >= 3 else None
            plane, _ = ops.segment_plane(x, self.distance_threshold, 3, self.num_iterations, samples=samples)
            # reference processors.py:640-650: point_on_plane = -d n; flip if n.(0 - p) < 0
            if np.dot(plane[:3], plane[3] * plane[:3]) < 0:
                plane = -plane
            return plane

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            if self._vd:
                pcds_data = self._vd.forward_raw(pcds_data)
            for i, p in enumerate(pcds_data):
                plane = self.detect(p)
                self.best_planes[i] = (np.asarray(self.best_planes[i]) * (1.0 - self.alpha) +
                                       plane * self.alpha).tolist()
            meta[self.uuid] = self.best_planes
            return pcds_data

    class PlaneNormalize(PointCloudMatProcessor):
        """Rotate each cloud so the detected plane (meta[detection_uuid]) becomes
        z = 0 (reference processors.py:701-759).  T is built the reference's
        way, in the data's dtype on the data's device (rotation_matrix_from_
        vectors, including its quirk: normals within 1e-6 of parallel OR
        anti-parallel to z give the identity, :713-714), and applied as the
        homogeneous product (T @ [xyz | 1]^T)^T, so the output equals the
        reference's bit for bit."""
        title: str = "plane_normalize"
        detection_uuid: str
        filter_pcd: bool = False

        def validate_pcd(self, idx, pcd):
            self.init_common_utility_methods(idx, pcd.is_ndarray())

        def rotation_matrix_from_vectors(self, vec1, vec2, device=None, i=0):
            f = self._mat_funcs[i]
            a = vec1 / f.norm(vec1)
            b = vec2 / f.norm(vec2)
            v = f.cross(a, b)
            if f.norm(v) < 1e-6:
                return f.eye(3, dtype=a.dtype, device=device)
            c = f.dot(a, b)
            s = f.norm(v)
            kmat = f.mat([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]], dtype=a.dtype, device=device)
            return f.eye(3, dtype=a.dtype, device=device) + kmat + f.matmul(kmat, kmat) * ((1 - c) / (s ** 2))

        def rotate_to_plane(self, pcd_data, plane, device=None, i=0):
            f = self._mat_funcs[i]
            a, b, c, d = plane
            xyz = pcd_data[:, :3]
            normal = f.mat([a, b, c], dtype=pcd_data.dtype, device=device)
            z_axis = f.mat([0, 0, 1], dtype=pcd_data.dtype, device=device)
            R = self.rotation_matrix_from_vectors(normal, z_axis, device, i)
            point_on_plane = -d * normal / f.dot(normal, normal)
            t = -f.matmul(R, point_on_plane)
            T = f.eye(4, dtype=pcd_data.dtype, device=device)
            T[:3, :3] = R
            T[:3, 3] = t
            ones_row = f.ones((pcd_data.shape[0], 1), dtype=pcd_data.dtype, device=device)
            homo = f.hstack([xyz, ones_row])
            return f.matmul(T, homo.T).T[:, :3], T

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            planes = meta[self.detection_uuid]
            self.forward_T = []
            res = []
            for i, p in enumerate(pcds_data):
                device = p.device if hasattr(p, "device") else None
                xyz, T = self.rotate_to_plane(p, planes[i], device=device, i=i)
                res.append(self._mat_funcs[i].hstack([xyz, p[:, 3:]]) if p.shape[1] > 3 else xyz)
                self.forward_T.append(self._mat_funcs[i].to_numpy(T).tolist())
            return res

    class ICP(PointCloudMatProcessor):
        """Point-to-plane ICP of input 0 (source) onto input 1 (target, must
        carry normals: ShapeType ...N).  Output: the transformed source;
        meta[uuid] = {'transformation', 'fitness', 'inlier_rmse'}.  North-star
        op — the reference has no ICP."""
        title: str = "icp_point_to_plane"
        max_correspondence_distance: float = 0.02
        max_iteration: int = 30
        relative_fitness: float = 1e-6
        relative_rmse: float = 1e-6
        init: Optional[List[List[float]]] = None
        result: dict = {}

        def validate_pcd(self, pcd_idx, pcd):
            if pcd_idx == 1 and not pcd.info.shape_type.contains_normals():
                raise TypeError("ICP target must carry normals (ShapeType ending in 'N')")

        def build_out_mats(self, validated_pcds, converted_raw_pcds):
            self.out_mats = [PointCloudMat(shape_type=validated_pcds[0].info.shape_type).build(converted_raw_pcds[0])]
            return self.out_mats

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            src, tgt = pcds_data[0], pcds_data[1]
            st = pcds_info[1].shape_type
            ncol = {ShapeType.XYZN: 3, ShapeType.XYZRGBN: 6, ShapeType.XYZiN: 4, ShapeType.XYZRGBiN: 7}[st]
            tn = _to_gpu(tgt)[:, ncol:ncol + 3].float().contiguous()
            r = ops.registration_icp(_xyz(src), _xyz(tgt), tn, self.max_correspondence_distance, self.init,
                                     self.max_iteration, self.relative_fitness, self.relative_rmse,
                                     return_corr=False)
            T = r["transformation"]
            self.result = {"transformation": T.tolist(), "fitness": r["fitness"], "inlier_rmse": r["inlier_rmse"]}
            meta[self.uuid] = self.result
            if isinstance(src, torch.Tensor):
                Tt = torch.as_tensor(T, dtype=torch.float64, device=src.device)
                xyz = (src[:, :3].double() @ Tt[:3, :3].T + Tt[:3, 3]).to(src.dtype)
                out = torch.hstack([xyz, src[:, 3:]]) if src.shape[1] > 3 else xyz
            else:
                xyz = (src[:, :3].astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(src.dtype)
                out = np.hstack([xyz, src[:, 3:]]) if src.shape[1] > 3 else xyz
            return [out]

    class Lambda(PointCloudMatProcessor):
        title: str = "lambda"
        out_shape_types: List[ShapeType] = []
        _forward_raw: Optional[Callable] = None

        def validate_pcd(self, idx, pcd):
            self.init_common_utility_methods(idx, pcd.is_ndarray())

        def build_out_mats(self, validated_pcds, converted_raw_pcds):
            if not self.out_shape_types:
                return super().build_out_mats(validated_pcds, converted_raw_pcds)
            self.out_mats = [PointCloudMat(shape_type=s).build(p)
                             for s, p in zip(self.out_shape_types, converted_raw_pcds)]
            return self.out_mats

        def forward_raw(self, pcds_data, pcds_info=[], meta={}):
            if self._forward_raw is None:
                raise NotImplementedError("forward_raw function is not set")
            return self._forward_raw(pcds_data, pcds_info, meta)


class PointCloudMatProcessors:
    """Pipeline runner (reference processors.py:1043-1098)."""

    @staticmethod
    def dumps(pipes: List[PointCloudMatProcessor]) -> str:
        return json.dumps([p.model_dump(exclude={"input_mats", "out_mats", "meta"}) for p in pipes])

    @staticmethod
    def loads(pipes_json: str) -> List[PointCloudMatProcessor]:
        table = {k: v for k, v in Processors.__dict__.items() if "__" not in k}
        return [table[p["uuid"].split(":")[0]](**p) for p in json.loads(pipes_json)]

    @staticmethod
    def run_once(imgs, meta={}, pipes: List[PointCloudMatProcessor] = [], validate=False):
        fn = None
        try:
            for fn in pipes:
                imgs, meta = (fn.validate if validate else fn)(imgs, meta)
        except Exception as e:
            logger(getattr(fn, "uuid", "?"), e)
            raise
        return imgs, meta

    @staticmethod
    def run(gen, pipes: Union[str, List[PointCloudMatProcessor]] = [], meta={}, validate_once=False):
        if isinstance(pipes, str):
            pipes = PointCloudMatProcessors.loads(pipes)
        for imgs in gen:
            PointCloudMatProcessors.run_once(imgs, meta, pipes, validate_once)
            if validate_once:
                return

    @staticmethod
    def validate_once(gen, pipes: List[PointCloudMatProcessor] = []):
        PointCloudMatProcessors.run(gen, pipes, validate_once=True)

    @staticmethod
    def worker(pipes_serialized):
        pipes = PointCloudMatProcessors.loads(pipes_serialized)
        imgs, meta = [], {}
        while True:
            for fn in pipes:
                imgs, meta = fn(imgs, meta)

    @staticmethod
    def run_async(pipes: Union[str, List[PointCloudMatProcessor]]):
        ser = pipes if isinstance(pipes, str) else PointCloudMatProcessors.dumps(pipes)
        p = multiprocessing.Process(target=PointCloudMatProcessors.worker, args=(ser,))
        p.start()
        return p
