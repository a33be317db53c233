"""Data model + operator contract of the processor pipeline — drop-in for
/root/reference/open3dpypro/PointCloudMat.py (ShapeType, PointCloudMatInfo,
PointCloudMat, MatOps, PointCloudMatProcessor).

Kept: field names, defaults, validation errors (TypeError / ValueError), the
1->1 / 1->many / many->1 out-mat rules and the meta[uuid] contract.  Dropped:
the CPU shared-memory transport (shmIO), which is out of the GPU hot path's
scope; shmIO_mode other than False raises.
"""
from __future__ import annotations

import enum
import uuid as _uuid
from typing import Any, Dict, List, Literal, Optional, Tuple, Union

import numpy as np
import torch
from pydantic import BaseModel, ConfigDict


class DeviceType(str, enum.Enum):
    CPU = "cpu"
    GPU = "gpu"


class ShapeType(str, enum.Enum):
    XYZ = "XYZ"
    XYZRGB = "XYZRGB"
    XYZi = "XYZi"
    XYZiRGB = "XYZiRGB"
    XYZRGBi = "XYZRGBi"
    XYZN = "XYZN"
    XYZRGBN = "XYZRGBN"
    XYZiN = "XYZiN"
    XYZRGBiN = "XYZRGBiN"

    def contains_normals(self) -> bool:
        return self.value.endswith("N")

    def add_normals(self) -> "ShapeType":
        return self if self.contains_normals() else ShapeType(self.value + "N")

    @property
    def dims(self) -> int:
        return SHAPE_DIMS[self]


SHAPE_DIMS = {ShapeType.XYZ: 3, ShapeType.XYZRGB: 6, ShapeType.XYZi: 4, ShapeType.XYZiRGB: 7,
              ShapeType.XYZRGBi: 7, ShapeType.XYZN: 6, ShapeType.XYZRGBN: 9, ShapeType.XYZiN: 7,
              ShapeType.XYZRGBiN: 10}


class ColorDataType(str, enum.Enum):
    Float32Color = "Float32Color"


torch_pcd_dtype = torch.float32
numpy_pcd_dtype = np.float32


class PointCloudMatInfo(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True)
    type: Optional[str] = None
    _dtype: Any = None
    device: str = ""
    shape_type: Optional[ShapeType] = None
    raw_shape: List[int] = []
    N: int = 0
    uuid: str = ""

    @staticmethod
    def torch_pcd_dtype():
        return torch_pcd_dtype

    @staticmethod
    def numpy_pcd_dtype():
        return numpy_pcd_dtype

    def model_post_init(self, context):
        self.uuid = f"{self.__class__.__name__}:{_uuid.uuid4()}"
        return super().model_post_init(context)

    def build(self, pcd_data, shape_type: Optional[ShapeType] = None):
        st = ShapeType(shape_type) if shape_type is not None else self.shape_type
        if isinstance(pcd_data, np.ndarray):
            self.device = "cpu"
        elif isinstance(pcd_data, torch.Tensor):
            self.device = str(pcd_data.device)
        else:
            raise TypeError(f"pcd_data must be np.ndarray or torch.Tensor, got {type(pcd_data)}")
        self.type = type(pcd_data).__name__
        self._dtype = pcd_data.dtype
        if pcd_data.ndim != 2:
            raise ValueError(f"Point cloud data must be 2D (N, D). Got shape: {tuple(pcd_data.shape)}")
        if st not in SHAPE_DIMS:
            raise ValueError(f"Unsupported shape type {st} for point cloud.")
        D = SHAPE_DIMS[st]
        if pcd_data.shape[1] != D:
            raise ValueError(f"Shape type '{st.value}' expects feature dimension {D}, but got "
                             f"{pcd_data.shape[1]}. Full shape: {tuple(pcd_data.shape)}")
        self.shape_type = st
        self.N = int(pcd_data.shape[0])
        self.raw_shape = [int(v) for v in pcd_data.shape]
        return self


class PointCloudMat(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True)
    shape_type: ShapeType
    info: Optional[PointCloudMatInfo] = None
    _pcd_data: Any = None
    shmIO_mode: Literal[False, "writer", "reader"] = False

    def model_post_init(self, context):
        if self.shmIO_mode:
            raise NotImplementedError("shared-memory transport (shmIO) is not part of the GPU build")
        return super().model_post_init(context)

    @staticmethod
    def random(shape_type, num_points: int = 1000, lib: str = "np", device: str = "cpu"):
        st = ShapeType(shape_type)
        D = SHAPE_DIMS[st]
        if lib == "np":
            data = np.random.rand(num_points, D).astype(numpy_pcd_dtype)
        elif lib == "torch":
            data = torch.rand(num_points, D, dtype=torch_pcd_dtype, device=device)
        else:
            raise TypeError(f"Unsupported library: {lib}")
        return PointCloudMat(shape_type=st).build(data)

    def build(self, pcd_data, info: Optional[PointCloudMatInfo] = None):
        self.info = info or PointCloudMatInfo(shape_type=self.shape_type).build(pcd_data)
        self._pcd_data = pcd_data
        return self

    def _dup(self, data):
        return PointCloudMat(shape_type=self.info.shape_type if self.info else self.shape_type).build(data)

    def clone(self):
        d = self._pcd_data.copy() if isinstance(self._pcd_data, np.ndarray) else self._pcd_data.clone()
        return PointCloudMat(shape_type=self.shape_type).build(d, self.info.model_copy())

    def copy(self) -> "PointCloudMat":
        if isinstance(self._pcd_data, np.ndarray):
            return self._dup(self._pcd_data.copy())
        if isinstance(self._pcd_data, torch.Tensor):
            return self._dup(self._pcd_data.clone())
        raise TypeError("pcd_data must be np.ndarray or torch.Tensor")

    def zero_clone(self):
        return self._dup(self._pcd_data * 0)

    def random_clone(self):
        n, d = self._pcd_data.shape
        if isinstance(self._pcd_data, np.ndarray):
            return self._dup(np.random.rand(n, d).astype(self._pcd_data.dtype))
        return self._dup(torch.rand(n, d, dtype=self._pcd_data.dtype, device=self._pcd_data.device))

    def build_shmIO(self, shmIO_mode=False, target_mat_info=None):
        if shmIO_mode:
            raise NotImplementedError("shared-memory transport (shmIO) is not part of the GPU build")
        return self

    def release(self):
        pass

    def update_mat(self, pcd_data) -> "PointCloudMat":
        self.info = PointCloudMatInfo(shape_type=self.info.shape_type).build(pcd_data)
        return self.unsafe_update_mat(pcd_data)

    def unsafe_update_mat(self, pcd_data) -> "PointCloudMat":
        self._pcd_data = pcd_data
        return self

    def data(self):
        return self._pcd_data

    def is_ndarray(self) -> bool:
        return isinstance(self._pcd_data, np.ndarray)

    def is_torch_tensor(self) -> bool:
        return isinstance(self._pcd_data, torch.Tensor)

    def require_ndarray(self):
        if not isinstance(self._pcd_data, np.ndarray):
            raise TypeError(f"Expected np.ndarray, got {type(self._pcd_data)}")

    def require_torch_tensor(self):
        if not isinstance(self._pcd_data, torch.Tensor):
            raise TypeError(f"Expected torch.Tensor, got {type(self._pcd_data)}")

    def require_torch_float(self):
        self.require_torch_tensor()
        if self._pcd_data.dtype != torch_pcd_dtype:
            raise TypeError(f"Point cloud data must be {torch_pcd_dtype}. Got {self._pcd_data.dtype}")

    def require_shape_type(self, shape_type: ShapeType):
        if self.info.shape_type != shape_type:
            raise TypeError(f"Expected shape type {ShapeType(shape_type).value}, got {self.info.shape_type.value}")

    def require_shape_types(self, shape_types: List[ShapeType]):
        if self.info.shape_type not in shape_types:
            raise TypeError(f"Expected shape types {shape_types}, got {self.info.shape_type.value}")


class MatOps:
    """Backend-neutral array helpers (reference PointCloudMat.py:269-370)."""
    int32 = np.int32
    uint8 = np.uint8
    float32 = np.float32
    float16 = np.float16


class NumpyMatOps(MatOps):
    def mat(self, pylist, dtype, device=None): return np.array(pylist, dtype=dtype)
    def eye(self, size, dtype, device=None): return np.eye(size, dtype=dtype)
    def ones(self, shape, dtype, device=None): return np.ones(shape, dtype=dtype)
    def zeros(self, shape, dtype, device=None): return np.zeros(shape, dtype=dtype)
    def hstack(self, arrays): return np.hstack(arrays)
    def norm(self, x): return np.linalg.norm(x)
    def dot(self, a, b): return np.dot(a, b)
    def cross(self, a, b, dim=-1): return np.cross(a, b, axis=dim)
    def matmul(self, a, b): return a @ b
    def to_numpy(self, x): return x
    def mean(self, x, dim=0): return np.mean(x, axis=dim)
    def median(self, x, dim=0): return np.median(x, axis=dim)
    def std(self, x, dim=0): return np.std(x, axis=dim)
    def max(self, x, dim=0): return np.max(x, axis=dim)
    def min(self, x, dim=0): return np.min(x, axis=dim)
    def abs(self, x): return np.abs(x)
    def stack(self, xs, dim=0): return np.stack(xs, axis=dim)
    def cat(self, xs, dim=0): return np.concatenate(xs, axis=dim)
    def reshape(self, x, shape): return np.reshape(x, shape)
    def copy_mat(self, x): return x.copy()
    def logical_and(self, a, b): return np.logical_and(a, b)
    def logical_or(self, a, b): return np.logical_or(a, b)
    def clip(self, x, lo, hi): return np.clip(x, lo, hi)
    def astype_int32(self, x): return x.astype(np.int32)
    def astype_uint8(self, x): return x.astype(np.uint8)
    def astype_float32(self, x): return x.astype(np.float32)
    def astype_float16(self, x): return x.astype(np.float16)
    def nonzero(self, x): return np.nonzero(x)


class TorchMatOps(MatOps):
    int32 = torch.int32
    uint8 = torch.uint8
    float32 = torch.float32
    float16 = torch.float16
    def mat(self, pylist, dtype, device=None): return torch.tensor(pylist, dtype=dtype, device=device)
    def eye(self, size, dtype, device=None): return torch.eye(size, dtype=dtype, device=device)
    def ones(self, shape, dtype, device=None): return torch.ones(shape, dtype=dtype, device=device)
    def zeros(self, shape, dtype, device=None): return torch.zeros(shape, dtype=dtype, device=device)
    def hstack(self, arrays): return torch.cat(arrays, dim=1)
    def norm(self, x): return torch.norm(x)
    def dot(self, a, b): return torch.dot(a, b)
    def cross(self, a, b, dim=-1): return torch.cross(a, b, dim=dim)
    def matmul(self, a, b): return torch.matmul(a, b)
    def to_numpy(self, x): return x.detach().cpu().numpy()
    def mean(self, x, dim=0): return torch.mean(x, dim=dim)
    def median(self, x, dim=0): return torch.median(x, dim=dim).values
    def std(self, x, dim=0): return torch.std(x, dim=dim, unbiased=False)
    def max(self, x, dim=0): return torch.max(x, dim=dim).values
    def min(self, x, dim=0): return torch.min(x, dim=dim).values
    def abs(self, x): return torch.abs(x)
    def stack(self, xs, dim=0): return torch.stack(xs, dim=dim)
    def cat(self, xs, dim=0): return torch.cat(xs, dim=dim)
    def reshape(self, x, shape): return x.reshape(shape)
    def copy_mat(self, x): return x.clone()
    def logical_and(self, a, b): return torch.logical_and(a, b)
    def logical_or(self, a, b): return torch.logical_or(a, b)
    def clip(self, x, lo, hi): return torch.clamp(x, min=lo, max=hi)
    def astype_int32(self, x): return x.to(torch.int32)
    def astype_uint8(self, x): return x.to(torch.uint8)
    def astype_float32(self, x): return x.to(torch.float32)
    def astype_float16(self, x): return x.to(torch.float16)
    def nonzero(self, x): return torch.nonzero(x)


class PointCloudMatProcessor(BaseModel):
    """Operator contract (reference PointCloudMat.py:374-545): subclasses
    implement validate_pcd(idx, mat) and forward_raw(datas, infos, meta)."""

    class MetaData(BaseModel):
        model_config = {"arbitrary_types_allowed": True}

    model_config = ConfigDict(arbitrary_types_allowed=True)
    title: str
    uuid: str = ""
    save_results_to_meta: bool = False
    input_mats: List[PointCloudMat] = []
    out_mats: List[PointCloudMat] = []
    meta: dict = {}
    num_devices: List[str] = ["cpu"]
    num_gpus: int = 0
    _enable: bool = True
    forward_T: List[List[List[float]]] = []
    _mat_funcs: List[MatOps] = []

    def init_common_utility_methods(self, idx, is_ndarray=True):
        ops_ = NumpyMatOps() if is_ndarray else TorchMatOps()
        if idx < len(self._mat_funcs):
            self._mat_funcs[idx] = ops_
        else:
            self._mat_funcs.append(ops_)

    def print(self, *args):
        print(f"##############[{self.uuid}]#################")
        print(f"[{self.uuid}]", *args)
        print("############################################")

    def model_post_init(self, context: Any, /) -> None:
        if not self.title:
            self.title = self.__class__.__name__
        if not self.uuid:
            self.uuid = f"{self.__class__.__name__}:{_uuid.uuid4()}"
        self._mat_funcs = []
        for i, m in enumerate(self.input_mats):
            self.init_common_utility_methods(i, m.is_ndarray())
        return super().model_post_init(context)

    def is_enable(self):
        return self._enable

    def on(self):
        self._enable = True

    def off(self):
        self._enable = False

    def devices_info(self, gpu=True, multi_gpu=-1):
        self.num_devices = ["cpu"]
        self.num_gpus = 0
        if gpu and torch.cuda.is_available():
            self.num_gpus = torch.cuda.device_count()
            k = self.num_gpus if (multi_gpu <= 0 or multi_gpu > self.num_gpus) else multi_gpu
            self.num_devices = [f"cuda:{i}" for i in range(k)]
        return self.num_devices

    def validate_pcd(self, idx: int, pcd: PointCloudMat):
        raise NotImplementedError()

    def validate(self, pcds: List[PointCloudMat], meta: Dict = {}, run=True):
        self.input_mats = pcds
        for i, p in enumerate(pcds):
            if p.shmIO_mode:
                raise ValueError(f"pcd shmIO_mode must be False. Got {p.shmIO_mode}")
            self.validate_pcd(i, p)
        self.input_mats = list(pcds)
        self.forward_T = [np.eye(4).tolist() for _ in self.input_mats]
        if run:
            return self(self.input_mats, meta)
        return self.input_mats

    def build_out_mats(self, validated_pcds: List[PointCloudMat], converted_raw_pcds):
        nin, nout = len(validated_pcds), len(converted_raw_pcds)
        if nin == nout:
            st = [v.info.shape_type for v in validated_pcds]
        elif nin == 1 and nout > 1:
            st = [validated_pcds[0].info.shape_type] * nout
        elif nin > 1 and nout == 1:
            kinds = {v.info.shape_type for v in validated_pcds}
            if len(kinds) > 1:
                raise ValueError(f"Shape type mismatch: {kinds}. All PointCloudMats must have the same shape type.")
            st = [kinds.pop()]
        else:
            raise ValueError(f"[{self.uuid}] Length mismatch: {nin} vs {nout}")
        self.out_mats = [PointCloudMat(shape_type=s).build(d) for s, d in zip(st, converted_raw_pcds)]
        return self.out_mats

    def forward_raw(self, pcds: List[Any], pcd_infos: List[PointCloudMatInfo] = [], meta={}) -> List[Any]:
        raise NotImplementedError()

    def forward(self, pcds: List[PointCloudMat], meta: Dict) -> Tuple[List[PointCloudMat], Dict]:
        if not pcds and self.input_mats:
            pcds = self.input_mats
        infos = [p.info for p in pcds]
        datas = [p.data() for p in pcds]
        if self._enable:
            datas = self.forward_raw(datas, infos, meta)
        if len(self.out_mats) == len(datas):
            outs = [self.out_mats[i].unsafe_update_mat(datas[i]) for i in range(len(datas))]
        else:
            outs = self.build_out_mats(self.input_mats, datas)
        self.out_mats = outs
        if self.save_results_to_meta:
            meta[self.uuid] = self
        return outs, meta

    def __call__(self, pcds: List[PointCloudMat], meta: dict = {}):
        return self.forward(pcds, meta)

    def release(self):
        for m in list(self.input_mats) + list(self.out_mats):
            m.release()
