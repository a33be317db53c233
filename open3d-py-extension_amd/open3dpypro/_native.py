"""ctypes binding of libo3dx.so (include/o3dx.h) — the only path to the kernels.

There is deliberately no CPU fallback: if the library or a GPU is missing,
every compute call raises RuntimeError (the exception type Open3D's pybind11
layer raises, which reference callers catch generically, e.g.
/root/reference/open3dpypro/PointCloud.py:964-968).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# O3DX_LIB: another in-tree build of the same library (A/B timing of kernel
# variants in one GPU call; tools/ scripts only)
LIB_PATH = os.environ.get("O3DX_LIB") or os.path.join(_HERE, "_lib", "libo3dx.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "o3dx.h")

SEARCH_KNN, SEARCH_RADIUS, SEARCH_HYBRID = 0, 1, 2
MAX_KNN = 64
ICP_NSUMS = 32
ICP_DESC_LEN = 24  # include/o3dx.h O3DX_ICP_DESC_LEN
PCD_TYPES = {("F", 4): 1, ("F", 8): 2, ("U", 1): 3, ("U", 2): 4, ("U", 4): 5, ("I", 1): 6, ("I", 2): 7,
             ("I", 4): 8}
PCD_RGB = 9

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int
_D = ctypes.c_double
_SZ = ctypes.c_size_t

# name -> (restype, argtypes)
_SIGS = {
    "o3dx_abi_version": (_I32, []),
    "o3dx_last_error": (ctypes.c_char_p, []),
    "o3dx_fx_to_double": (_I32, [_P, _I64, _P]),
    "o3dx_set_kernel_timing": (None, [_I32]),
    "o3dx_reset_kernel_timing": (None, []),
    "o3dx_kernel_timing_filter": (None, [ctypes.c_char_p]),
    "o3dx_kernel_timing": (_I32, [ctypes.c_char_p, _P, _P]),
    "o3dx_set_search_stats": (_I32, [_I32]),
    "o3dx_search_stats": (_I32, [_P]),
    "o3dx_set_debug_neighbors": (_I32, [_P, _I64, _I32]),
    "o3dx_fast_eigen3x3": (_I32, [_P, _I64, _P, _P]),
    "o3dx_libm_probe": (_I32, [_P, _I64, _I32, _P, _P]),
    "o3dx_aabb_workspace_bytes": (_SZ, [_I64]),
    "o3dx_aabb": (_I32, [_P, _I64, _P, _P, _SZ, _P]),
    "o3dx_aabb_device": (_I32, [_P, _I64, _P, _P, _SZ, _P]),
    "o3dx_voxel_workspace_bytes": (_SZ, [_I64]),
    "o3dx_voxel_down_sample": (_I32, [_P, _I64, _P, _P, _D, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_voxel_grid_cells": (_I64, [_I64, _P, _P, _D]),
    "o3dx_voxel_grid_capacity": (_I64, [_I64]),
    "o3dx_voxel_down_sample_grid": (_I32, [_P, _I64, _P, _P, _D, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _SZ, _P]),
    "o3dx_voxel_down_sample_window": (_I32, [_P, _I64, _P, _P, _D, _I64, _I64, _P, _P, _P, _P, _I64, _P, _P, _SZ,
                                              _P]),
    "o3dx_voxel_table_workspace_bytes": (_SZ, []),
    "o3dx_voxel_table_build": (_I32, [_P, _I64, _P, _P, _D, _I64, _I64, _P, _I64, _P, _P, _SZ, _P]),
    "o3dx_voxel_table_build_deferred": (_I32, [_P, _I64, _P, _P, _D, _I64, _I64, _P, _I64, _P, _P, _P]),
    "o3dx_normals_workspace_bytes": (_SZ, [_I64]),
    "o3dx_estimate_normals_voxel": (_I32, [_P, _P, _P, _I64, _I32, _I32, _D, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_estimate_normals": (_I32, [_P, _I64, _I32, _I32, _D, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_voxel_down_sample_normals": (_I32, [_P, _I64, _P, _P, _D, _I32, _P, _P, _P, _P, _P, _I64, _P, _P, _SZ, _P,
                                               _SZ, _P]),
    "o3dx_knn_workspace_bytes": (_SZ, [_I64]),
    "o3dx_knn_search": (_I32, [_P, _I64, _P, _I64, _I32, _I32, _D, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_ransac_samples": (_I32, [_I64, _I32, _I32, ctypes.c_uint64, _P]),
    "o3dx_segment_plane_workspace_bytes": (_SZ, [_I64, _I32]),
    "o3dx_segment_plane": (_I32, [_P, _I64, _D, _I32, _I32, _D, _P, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_plane_from_points": (_I32, [_P, _I32, _P]),
    "o3dx_planes_from_samples": (_I32, [_P, _I32, _I32, _P]),
    "o3dx_plane_count_workspace_bytes": (_SZ, [_I64, _I32]),
    "o3dx_plane_count": (_I32, [_P, _I64, _P, _I32, _D, _P, _P, _SZ, _P]),
    "o3dx_plane_abs_sum": (_I32, [_P, _I64, _P, _P, _I32, _D, _P, _P, _P, _SZ, _P]),
    "o3dx_ransac_tied": (_I32, [_P, _P, _I32, _I64, _I32, _D, _P, _P]),
    "o3dx_plane_count_upper": (_I32, [_P, _I64, _P, _I32, _D, _P, _P, _P, _SZ, _P]),
    "o3dx_ransac_needed": (_I32, [_P, _P, _P, _I32, _I64, _I32, _D, _P, _P]),
    "o3dx_ransac_select": (_I32, [_P, _P, _P, _I32, _I64, _I32, _D]),
    "o3dx_plane_inliers": (_I32, [_P, _I64, _P, _D, _P, _P, _P, _SZ, _P]),
    "o3dx_plane_select_workspace_bytes": (_SZ, [_I64]),
    "o3dx_plane_select": (_I32, [_P, _I64, _P, _I32, _D, _D, _I32, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_plane_select_f64": (_I32, [_P, _I64, _P, _I32, _D, _D, _I32, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_plane_moments_workspace_bytes": (_SZ, [_I64]),
    "o3dx_plane_moments": (_I32, [_P, _P, _I64, _P, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_plane_from_moments": (_I32, [_P, _I64, _P, _P]),
    "o3dx_icp_target_workspace_bytes": (_SZ, [_I64]),
    "o3dx_icp_target_build": (_I32, [_P, _P, _I64, _D, _P, _SZ, _P, _P]),
    "o3dx_icp_accumulate_workspace_bytes": (_SZ, [_I64]),
    "o3dx_icp_accumulate": (_I32, [_P, _I64, _I32, _P, _P, _P, _D, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_spatial_sort_workspace_bytes": (_SZ, [_I64]),
    "o3dx_spatial_sort": (_I32, [_P, _I64, _D, _P, _P, _SZ, _P]),
    "o3dx_spatial_sort_bounds": (_I32, [_P, _I64, _D, _P, _P, _P, _SZ, _P]),
    "o3dx_pcd_unpack": (_I32, [_P, _I64, _I32, _P, _P, _P, _P, _P, _P]),
    "o3dx_lzf_decompress": (_I64, [_P, _I64, _P, _I64]),
    "o3dx_registration_icp_workspace_bytes": (_SZ, [_I64]),
    "o3dx_icp_solve_point_to_plane": (_I32, [_P, _P]),
    "o3dx_icp_update": (_I32, [_P, _P]),
    "o3dx_icp_shard_begin": (_I32, [_P, _P, _D, _I64, _P, _SZ, _P]),
    "o3dx_icp_shard_step": (_I32, [_P, _I64, _I32, _P, _P, _D, _I32, _D, _P, _P, _SZ, _P]),
    "o3dx_icp_shard_finish": (_I32, [_P, _I64, _I32, _I32, _D, _D, _D, _P, _P, _I32, _D, _I64, _P, _SZ, _P]),
    "o3dx_icp_shard_state": (_I32, [_I64, _P, _SZ, _P, _P, _P, _P, _P]),
    "o3dx_icp_shard_resume": (_I32, [_I64, _P, _SZ, _P]),
    "o3dx_icp_register": (_I32, [_P, _I64, _I32, _P, _P, _P, _I32, _D, _D, _D, _P, _P, _P, _P, _P, _P, _P, _SZ,
                                 _P]),
    "o3dx_registration_icp_point_to_plane": (_I32, [_P, _I64, _P, _P, _I64, _D, _P, _I32, _D, _D, _P, _P,
                                                     _P, _P, _P, _P, _SZ, _P, _SZ, _P]),
    "o3dx_search_one_workspace_bytes": (_SZ, [_I64]),
    "o3dx_search_one": (_I32, [_P, _I32, _I64, _P, _I32, _I64, _D, _P, _P, _I64, _P, _P, _SZ, _P]),
    # the float64 boundary (ABI 5)
    "o3dx_aabb_f64_workspace_bytes": (_SZ, [_I64]),
    "o3dx_aabb_f64": (_I32, [_P, _I64, _P, _P, _SZ, _P]),
    "o3dx_voxel_f64_workspace_bytes": (_SZ, [_I64]),
    "o3dx_voxel_down_sample_f64": (_I32, [_P, _I64, _P, _P, _D, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_normals_f64_workspace_bytes": (_SZ, [_I64]),
    "o3dx_estimate_normals_f64": (_I32, [_P, _I64, _I32, _I32, _D, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_knn_f64_workspace_bytes": (_SZ, [_I64]),
    "o3dx_knn_search_f64": (_I32, [_P, _I64, _P, _I64, _I32, _I32, _D, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_plane_count_f64": (_I32, [_P, _I64, _P, _I32, _D, _P, _P, _SZ, _P]),
    "o3dx_segment_plane_f64_workspace_bytes": (_SZ, [_I64, _I32]),
    "o3dx_segment_plane_f64": (_I32, [_P, _I64, _D, _I32, _I32, _D, _P, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_icp_target_f64_workspace_bytes": (_SZ, [_I64]),
    "o3dx_icp_target_build_f64": (_I32, [_P, _P, _I64, _D, _P, _SZ, _P, _P]),
    "o3dx_spatial_sort_f64_workspace_bytes": (_SZ, [_I64]),
    "o3dx_spatial_sort_f64": (_I32, [_P, _I64, _D, _P, _P, _SZ, _P]),
    "o3dx_icp_register_f64": (_I32, [_P, _I64, _I32, _P, _P, _P, _I32, _D, _D, _D, _P, _P, _P, _P, _P, _P, _P,
                                     _SZ, _P]),
    "o3dx_registration_icp_f64_workspace_bytes": (_SZ, [_I64]),
    "o3dx_registration_icp_point_to_plane_f64": (_I32, [_P, _I64, _P, _P, _I64, _D, _P, _I32, _D, _D, _P, _P,
                                                         _P, _P, _P, _P, _SZ, _P, _SZ, _P]),
    # the slab step's device side (ABI 6)
    "o3dx_voxel_down_sample_window_deferred": (_I32, [_P, _I64, _P, _P, _D, _I64, _I64, _P, _P, _P, _P, _SZ, _P]),
    "o3dx_slab_pack_workspace_bytes": (_SZ, [_I64]),
    "o3dx_slab_halo_pack": (_I32, [_P, _P, _P, _P, _I64, _D, _D, _I64, _I64, _I32, _I32, _P, _P, _I64, _P, _SZ,
                                   _P]),
    "o3dx_slab_halo_merge": (_I32, [_P, _P, _P, _I64, _P, _I64, _I64, _P, _I64, _P, _P, _P]),
    "o3dx_slab_verdict": (_I32, [_P, _P, _P, _I64, _P, _P, _D, _D, _I32, _I32, _D, _P, _P, _P, _P, _P]),
}

_lib = None
_lock = threading.Lock()


def declared_symbols():
    """Every function name declared in include/o3dx.h."""
    return list(_SIGS)


def load():
    """Load libo3dx.so (raises RuntimeError when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"libo3dx.so not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load().o3dx_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg}" if what else msg)


def require_device(t: torch.Tensor, what: str = "input"):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError(f"{what} must be a torch tensor on a ROCm GPU (got "
                           f"{getattr(t, 'device', type(t))}); no CPU path exists")


def default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("no ROCm GPU visible: the open3dpypro-mi355x kernels need an MI355X")
    return torch.device("cuda", torch.cuda.current_device())


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device: torch.device) -> int:
    # the raw handle without building a torch.cuda.Stream (launch-path cost)
    if _raw_stream is not None and device.index is not None:
        return _raw_stream(device.index)
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


# per (device, stream) scratch buffers, grown on demand
_ws = {}


def workspace(nbytes: int, device: torch.device, slot: str = "main") -> torch.Tensor:
    key = (device.index, stream_ptr(device), slot)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf


def set_kernel_timing(enable: bool):
    load().o3dx_set_kernel_timing(1 if enable else 0)


def kernel_timing_filter(names=None):
    """Only the named library timers record while timing is on (None: all)."""
    load().o3dx_kernel_timing_filter(",".join(names).encode() if names else None)


def reset_kernel_timing():
    load().o3dx_reset_kernel_timing()


def kernel_timing(name: str):
    """(total_ms, launches) of a library kernel recorded while timing was on."""
    ms = ctypes.c_double(0.0)
    cnt = ctypes.c_int64(0)
    load().o3dx_kernel_timing(name.encode(), ctypes.byref(ms), ctypes.byref(cnt))
    return ms.value, cnt.value


def search_stats(enable=None):
    """Debug: enable/disable neighbour-search counters, or read
    {queries, cells, candidates, shells, tile/hist hand-offs} when called
    without arguments."""
    import numpy as _np

    if enable is not None:
        check(load().o3dx_set_search_stats(1 if enable else 0), "search_stats")
        return None
    out = _np.zeros(8, _np.int64)
    check(load().o3dx_search_stats(out.ctypes.data_as(ctypes.c_void_p)), "search_stats")
    q = max(int(out[0]), 1)
    return {"queries": int(out[0]), "cells_per_query": out[1] / q, "cands_per_query": out[2] / q,
            "shells_per_query": out[3] / q, "tile_fallbacks": int(out[4]), "wave_fallbacks": int(out[5]),
            "tile_box_overflow": int(out[6]), "tile_short_radius": int(out[7])}


def release_workspaces():
    _ws.clear()
