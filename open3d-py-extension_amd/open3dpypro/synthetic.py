"""Counter-based synthetic clouds.

Every coordinate is a function of (seed, global index) only — splitmix64 of
the counter, top 24 bits -> float32 in [0, 1) — so any shard / rank / device
regenerates exactly the same points with integer torch ops (bit-identical on
CPU and GPU).  Not part of the reference API (data plumbing for tests/bench).
"""
from __future__ import annotations

import math

import numpy as np
import torch

_GOLD = -7046029254386353131        # 0x9E3779B97F4A7C15 as int64
_M1 = -4658895280553007687          # 0xBF58476D1CE4E5B9
_M2 = -7723592293110705685          # 0x94D049BB133111EB


def _srl(z: torch.Tensor, k: int) -> torch.Tensor:
    """logical right shift on int64"""
    return (z >> k) & ((1 << (64 - k)) - 1)


def splitmix64(counter: torch.Tensor, seed: int) -> torch.Tensor:
    z = counter.to(torch.int64) * _GOLD + (seed * 0x632BE59BD9B4E019 & 0x7FFFFFFFFFFFFFFF)
    z = (z ^ _srl(z, 30)) * _M1
    z = (z ^ _srl(z, 27)) * _M2
    return z ^ _srl(z, 31)


def uniform01(counter: torch.Tensor, seed: int) -> torch.Tensor:
    """float32 in [0,1) with a 24-bit mantissa grid (exact in float32)."""
    return (_srl(splitmix64(counter, seed), 40).to(torch.float32)) * (1.0 / 16777216.0)


def uniform_cube(n: int, seed: int = 0, offset: int = 0, device="cpu") -> torch.Tensor:
    """C2/C4: (n,3) float32 ~ U[0,1)^3; point i uses counters 3*(offset+i)+a."""
    i = torch.arange(offset, offset + n, dtype=torch.int64, device=device)
    c = (3 * i).unsqueeze(1) + torch.arange(3, dtype=torch.int64, device=device)
    return uniform01(c, seed)


def _normal(counter: torch.Tensor, seed: int) -> torch.Tensor:
    u1 = uniform01(2 * counter, seed + 101).double().clamp_min(2.0 ** -25)
    u2 = uniform01(2 * counter + 1, seed + 101).double()
    return torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2)


def planted_plane(n: int, seed: int = 0, frac: float = 0.2, z0: float = 0.5, sigma: float = 0.002,
                  offset: int = 0, device="cpu") -> torch.Tensor:
    """C3 RANSAC cloud: (1-frac) uniform cube + frac on z = z0 + N(0, sigma)."""
    p = uniform_cube(n, seed, offset, device)
    i = torch.arange(offset, offset + n, dtype=torch.int64, device=device)
    on = uniform01(i, seed + 7) < frac
    z = (z0 + sigma * _normal(i, seed)).to(torch.float32)
    p[:, 2] = torch.where(on, z, p[:, 2])
    return p


def box_surface(n: int, seed: int = 0, dims=(1.0, 0.8, 0.6), offset: int = 0, device="cpu") -> torch.Tensor:
    """C3 ICP target/source: uniform samples on the surface of [0,a]x[0,b]x[0,c]."""
    a, b, c = dims
    areas = np.array([b * c, b * c, a * c, a * c, a * b, a * b], np.float64)
    cum = torch.tensor(np.cumsum(areas) / areas.sum(), dtype=torch.float64, device=device)
    i = torch.arange(offset, offset + n, dtype=torch.int64, device=device)
    f = torch.searchsorted(cum, uniform01(i, seed + 13).double(), right=True).clamp_max(5)
    u = uniform01(3 * i, seed + 17)
    v = uniform01(3 * i + 1, seed + 17)
    p = torch.empty((n, 3), dtype=torch.float32, device=device)
    axis = f // 2                      # 0: x-faces, 1: y-faces, 2: z-faces
    side = (f % 2).to(torch.float32)   # 0: min face, 1: max face
    D = torch.tensor([a, b, c], dtype=torch.float32, device=device)
    for ax in range(3):
        m = axis == ax
        o1, o2 = [k for k in range(3) if k != ax]
        p[m, ax] = side[m] * D[ax]
        p[m, o1] = u[m] * D[o1]
        p[m, o2] = v[m] * D[o2]
    return p


def rigid_transform(angle_deg: float = 1.0, axis=(1.0, 2.0, 3.0), t=(0.005, -0.003, 0.002)) -> np.ndarray:
    """T_gt of config C3: rotation by angle about axis (Rodrigues) + translation."""
    k = np.asarray(axis, np.float64)
    k = k / np.linalg.norm(k)
    th = math.radians(angle_deg)
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * (K @ K)
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def apply_transform(p: torch.Tensor, T: np.ndarray) -> torch.Tensor:
    Tt = torch.tensor(T, dtype=torch.float64, device=p.device)
    return (p.double() @ Tt[:3, :3].T + Tt[:3, 3]).to(torch.float32)


LAS_OFFSET = (512345.6789, 431234.5678, 118.765)


def uniform01_f64(counter: torch.Tensor, seed: int) -> torch.Tensor:
    """float64 in [0,1) with a full 53-bit mantissa."""
    return (_srl(splitmix64(counter, seed), 11).to(torch.float64)) * (1.0 / 9007199254740992.0)


def las_scene(n: int, seed: int = 0, dims=(40.0, 32.0, 24.0), offset=LAS_OFFSET, T=None,
              device="cpu") -> torch.Tensor:
    """(n,3) float64 LAS-like scan: uniform samples on the surface of the box
    [0,a]x[0,b]x[0,c] metres with full-mantissa float64 coordinates, moved by
    the rigid motion T (about the box centre; None: identity) and placed at a
    georeferenced offset (~5e5 m).  Not float32-representable: the float64
    boundary's test cloud."""
    a, b, c = dims
    areas = np.array([b * c, b * c, a * c, a * c, a * b, a * b], np.float64)
    cum = torch.tensor(np.cumsum(areas) / areas.sum(), dtype=torch.float64, device=device)
    i = torch.arange(n, dtype=torch.int64, device=device)
    f = torch.searchsorted(cum, uniform01_f64(i, seed + 13), right=True).clamp_max(5)
    u = uniform01_f64(3 * i, seed + 17)
    v = uniform01_f64(3 * i + 1, seed + 17)
    p = torch.empty((n, 3), dtype=torch.float64, device=device)
    axis = f // 2
    side = (f % 2).to(torch.float64)
    D = torch.tensor([a, b, c], dtype=torch.float64, device=device)
    for ax in range(3):
        m = axis == ax
        o1, o2 = [k for k in range(3) if k != ax]
        p[m, ax] = side[m] * D[ax]
        p[m, o1] = u[m] * D[o1]
        p[m, o2] = v[m] * D[o2]
    if T is not None:
        ctr = D * 0.5
        Tt = torch.tensor(np.asarray(T, np.float64), dtype=torch.float64, device=device)
        p = (p - ctr) @ Tt[:3, :3].T + Tt[:3, 3] + ctr
    return p + torch.tensor(offset, dtype=torch.float64, device=device)


def las_motion_world(T: np.ndarray, dims=(40.0, 32.0, 24.0), offset=LAS_OFFSET) -> np.ndarray:
    """The world-frame 4x4 of las_scene's motion T (applied about the box
    centre): the transformation registration_icp recovers, source -> target,
    when the source is las_scene(T=T) and the target las_scene()."""
    c = np.asarray(dims, np.float64) * 0.5 + np.asarray(offset, np.float64)
    A, B = np.eye(4), np.eye(4)
    A[:3, 3] = c
    B[:3, 3] = -c
    return A @ np.asarray(T, np.float64) @ B


def voxel_size_for(n: int) -> float:
    """C2/C4 voxel size (4/N)^(1/3): ~4 points per voxel on the unit cube."""
    return (4.0 / n) ** (1.0 / 3.0)
