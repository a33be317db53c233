#!/usr/bin/env python
"""bench.py — headline benchmark: Mpoints/s of voxel_down_sample + estimate_normals
(KNN30) on synthetic uniform-random 10M-point float32 clouds (BASELINE.json
configs[1]), plus ICP iterations/s and RANSAC time (C3) as
secondary figures.

One step = one pass of the hot path over one cloud that is already resident
in HBM: voxel_down_sample(vs=(4/N)^(1/3)) -> estimate_normals(KNN 30) on the
M representatives.  Multi-GPU: one process per GPU (torchrun), each rank owns
one 10M-point spatial tile (an independent cloud, no data-path collective):
weak scaling.  `value` = points processed by all ranks / max-over-ranks time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
   or: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "open3d-py-extension_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from open3dpypro import _native, ops, synthetic  # noqa: E402

METRIC = "Mpoints/sec voxel_down_sample+estimate_normals; ICP iters/sec @ N=10M"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_VALU_PEAK_TFLOPS = 78.6   # vector FP64 (half of the 157.3 TF FP32 vector peak)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=10_000_000, help="points per GPU (C2: 10M)")
    ap.add_argument("--knn", type=int, default=30)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--sorted-grid", action="store_true",
                    help="normals sort the representatives into their own grid (no voxel table hand-over)")
    ap.add_argument("--cpu-n", type=int, default=2_000_000, help="CPU baseline sample size")
    ap.add_argument("--no-secondary", action="store_true", help="skip the ICP / RANSAC figures")
    ap.add_argument("--icp-n", type=int, default=10_000_000)
    ap.add_argument("--icp-iters", type=int, default=30)
    ap.add_argument("--ransac-iters", type=int, default=1000)
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--c4-n", type=int, default=50_000_000, help="C4 cloud size (0: skip the C4 legs)")
    ap.add_argument("--dist-icp", action="store_true",
                    help="also run the sharded-ICP leg (RCCL) when world == 1 (under torchrun)")
    return ap.parse_args()


def setup_dist(force=False):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or (force and "MASTER_PORT" in os.environ):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    return world, rank, dev


def barrier(world, dev):
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_entry(path, kernel):
    """Per-launch PMC figures of `kernel` from the committed rocprofv3 summary
    (tools/pmc.sh + tools/pmc_summary.py): HBM bytes, VALU-issue floor."""
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("kernels", {}).get(kernel) or {}
    except (OSError, ValueError, TypeError):
        return {}


def cpu_baseline(n_cpu: int):
    """Oracle restatement of Open3D's CPU path (voxel trace single-threaded as in
    Open3D, KNN30 normals with OpenMP) on a bounded C2-shaped sample."""
    from oracle import oracle as O

    pts = synthetic.uniform_cube(n_cpu, seed=0).numpy()
    vs = synthetic.voxel_size_for(n_cpu)
    O.lib()
    t0 = time.perf_counter()
    rep = O.voxel_down_sample(pts, vs)
    t1 = time.perf_counter()
    O.estimate_normals(pts[rep], O.KNN, 30)
    t2 = time.perf_counter()
    el = t2 - t0
    return {"value": round(n_cpu / el / 1e6, 4), "unit": "Mpoints/s", "cores": O.num_threads(),
            "kind": "port",
            "sample": (f"C2 shape at N={n_cpu} (uniform cube, vs=(4/N)^(1/3), M={len(rep)}): "
                       f"Open3D-equivalent C++ restatement (oracle/): voxel trace 1 thread "
                       f"{t1 - t0:.2f}s + KD-tree KNN30 normals {O.num_threads()} OpenMP threads "
                       f"{t2 - t1:.2f}s; host {platform.processor() or platform.machine()}"),
            "seconds": round(el, 3)}


def secondary(dev, args):
    """C3 on one GPU: RANSAC 1000 hypotheses and point-to-plane ICP, 10M points."""
    out = {}
    n = args.icp_n
    _native.set_kernel_timing(True)
    # RANSAC: planted plane, Open3D RandomSampler samples, full hypothesis sweep
    pts = synthetic.planted_plane(n, seed=1, device=dev)
    samples = ops.ransac_samples(n, 3, args.ransac_iters, seed=7)
    ops.segment_plane(pts, 0.01, 3, args.ransac_iters, samples=samples)  # warm
    _native.reset_kernel_timing()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    plane, inl = ops.segment_plane(pts, 0.01, 3, args.ransac_iters, samples=samples)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    pc_ms, pc_n = _native.kernel_timing("plane_count")
    pairs = float(n) * args.ransac_iters
    out["ransac"] = {"n": n, "iterations": args.ransac_iters, "ms": round((t1 - t0) * 1e3, 3),
                     "plane_count_kernel_ms": round(pc_ms, 3), "inliers": int(inl.numel()),
                     "plane": [round(float(v), 6) for v in plane],
                     "Gpairs_per_s": round(pairs / (pc_ms * 1e-3) / 1e9, 2) if pc_ms > 0 else None}
    del pts, inl
    # ICP: box-surface target with KNN30 normals, source = independent sample moved by T_gt
    tgt = synthetic.box_surface(n, seed=1, device=dev)
    src = synthetic.apply_transform(synthetic.box_surface(n, seed=2, device=dev), synthetic.rigid_transform())
    t0 = time.perf_counter()
    tn = ops.estimate_normals(tgt, knn=30)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    target = ops.ICPTarget(tgt, tn, 0.02)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    src4 = ops.spatial_sort(src)          # once per source cloud
    torch.cuda.synchronize(dev)
    t2b = time.perf_counter()
    T = np.eye(4)
    sums, _ = target.accumulate(src4, T)  # warm
    _native.reset_kernel_timing()
    torch.cuda.synchronize(dev)
    t3 = time.perf_counter()
    for _ in range(args.icp_iters):
        sums, _ = target.accumulate(src4, T)
        T = ops.icp_solve(sums) @ T
    torch.cuda.synchronize(dev)
    t4 = time.perf_counter()
    acc_ms, acc_n = _native.kernel_timing("icp_accumulate")
    m_ms, m_n = _native.kernel_timing("icp_match")
    _native.set_kernel_timing(False)
    err = np.abs(T - np.linalg.inv(synthetic.rigid_transform())).max()
    out["icp"] = {"n_source": n, "n_target": n, "iterations": args.icp_iters,
                  "iters_per_s": round(args.icp_iters / (t4 - t3), 3),
                  "ms_per_iter": round((t4 - t3) / args.icp_iters * 1e3, 3),
                  "accumulate_kernel_ms": round(acc_ms / max(acc_n, 1), 3),
                  "match_kernel_ms": round(m_ms / max(m_n, 1), 3),
                  "target_normals_s": round(t1 - t0, 3), "target_build_s": round(t2 - t1, 3),
                  "source_sort_s": round(t2b - t2, 3),
                  "fitness": round(float(sums[28]) / n, 6), "T_err_vs_gt_inverse": float(err),
                  "achieved_GBs_36B_per_src_pt": round(36.0 * n / (acc_ms / max(acc_n, 1) * 1e-3) / 1e9, 2)
                  if acc_ms > 0 else None}
    return out


def secondary_sharded_icp(dev, args, world, rank):
    """C3/C5-style ICP with the source sharded over the ranks (strong scaling of
    one 10M source) and the target replicated; the 29 float64 moments are
    all-gathered over RCCL once per iteration (open3dpypro.distributed)."""
    from open3dpypro import distributed as D

    n = args.icp_n
    tgt = synthetic.box_surface(n, seed=1, device=dev)
    src = synthetic.apply_transform(synthetic.box_surface(n, seed=2, device=dev), synthetic.rigid_transform())
    target = ops.ICPTarget(tgt, ops.estimate_normals(tgt, knn=30), 0.02)
    a, b = D.shard_range(n, world, rank)
    shard = ops.spatial_sort(src[a:b].contiguous())
    del src
    acc = lambda T: target.accumulate(shard, T)[0]  # noqa: E731
    D.registration_icp_point_to_plane(acc, n, max_iteration=1)  # warm
    barrier(world, dev)
    t0 = time.perf_counter()
    T, fit, rm = D.registration_icp_point_to_plane(acc, n, max_iteration=args.icp_iters, relative_fitness=0.0,
                                                   relative_rmse=0.0)
    barrier(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    err = float(np.abs(T - np.linalg.inv(synthetic.rigid_transform())).max())
    return {"icp_sharded": {"n_source": n, "n_target": n, "ranks": world, "iterations": args.icp_iters,
                            "iters_per_s": round(args.icp_iters / el, 3), "fitness": round(fit, 6),
                            "T_err_vs_gt_inverse": err,
                            "collective": "all_gather of 32 float64 per iteration (RCCL), summed in rank order"}}


def c4_single_gpu(dev, args):
    """C4's cloud size on one GPU (north star: voxel_down_sample +
    estimate_normals at N=50M): the headline step on 50M uniform points."""
    n = args.c4_n
    pts = synthetic.uniform_cube(n, seed=0, device=dev)
    vs = synthetic.voxel_size_for(n)

    def step():
        out = ops.voxel_down_sample(pts, vs, keep_grid=True)
        ops.estimate_normals(out["rep_xyz"], knn=args.knn, voxel_grid=out.get("voxel_grid"))
        return out["rep_idx"].numel()

    step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(3):
        m = step()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / 3
    algo = 12.0 * n + 28.0 * m
    del pts
    torch.cuda.empty_cache()
    return {"c4_single_gpu": {"n": n, "voxels": int(m), "ms": round(el * 1e3, 3),
                              "Mpoints_per_s": round(n / el / 1e6, 2),
                              "pipeline_algorithmic_GBs": round(algo / el / 1e9, 2),
                              "frac_of_hbm_peak": round(algo / el / 1e9 / HBM_PEAK_GBS, 5),
                              "algorithmic_bytes": "12 N + 28 M (SURVEY.md 8(d))"}}


def c4_slabs(dev, args, world, rank):
    """C4 across the ranks: ONE 50M cloud (this rank holds an index range of
    it), voxel-aligned x-slabs, points to their slab owner and a verified halo
    of representatives to the neighbours (all-to-all over RCCL), voxel reps +
    KNN normals per slab (open3dpypro.distributed.voxel_normals_slabs)."""
    from open3dpypro import distributed as D

    n = args.c4_n
    a, b = D.shard_range(n, world, rank)
    pts = synthetic.uniform_cube(b - a, seed=0, offset=a, device=dev)
    gidx = torch.arange(a, b, dtype=torch.int64, device=dev)
    vs = synthetic.voxel_size_for(n)
    D.voxel_normals_slabs(pts, gidx, vs, knn=args.knn)  # warm
    barrier(world, dev)
    t0 = time.perf_counter()
    rg, _, _ = D.voxel_normals_slabs(pts, gidx, vs, knn=args.knn)
    barrier(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    m = torch.tensor([rg.numel()], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(m)
    return {"c4_slabs": {"n": n, "ranks": world, "voxels": int(m.item()), "ms": round(el * 1e3, 3),
                         "Mpoints_per_s": round(n / el / 1e6, 2), "scaling": "strong",
                         "collectives": "all_reduce (AABB, halo check), all_to_all (points to slab owners, halo reps)"}}


def main():
    args = parse()
    world, rank, dev = setup_dist(args.dist_icp)
    N = args.n
    vs = synthetic.voxel_size_for(N)
    # this rank's tile: an independent 10M cloud, shifted to x in [rank, rank+1)
    pts = synthetic.uniform_cube(N, seed=0, offset=rank * N, device=dev)
    pts[:, 0] += float(rank)
    torch.cuda.synchronize(dev)

    keep = not args.sorted_grid

    def step():
        # PointCloud.voxel_down_sample(vs).estimate_normals(): the voxel table
        # of the first call is the search grid of the second
        out = ops.voxel_down_sample(pts, vs, keep_grid=keep)
        nrm = ops.estimate_normals(out["rep_xyz"], knn=args.knn, voxel_grid=out.get("voxel_grid"))
        return out["rep_idx"].numel(), nrm

    for _ in range(args.warmup):
        M, _ = step()
    _native.reset_kernel_timing()
    _native.set_kernel_timing(True)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier(world, dev)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        M, _ = step()
    ev1.record()
    barrier(world, dev)
    t1 = time.perf_counter()
    _native.set_kernel_timing(False)
    elapsed = max_over_ranks(t1 - t0, world, dev)
    ev_ms = ev0.elapsed_time(ev1)

    kernels = {}
    for name in ("voxel_assign", "voxel_compact", "grid_count", "grid_sort", "normals_stile", "normals_tile",
                 "normals_wave", "normals_knn"):
        ms, cnt = _native.kernel_timing(name)
        if cnt:
            kernels[name] = {"avg_ms": round(ms / cnt, 4), "launches": cnt}
    # algorithmic bytes per launch:
    #   normals_stile / normals_tile: M queries x (12 B xyz read + 12 B normal written)
    #   voxel_assign: N points x (12 B xyz read + 4 B voxel id written)
    algo_bytes = {"normals_stile": 24.0 * M, "normals_tile": 24.0 * M, "voxel_assign": 16.0 * N}
    dom = max((k for k in kernels if k in algo_bytes), key=lambda k: kernels[k]["avg_ms"], default=None)
    roof = None
    if dom is not None:
        avg_s = kernels[dom]["avg_ms"] * 1e-3
        ach = algo_bytes[dom] / avg_s / 1e9
        pmc = pmc_entry(args.pmc_json, dom)
        traffic = pmc.get("hbm_bytes_per_launch")
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": traffic,
                "algorithmic_bytes_per_launch": algo_bytes[dom],
                "note": "kNN selection is VALU/LDS-issue bound, not HBM bound: see DESIGN.md (Roofline)"}
        if pmc.get("valu_issue_floor_ms"):
            # the bound that actually applies: VALU issue (PMC SQ_INSTS_VALU x 4 cycles / 1024 SIMDs @ 2.4 GHz)
            roof["valu_issue_floor_ms"] = round(pmc["valu_issue_floor_ms"], 4)
            roof["valu_issue_frac"] = round(pmc["valu_issue_floor_ms"] / kernels[dom]["avg_ms"], 4)

    total_pts = float(N) * world * args.steps
    value = total_pts / elapsed / 1e6
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "Mpoints/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C2: uniform-random 10M pts float32 per GPU, voxel_down_sample(vs=(4/N)^(1/3)) "
                               "+ estimate_normals(KNN30) on the representatives",
                   "n_points_per_gpu": N, "voxel_size": vs, "voxels_per_gpu": int(M), "knn": args.knn,
                   "parallelism": f"tile-per-gpu x{world}"},
        "roofline": roof,
        "cpu_baseline": None,
        "extra": {"stream_event_ms_per_step_rank0": round(ev_ms / args.steps, 3), "kernels": kernels,
                  "pipeline_algorithmic_GBs": round((12.0 * N + 28.0 * M) * args.steps * world / elapsed / 1e9, 2),
                  "storage_dtype": "f32", "arith": "float64 voxel keys / distances / covariance"},
    }
    del pts
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_secondary:
        try:
            line["extra"].update(secondary(dev, args))
        except RuntimeError as e:  # report, never hide
            line["extra"]["secondary_error"] = str(e)
    if (world > 1 or args.dist_icp) and not args.no_secondary:
        try:
            line["extra"].update(secondary_sharded_icp(dev, args, world, rank))
        except RuntimeError as e:  # report, never hide
            line["extra"]["secondary_error"] = str(e)
    if args.c4_n > 0 and not args.no_secondary:
        try:
            if world == 1:
                line["extra"].update(c4_single_gpu(dev, args))
            else:
                line["extra"].update(c4_slabs(dev, args, world, rank))
        except RuntimeError as e:  # report, never hide
            line["extra"]["c4_error"] = str(e)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args.cpu_n)
        if line["cpu_baseline"]["value"] > 0:
            line["extra"]["gpu_over_cpu"] = round(value / line["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
