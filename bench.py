#!/usr/bin/env python
"""bench.py — headline benchmark (BASELINE.json metric): Mpoints/s of
voxel_down_sample + estimate_normals (KNN30), plus ICP iterations/s.

N = 1 (default): C2 — one synthetic uniform-random 10M-point float32 cloud
resident in HBM; one step = voxel_down_sample(vs=(4/N)^(1/3)) ->
estimate_normals(KNN 30) on the M representatives.  Secondary figures on the
same GPU: C3 (RANSAC 1000 hypotheses + point-to-plane ICP 30 iterations at
10M), C4's size on one GPU (50M) and C5 (200M full pipeline incl. ICP), and
the CPU baselines (the oracle, an Open3D-equivalent C++ restatement) of the
voxel+normals step, RANSAC and ICP on the same inputs.

N > 1 (one process per GPU, RCCL): C2 per GPU, weak scaling — ONE
uniform-random cloud of N x 10M points over [0,N) x [0,1)^2 (the C2 density,
C2's voxel size), tiled over the ranks as voxel-aligned x-slabs (each rank's
~10M points resident in its slab); one step = global AABB all-reduce, slab
voxel reps, halo exchange of boundary representatives (all-to-all), normals
off the slab's voxel table, halo-proof verdict all-gather
(open3dpypro.distributed.voxel_normals_slabs).  `value` = points of the whole
job / max-over-ranks time.  Beside it: C4 (ONE 50M cloud over the same ranks,
strong scaling), the sharded ICP and the sharded C5 pipeline.

Launch forms:
  python bench.py --gpus N      (no WORLD_SIZE in the environment, N > 1): the
      parent never touches a GPU; it starts fresh child processes, one per GPU
      (RANK / LOCAL_RANK / WORLD_SIZE, RCCL), for 1, 2, 4, ... N ranks in turn
      and prints ONE line: the N-rank figures, the whole 1 -> N curve
      (`scaling_curve`, C2-per-GPU weak and C4 strong) and the CPU baseline
      (timed by the parent after the GPU runs);
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
      (WORLD_SIZE set): this process is one rank of an N-rank run; rank 0
      prints the N-rank line.
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=25,
                    help="untimed steps first (the clocks settle over ~20 steps: profiles/r02_call_structure.txt)")
    ap.add_argument("--n", type=int, default=10_000_000, help="points per GPU (C2: 10M)")
    ap.add_argument("--knn", type=int, default=30)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--sorted-grid", action="store_true",
                    help="normals sort the representatives into their own grid (no voxel table hand-over)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="no HIP events inside the timed region (the dominant kernel is then timed in a later pass)")
    ap.add_argument("--two-call", action="store_true",
                    help="time voxel_down_sample and estimate_normals as two library calls (default: the one-call "
                         "pipeline o3dx_voxel_down_sample_normals)")
    ap.add_argument("--cpu-n", type=int, default=10_000_000, help="CPU baseline size (C2 input: 10M)")
    ap.add_argument("--cpu-icp-iters", type=int, default=2, help="ICP iterations of the CPU ICP leg (bounded sample)")
    ap.add_argument("--c5-n", type=int, default=200_000_000, help="C5 cloud size (0: skip the C5 leg)")
    ap.add_argument("--no-secondary", action="store_true", help="skip the ICP / RANSAC figures")
    ap.add_argument("--icp-n", type=int, default=10_000_000)
    ap.add_argument("--icp-iters", type=int, default=30)
    ap.add_argument("--ransac-iters", type=int, default=1000)
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--c4-n", type=int, default=50_000_000, help="C4 cloud size (0: skip the C4 legs)")
    ap.add_argument("--dist-icp", action="store_true",
                    help="also run the sharded-ICP leg (RCCL) when world == 1 (under torchrun)")
    ap.add_argument("--scaling-child", action="store_true",
                    help="(set by the --gpus N launcher) one point of the scaling curve: the headline and C4 "
                         "only, no CPU legs")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU work: each rank joins a gloo rendezvous, all-reduces its rank count and rank 0 "
                         "prints a placeholder line (checks the --gpus N launcher on a CPU host)")
    ap.add_argument("--child-timeout", type=int, default=900,
                    help="seconds one rank count of the --gpus N sweep may take before its processes are killed")
    return ap.parse_args()


def setup_dist(force=False):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-GPU path on a one-GPU box: every rank on cuda:0, gloo
    shared = os.environ.get("O3DX_BENCH_SHARED_GPU") == "1"
    if shared:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or (force and "MASTER_PORT" in os.environ):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if shared:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    return world, rank, dev


def comm_dev(dev):
    return dev if dist.is_initialized() and dist.get_backend() == "nccl" else torch.device("cpu")


def barrier(world, dev):
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=comm_dev(dev))
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


def host_info():
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(n_cpu: int, pts_dev=None):
    """The oracle (an Open3D-equivalent C++ restatement, oracle/) of the C2
    step on the C2 input itself: voxel trace single-threaded as Open3D's,
    KD-tree KNN30 normals with OpenMP — on the inherited OMP_NUM_THREADS (the
    box's share, 16) and again on every host thread (os.cpu_count())."""
    from oracle import oracle as O

    pts = (pts_dev.cpu().numpy() if pts_dev is not None and pts_dev.shape[0] == n_cpu
           else synthetic.uniform_cube(n_cpu, seed=0).numpy())
    vs = synthetic.voxel_size_for(n_cpu)
    O.lib()
    t0 = time.perf_counter()
    rep = O.voxel_down_sample(pts, vs)
    t1 = time.perf_counter()
    O.estimate_normals(pts[rep], O.KNN, 30)
    t2 = time.perf_counter()
    el = t2 - t0
    out = {"value": round(n_cpu / el / 1e6, 4), "unit": "Mpoints/s", "cores": O.num_threads(),
           "kind": "port",
           "sample": (f"the C2 input itself (N={n_cpu}, M={len(rep)}): Open3D-equivalent C++ restatement "
                      f"(oracle/o3d_restate.cpp): voxel trace 1 thread {t1 - t0:.2f}s + KD-tree KNN30 normals "
                      f"{O.num_threads()} OpenMP threads {t2 - t1:.2f}s"),
           "seconds": round(el, 3), **host_info()}
    allc = os.cpu_count() or 1
    if allc > O.num_threads():
        # the normals on every host thread (the voxel trace stays serial, as Open3D's)
        O.set_num_threads(allc)
        t3 = time.perf_counter()
        O.estimate_normals(pts[rep], O.KNN, 30)
        t4 = time.perf_counter()
        O.set_num_threads(out["cores"])
        out["all_threads"] = {"cores": allc, "normals_s": round(t4 - t3, 3),
                              "value": round(n_cpu / ((t1 - t0) + (t4 - t3)) / 1e6, 4)}
    return out


def cpu_secondary(dev, args, tn_dev=None):
    """CPU legs of C3 through the oracle (labelled as the restatement):
    segment_plane 1000 hypotheses on the 10M planted-plane cloud (OpenMP over
    hypotheses, as Open3D), and point-to-plane ICP on the 10M box-surface
    clouds — a bounded sample of iterations (KD-tree build + per-iteration
    rate reported separately)."""
    from oracle import oracle as O

    out = {}
    n = args.icp_n
    pts = synthetic.planted_plane(n, seed=1).numpy()
    samples = ops.ransac_samples(n, 3, args.ransac_iters, seed=7)
    t0 = time.perf_counter()
    O.segment_plane(pts, 0.01, 3, args.ransac_iters, samples)
    el = time.perf_counter() - t0
    out["cpu_ransac"] = {"n": n, "iterations": args.ransac_iters, "seconds": round(el, 3),
                         "Gpairs_per_s": round(n * args.ransac_iters / el / 1e9, 3), "cores": O.num_threads(),
                         "kind": "port (oracle segment_plane, OpenMP over hypotheses)"}
    del pts
    tgt = synthetic.box_surface(n, seed=1).numpy()
    src = synthetic.apply_transform(synthetic.box_surface(n, seed=2), synthetic.rigid_transform()).numpy()
    tn = tn_dev.cpu().numpy() if tn_dev is not None else O.estimate_normals(tgt, O.KNN, 30).astype(np.float32)
    k = max(1, args.cpu_icp_iters)
    t0 = time.perf_counter()
    O.registration_icp(src, tgt, tn, 0.02, max_iteration=0)
    t1 = time.perf_counter()
    O.registration_icp(src, tgt, tn, 0.02, max_iteration=k, relative_fitness=0.0, relative_rmse=0.0)
    t2 = time.perf_counter()
    per_iter = max((t2 - t1) - (t1 - t0), 1e-9) / k  # build + first correspondence pass cancel out
    out["cpu_icp"] = {"n_source": n, "n_target": n, "iterations_timed": k,
                      "iters_per_s": round(1.0 / per_iter, 4), "setup_s": round(t1 - t0, 3),
                      "cores": O.num_threads(),
                      "kind": "port (oracle registration_icp: KD-tree build + hybrid 1-NN per iteration, OpenMP "
                              "correspondences, sequential JTJ)",
                      "sample": f"{k} iterations of C3's 10M/10M ICP; target normals = the GPU's (equal to the "
                                f"oracle's within 1e-5)"}
    return out


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
    ops.segment_plane(pts, 0.01, 3, args.ransac_iters, samples=samples)  # kernel times (events on)
    torch.cuda.synchronize(dev)
    ub_ms, _ = _native.kernel_timing("plane_count_upper")  # the sweep: all hypotheses, upper bounds
    ex_ms, ex_n = _native.kernel_timing("plane_count")  # exact re-counts of the consulted few
    pc_ms = ub_ms + ex_ms
    _native.set_kernel_timing(False)  # the timed call carries no instrumentation events
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    plane, inl = ops.segment_plane(pts, 0.01, 3, args.ransac_iters, samples=samples)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    _native.set_kernel_timing(True)
    pairs = float(n) * args.ransac_iters
    out["ransac"] = {"n": n, "iterations": args.ransac_iters, "ms": round((t1 - t0) * 1e3, 3),
                     "plane_count_kernel_ms": round(pc_ms, 3), "upper_sweep_ms": round(ub_ms, 3),
                     "exact_recount_ms": round(ex_ms, 3), "exact_recount_calls": ex_n,
                     "inliers": int(inl.numel()),
                     "plane": [round(float(v), 6) for v in plane],
                     "Gpairs_per_s": round(pairs / (pc_ms * 1e-3) / 1e9, 2) if pc_ms > 0 else None}
    del inl
    # the general path on the raw C3 cloud (no voxel table: sorted search grid,
    # its thin dense plane puts hundreds of points in a cell)
    ops.estimate_normals(pts, knn=30)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ops.estimate_normals(pts, knn=30)
    torch.cuda.synchronize(dev)
    el_raw = (time.perf_counter() - t0) * 1e3
    # the grid build (count + cell sort: round 2's cliff) and the two search
    # kernels, event-timed in a second call
    _native.set_kernel_timing(True)
    _native.reset_kernel_timing()
    ops.estimate_normals(pts, knn=30)
    torch.cuda.synchronize(dev)
    parts = {}
    for name in ("grid_count", "grid_sort", "normals_tile", "normals_wave", "normals_knn"):
        ms, cnt = _native.kernel_timing(name)
        if cnt:
            parts[name + "_ms"] = round(ms, 3)
    out["normals_raw_c3"] = {"n": n, "ms": round(el_raw, 3), **parts,
                             "grid_build_ms": round(parts.get("grid_count_ms", 0) + parts.get("grid_sort_ms", 0), 3),
                             "path": "sorted grid (estimate_normals on the raw planted-plane cloud)"}
    del pts
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
    # the loop on the device (o3dx_icp_register): Open3D's registration_icp on
    # the built target, exactly icp_iters iterations from T = I (no
    # convergence stop); timed without instrumentation, then once more with
    # the per-iteration kernels event-timed
    res = target.register(src4, max_iteration=1, relative_fitness=0.0, relative_rmse=0.0)  # warm
    _native.set_kernel_timing(False)
    torch.cuda.synchronize(dev)
    t3 = time.perf_counter()
    res = target.register(src4, max_iteration=args.icp_iters, relative_fitness=0.0, relative_rmse=0.0)
    torch.cuda.synchronize(dev)
    t4 = time.perf_counter()
    T = res["transformation"]
    _native.reset_kernel_timing()
    _native.set_kernel_timing(True)
    target.register(src4, max_iteration=args.icp_iters, relative_fitness=0.0, relative_rmse=0.0)
    torch.cuda.synchronize(dev)
    m_ms, m_n = _native.kernel_timing("icp_match")
    loop_ms, _ = _native.kernel_timing("icp_loop")
    _native.set_kernel_timing(False)
    err = np.abs(T - np.linalg.inv(synthetic.rigid_transform())).max()
    step_ms = m_ms / max(m_n, 1)
    out["icp"] = {"n_source": n, "n_target": n, "iterations": args.icp_iters,
                  "iters_per_s": round(args.icp_iters / (t4 - t3), 3),
                  "ms_per_iter": round((t4 - t3) / args.icp_iters * 1e3, 3),
                  "loop": "device (o3dx_icp_register: fused step + on-device solve per iteration, one host wait)",
                  "step_kernel_ms": round(step_ms, 3), "step_launches": m_n,
                  "loop_events_ms": round(loop_ms, 3),
                  "target_normals_s": round(t1 - t0, 3), "target_build_s": round(t2 - t1, 3),
                  "source_sort_s": round(t2b - t2, 3),
                  "fitness": round(res["fitness"], 6), "T_err_vs_gt_inverse": float(err),
                  "achieved_GBs_36B_per_src_pt": round(36.0 * n / (step_ms * 1e-3) / 1e9, 2) if step_ms > 0 else None}
    return out


def secondary_sharded_icp(dev, args, world, rank):
    """C3-style ICP with the source sharded over the ranks (strong scaling of
    one 10M source) and the target replicated; the moments are exact fx sums
    all-reduced over RCCL once per iteration (open3dpypro.distributed), so T
    is the single-GPU result to the bit."""
    from open3dpypro import distributed as D

    n = args.icp_n
    tgt = synthetic.box_surface(n, seed=1, device=dev)
    src = synthetic.apply_transform(synthetic.box_surface(n, seed=2, device=dev), synthetic.rigid_transform())
    target = ops.ICPTarget(tgt, ops.estimate_normals(tgt, knn=30), 0.02)
    a, b = D.shard_range(n, world, rank)
    shard = src[a:b].contiguous()
    del src
    D.registration_icp_sharded(shard, target, max_iteration=1)  # warm
    barrier(world, dev)
    t0 = time.perf_counter()
    T, fit, rm = D.registration_icp_sharded(shard, target, max_iteration=args.icp_iters, relative_fitness=0.0,
                                            relative_rmse=0.0)
    barrier(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    err = float(np.abs(T - np.linalg.inv(synthetic.rigid_transform())).max())
    return {"icp_sharded": {"n_source": n, "n_target": n, "ranks": world, "iterations": args.icp_iters,
                            "iters_per_s": round(args.icp_iters / el, 3), "fitness": round(fit, 6),
                            "T_err_vs_gt_inverse": err,
                            "collective": "all_reduce of 32 x 2 int64 fx digits per iteration (RCCL): exact, "
                                          "order-free"}}


def c4_single_gpu(dev, args):
    """C4's cloud size on one GPU (north star: voxel_down_sample +
    estimate_normals at N=50M): the headline step on 50M uniform points."""
    n = args.c4_n
    pts = synthetic.uniform_cube(n, seed=0, device=dev)
    vs = synthetic.voxel_size_for(n)

    def step():
        return ops.voxel_down_sample_normals(pts, vs, knn=args.knn)["rep_idx"].numel()

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


def f64_las(dev, args):
    """The float64 boundary at C2's size: a 10M-point LAS-like scan (box
    surface at a ~5e5 m offset, full-mantissa float64 that float32 cannot
    hold) through voxel_down_sample (5 cm) + KNN30 normals on the
    representatives, both on the float64 kernels (o3dx_*_f64); beside it the
    same scan re-centred and rounded to float32 (the float32 kernels).
    tools/f64_time.py times the whole chain (RANSAC, ICP too)."""
    n = args.n
    las = synthetic.las_scene(n, seed=0, device=dev)
    x0 = torch.tensor(synthetic.LAS_OFFSET, dtype=torch.float64, device=dev)
    out = {}
    for tag, pts in (("f64", las), ("f32_recentred", (las - x0).float())):
        def step():
            reps = ops.voxel_down_sample(pts, 0.05)["rep_xyz"]
            return reps, ops.estimate_normals(reps, knn=args.knn)

        step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(3):
            reps, _nrm = step()
        torch.cuda.synchronize(dev)
        el = (time.perf_counter() - t0) / 3
        out[tag] = {"ms": round(el * 1e3, 3), "voxels": int(reps.shape[0]),
                    "Mpoints_per_s": round(n / el / 1e6, 2)}
        del reps, _nrm, pts
    del las
    torch.cuda.empty_cache()
    out["note"] = "two library calls (voxel_down_sample, estimate_normals) per step, 5 cm voxels, KNN30"
    return {"f64_las": out}


def c5_pipeline(dev, args):
    """C5's full pipeline on one GPU (200M points fit one MI355X's HBM):
    a 200M-point box-surface scene and an independent 200M-point sample of it
    moved by T_gt -> voxel_down_sample both (vs 0.5 mm) -> KNN30 normals on the
    target reps -> segment_plane (1000 hypotheses) on the target reps ->
    point-to-plane ICP source reps -> target reps, 30 iterations from T = I.

    The chain runs twice on the same clouds: an untimed warm-up (its stages
    are reported as `first_call_stages_ms`: the workspaces' first allocation
    and first touch after the C4 leg's empty_cache land there — the 521 ms
    voxel_target of BENCH_r03), then the timed run, as every other leg."""
    n = args.c5_n
    vs = 0.0005
    res = {"n": n, "voxel_size": vs}

    tgt = synthetic.box_surface(n, seed=1, device=dev)
    src = synthetic.apply_transform(synthetic.box_surface(n, seed=2, device=dev), synthetic.rigid_transform())
    samples = None

    def chain(stages):
        nonlocal samples

        def timed(name, fn):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize(dev)
            stages[name] = round((time.perf_counter() - t0) * 1e3, 3)
            return r

        torch.cuda.synchronize(dev)
        t_all = time.perf_counter()
        vt = timed("voxel_target", lambda: ops.voxel_down_sample(tgt, vs, keep_grid=True))
        vsrc = timed("voxel_source", lambda: ops.voxel_down_sample(src, vs))
        treps, sreps = vt["rep_xyz"], vsrc["rep_xyz"]
        tn = timed("normals_target", lambda: ops.estimate_normals(treps, knn=30, voxel_grid=vt.get("voxel_grid")))
        if samples is None:
            samples = ops.ransac_samples(treps.shape[0], 3, args.ransac_iters, seed=7)
        plane, inl = timed("segment_plane", lambda: ops.segment_plane(treps, 0.002, 3, args.ransac_iters,
                                                                      samples=samples))

        def icp():
            target = ops.ICPTarget(treps, tn, 0.02)
            s4 = ops.spatial_sort(sreps)
            return target.register(s4, max_iteration=args.icp_iters, relative_fitness=0.0, relative_rmse=0.0)

        reg = timed("icp_30", icp)
        T = reg["transformation"]
        total = time.perf_counter() - t_all
        return {"target_reps": int(treps.shape[0]), "source_reps": int(sreps.shape[0]), "total_ms":
                round(total * 1e3, 3), "plane": [round(float(v), 6) for v in plane], "plane_inliers": int(inl.numel()),
                "icp_fitness": round(reg["fitness"], 6),
                "T_err_vs_gt_inverse": float(np.abs(T - np.linalg.inv(synthetic.rigid_transform())).max())}

    first = {}
    r0 = chain(first)
    stages = {}
    r1 = chain(stages)
    if (r0["target_reps"], r0["plane_inliers"], r0["plane"]) != (r1["target_reps"], r1["plane_inliers"], r1["plane"]):
        raise RuntimeError("C5: the warm-up and the timed run disagree")
    res.update(r1)
    res.update({"stages_ms": stages, "first_call_stages_ms": first, "first_call_total_ms": r0["total_ms"],
                "Mpoints_per_s_voxel_normals_target":
                round(n / ((stages["voxel_target"] + stages["normals_target"]) * 1e-3) / 1e6, 2),
                "icp_iters_per_s": round(args.icp_iters / (stages["icp_30"] * 1e-3), 2)})
    del tgt, src
    torch.cuda.empty_cache()
    return {"c5_single_gpu": res}


def slab_headline(dev, args, world, rank, n, stretch, vs, timer_filter=None):
    """N > 1 step: ONE uniform-random n-point cloud over [0,stretch) x [0,1)^2,
    each rank's points resident in its voxel-aligned x-slab (a spatially tiled
    dataset; placement untimed), one step =
    open3dpypro.distributed.voxel_normals_slabs(presorted=True).
    stretch = world, vs = C2's: C2 per GPU (weak scaling); stretch = 1: C4
    (one 50M cloud, strong scaling).  Returns (max-over-ranks seconds, global
    reps, this rank's points, rank 0's host timeline of one more step)."""
    from open3dpypro import distributed as D

    full = synthetic.uniform_cube(n, seed=0, device=dev)
    if stretch != 1:
        full[:, 0] *= float(stretch)
    mn, mx = ops.aabb(full)
    keys = D.slab_bounds(mn, mx, vs, world)
    kx = torch.floor((full[:, 0].double() - float(mn[0])) / vs).to(torch.int64)
    gidx = torch.nonzero((kx >= keys[rank]) & (kx < keys[rank + 1])).flatten()
    pts = full[gidx].contiguous()
    del full, kx
    torch.cuda.empty_cache()

    def step():
        return D.voxel_normals_slabs(pts, gidx, vs, knn=args.knn, presorted=True)

    for _ in range(args.warmup):
        rg, _, _ = step()
    _native.reset_kernel_timing()
    _native.kernel_timing_filter(timer_filter)
    _native.set_kernel_timing(not args.no_kernel_events)
    barrier(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rg, _, _ = step()
    barrier(world, dev)
    t1 = time.perf_counter()
    _native.set_kernel_timing(False)
    _native.kernel_timing_filter(None)
    elapsed = max_over_ranks(t1 - t0, world, dev)
    m = torch.tensor([rg.numel()], dtype=torch.int64, device=comm_dev(dev))
    dist.all_reduce(m)
    # one more (untimed) step with host timestamps at each phase end: where
    # the host waits (bounds, verdict) and what they cost
    barrier(world, dev)
    tl = {}
    t2 = time.perf_counter()
    D.voxel_normals_slabs(pts, gidx, vs, knn=args.knn, presorted=True, timings=tl)
    tl["returned"] = round((time.perf_counter() - t2) * 1e3, 4)
    torch.cuda.synchronize()
    tl["synchronized"] = round((time.perf_counter() - t2) * 1e3, 4)
    n_local = int(pts.shape[0])
    del pts, gidx
    torch.cuda.empty_cache()
    return elapsed, int(m.item()), n_local, tl


def c5_sharded(dev, args, world, rank):
    """C5 over the ranks (BASELINE configs[4]): 200M-point box-surface target
    and an independent 200M sample of it moved by T_gt, each a spatially
    tiled dataset (every rank holds its x-slab; placement untimed), one pass =
    open3dpypro.distributed.pipeline_sharded: slab voxel reps + KNN30 normals
    of the target (halo exchange), slab voxel reps of the source,
    segment_plane 1000 hypotheses with the reps sharded (exact count / fx
    all-reduces), 30 ICP iterations with the source sharded and the fx
    moments all-reduced per iteration (RCCL).  Bit-identical to one GPU
    (tests/test_gpu_distributed.py::test_c5_pipeline_sharded_matches_single)."""
    from open3dpypro import distributed as D

    n = args.c5_n
    vs = 0.0005

    def tile(c):
        mn, mx = ops.aabb(c)
        keys = D.slab_bounds(mn, mx, vs, world)
        kx = torch.floor((c[:, 0].double() - float(mn[0])) / vs).to(torch.int64)
        owner = torch.searchsorted(torch.tensor(keys[1:-1], dtype=torch.int64, device=dev), kx, right=True)
        counts = torch.bincount(owner, minlength=world).cpu().tolist()
        own = torch.nonzero(owner == rank).flatten()
        start = sum(counts[:rank])
        return c[own].contiguous(), torch.arange(start, start + own.numel(), dtype=torch.int64, device=dev)

    t = synthetic.box_surface(n, seed=1, device=dev)
    tgt, tg = tile(t)
    del t
    s_ = synthetic.apply_transform(synthetic.box_surface(n, seed=2, device=dev), synthetic.rigid_transform())
    src, sg = tile(s_)
    del s_
    torch.cuda.empty_cache()

    def run(timings=None):
        return D.pipeline_sharded(tgt, tg, src, sg, vs, knn=30, distance_threshold=0.002,
                                  num_iterations=args.ransac_iters, seed=7, max_correspondence_distance=0.02,
                                  icp_iterations=args.icp_iters, presorted=True, timings=timings)

    run()  # warm
    barrier(world, dev)
    t0 = time.perf_counter()
    out = run()
    barrier(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    stages = {}
    run(stages)  # per-stage breakdown (synchronised stages; not the timed pass)
    res = {"n": n, "voxel_size": vs, "ranks": world, "ms": round(el * 1e3, 3),
           "Mpoints_per_s_target": round(n / el / 1e6, 2), "target_reps": out["target_reps"],
           "source_reps": out["source_reps"], "plane": [round(float(v), 6) for v in out["plane"]],
           "icp_fitness": round(out["fitness"], 6),
           "T_err_vs_gt_inverse": float(np.abs(out["transformation"] - np.linalg.inv(synthetic.rigid_transform())).max()),
           "stages_ms_rank0": stages,
           "collectives": "all_reduce (bounds, counts, fx digit sums, halo proof), all_to_all (halo reps; the "
                          "ICP target rows within reach of each rank's source: distributed.WindowedTarget), "
                          "all_gather (source boxes)"}
    del tgt, src, tg, sg, out
    torch.cuda.empty_cache()
    return {"c5_sharded": res}


def kernel_table():
    kernels = {}
    for name in ("voxel_assign", "voxel_compact", "grid_count", "grid_sort", "normals_stile", "normals_tile",
                 "normals_wave", "normals_knn"):
        ms, cnt = _native.kernel_timing(name)
        if cnt:
            kernels[name] = {"avg_ms": round(ms / cnt, 4), "launches": cnt}
    return kernels


# VALU instruction mix of the dominant kernels (fractions of their VALU
# instructions; static count over the disassembly of the launched variant,
# tools/valu_mix.py -> profiles/r02_valu_mix.json)
VALU_MIX = {"normals_stile": {"pk": 1476 / 9328, "f64": 1337 / 9328, "trans": 67 / 9328}}


def roofline(kernels, M, N, pmc_json):
    # algorithmic bytes per launch:
    #   normals_stile / normals_tile: M queries x (12 B xyz read + 12 B normal written)
    #   voxel_assign: N points x (12 B xyz read + 4 B voxel id written)
    algo_bytes = {"normals_stile": 24.0 * M, "normals_tile": 24.0 * M, "voxel_assign": 16.0 * N}
    dom = max((k for k in kernels if k in algo_bytes), key=lambda k: kernels[k]["avg_ms"], default=None)
    if dom is None:
        return None
    avg_s = kernels[dom]["avg_ms"] * 1e-3
    ach = algo_bytes[dom] / avg_s / 1e9
    pmc = pmc_entry(pmc_json, dom)
    roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": pmc.get("hbm_bytes_per_launch"),
            "algorithmic_bytes_per_launch": algo_bytes[dom],
            "note": "exact kNN selection is LDS / VALU-issue work, not HBM streaming: DESIGN.md §4.1"}
    if pmc.get("SQ_INSTS_VALU") and dom.startswith("normals"):
        # the headline stays SURVEY 8(d)'s algorithmic bytes / HBM peak; the
        # measured limit (PMC) is VALU issue, reported beside it: the launch's
        # VALU wave-instructions / its duration against one wave64 VALU
        # instruction per 2 cycles per SIMD (MI355X_MICROARCH.md), 1024 SIMDs at 2.4 GHz
        valu_peak = 1024 * 2.4e9 / 2.0 / 1e9
        valu_ach = pmc["SQ_INSTS_VALU"] / avg_s / 1e9
        roof["valu"] = {"achieved": round(valu_ach, 2), "peak": valu_peak, "unit": "G wave64-VALU-instr/s",
                        "frac": round(valu_ach / valu_peak, 4)}
        roof["note"] = ("exact kNN selection is VALU-issue / LDS work, not HBM streaming: the kernel's own limit "
                        "is the `valu` block (PMC in profiles/pmc_traffic.json; DESIGN.md §4.1)")
    if pmc.get("SQ_INSTS_VALU"):
        # VALU-issue floor (MI355X_MICROARCH.md: a wave64 VALU instruction issues in 2 cycles on a SIMD
        # holding >= 2 waves; float64 / transcendental ones take longer, so this is a lower bound)
        floor_ms = pmc["SQ_INSTS_VALU"] * 2.0 / (1024 * 2.4e9) * 1e3
        roof["valu_issue_floor_ms"] = round(floor_ms, 4)
        roof["valu_issue_frac"] = round(floor_ms / kernels[dom]["avg_ms"], 4)
        mix = VALU_MIX.get(dom)
        if mix:
            # weighted by the kernel's instruction mix (static count from its disassembly,
            # profiles/r02_valu_mix.json): packed f32 and f64 at 4 cycles, transcendental 8,
            # the rest 2 (the FP32 vector peak is the non-packed v_fma_f32 rate)
            cyc = 2.0 * (1 - mix["pk"] - mix["f64"] - mix["trans"]) + 4.0 * (mix["pk"] + mix["f64"]) + 8.0 * mix["trans"]
            wf = pmc["SQ_INSTS_VALU"] * cyc / (1024 * 2.4e9) * 1e3
            roof["valu_issue_floor_weighted_ms"] = round(wf, 4)
            roof["valu_issue_weighted_frac"] = round(wf / kernels[dom]["avg_ms"], 4)
    if pmc.get("SQ_LDS_IDX_ACTIVE") and pmc.get("GRBM_GUI_ACTIVE"):
        # LDS busy share: SQ_LDS_IDX_ACTIVE (LDS-array cycles, summed over CUs) / (256 CUs x kernel cycles)
        cyc = pmc["GRBM_GUI_ACTIVE"] / 8.0  # GRBM_GUI_ACTIVE sums the 8 XCDs
        roof["lds_busy_frac"] = round(pmc["SQ_LDS_IDX_ACTIVE"] / (256.0 * cyc), 4)
        if pmc.get("SQ_LDS_BANK_CONFLICT") is not None:
            roof["lds_conflict_frac"] = round(pmc["SQ_LDS_BANK_CONFLICT"] / pmc["SQ_LDS_IDX_ACTIVE"], 4)
    return roof


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args)  # before anything touches a GPU
    if args.dry_run:
        return dry_run(args)
    world, rank, dev = setup_dist(args.dist_icp)
    if world > 1:
        return main_multi(args, world, rank, dev)
    N = args.n
    vs = synthetic.voxel_size_for(N)
    pts = synthetic.uniform_cube(N, seed=0, device=dev)
    torch.cuda.synchronize(dev)
    keep = not args.sorted_grid

    def step_two_call():
        # PointCloud.voxel_down_sample(vs).estimate_normals(): the voxel table
        # of the first call is the search grid of the second
        out = ops.voxel_down_sample(pts, vs, keep_grid=keep)
        nrm = ops.estimate_normals(out["rep_xyz"], knn=args.knn, voxel_grid=out.get("voxel_grid"))
        return out["rep_idx"].numel(), nrm

    def step_fused():
        # the same pipeline as one library call: the normals are queued behind
        # the voxel kernels before the representative count is read back
        out = ops.voxel_down_sample_normals(pts, vs, knn=args.knn)
        return out["rep_idx"].numel(), out["normals"]

    step = step_two_call if (args.two_call or not keep) else step_fused

    for _ in range(args.warmup):
        M, _ = step()
    # the timed region records HIP events around the dominant kernel only
    # (every extra event pair adds launch-path work to the pipeline); the
    # per-kernel breakdown is a separate, untimed pass below
    _native.reset_kernel_timing()
    _native.kernel_timing_filter(["normals_stile"])
    _native.set_kernel_timing(not args.no_kernel_events)
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
    elapsed = t1 - t0
    ev_ms = ev0.elapsed_time(ev1)
    dom = kernel_table()
    _native.kernel_timing_filter(None)
    _native.reset_kernel_timing()
    _native.set_kernel_timing(True)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    _native.set_kernel_timing(False)
    kernels = kernel_table()  # breakdown (all timers on; not the timed region)
    if dom:
        kernels.update(dom)   # the dominant kernel as timed inside the timed region
    value = float(N) * args.steps / elapsed / 1e6
    other = step_two_call if step is step_fused else (step_fused if keep else None)
    other_ms = None
    if other is not None:  # the other call structure, same pipeline, for the record
        other()
        torch.cuda.synchronize(dev)
        ta = time.perf_counter()
        for _ in range(args.steps):
            other()
        torch.cuda.synchronize(dev)
        other_ms = round((time.perf_counter() - ta) / args.steps * 1e3, 3)
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "Mpoints/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak",  # the first point of the --gpus N weak curve (C2 per GPU)
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C2: uniform-random 10M pts float32, voxel_down_sample(vs=(4/N)^(1/3)) "
                               "+ estimate_normals(KNN30) on the representatives",
                   "n_points": N, "voxel_size": vs, "voxels": int(M), "knn": args.knn, "parallelism": "single"},
        "roofline": roofline(kernels, M, N, args.pmc_json),
        "cpu_baseline": None,
        "extra": {"stream_event_ms_per_step": round(ev_ms / args.steps, 3), "kernels": kernels,
                  "call_structure": "one call (o3dx_voxel_down_sample_normals)" if step is step_fused
                  else "two calls (voxel_down_sample, estimate_normals)",
                  ("two_call_ms_per_step" if step is step_fused else "one_call_ms_per_step"): other_ms,
                  "pipeline_algorithmic_GBs": round((12.0 * N + 28.0 * M) * args.steps / elapsed / 1e9, 2),
                  "storage_dtype": "f32", "arith": "float64 voxel keys / distances / covariance"},
    }
    if not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args.cpu_n, pts)
        if line["cpu_baseline"]["value"] > 0:
            line["extra"]["gpu_over_cpu"] = round(value / line["cpu_baseline"]["value"], 1)
    del pts
    torch.cuda.empty_cache()
    if args.scaling_child and args.c4_n > 0:  # one point of the --gpus N curve: C2 + C4 only
        try:
            line["extra"].update(c4_single_gpu(dev, args))
        except RuntimeError as e:
            line["extra"]["c4_error"] = str(e)
    elif not args.no_secondary:
        for name, fn in (("secondary", lambda: secondary(dev, args)),
                         ("c4", lambda: c4_single_gpu(dev, args) if args.c4_n > 0 else {}),
                         ("c5", lambda: c5_pipeline(dev, args) if args.c5_n > 0 else {}),
                         ("f64_las", lambda: f64_las(dev, args))):
            try:
                line["extra"].update(fn())
            except RuntimeError as e:  # report, never hide
                line["extra"][f"{name}_error"] = str(e)
            torch.cuda.empty_cache()
        if args.dist_icp:
            line["extra"].update(secondary_sharded_icp(dev, args, world, rank))
        if not args.no_cpu:
            try:
                tn = ops.estimate_normals(synthetic.box_surface(args.icp_n, seed=1, device=dev), knn=30)
                line["extra"].update(cpu_secondary(dev, args, tn))
            except RuntimeError as e:
                line["extra"]["cpu_secondary_error"] = str(e)
            ex = line["extra"]
            if "cpu_ransac" in ex and "ransac" in ex:
                ex["cpu_ransac"]["gpu_over_cpu"] = round(ex["cpu_ransac"]["seconds"] * 1e3 / ex["ransac"]["ms"], 1)
            if "cpu_icp" in ex and "icp" in ex:
                ex["cpu_icp"]["gpu_over_cpu"] = round(ex["icp"]["iters_per_s"] / ex["cpu_icp"]["iters_per_s"], 1)
    print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def main_multi(args, world, rank, dev):
    """N > 1 ranks: the headline is C2 per GPU (weak scaling: one N x 10M
    cloud over [0,N) x [0,1)^2 in x-slabs, C2's voxel size); beside it C4 (one
    50M cloud over the same ranks: strong scaling), the sharded ICP and C5."""
    n_per = args.n
    N = n_per * world
    vs = synthetic.voxel_size_for(n_per)
    elapsed, M, n_local, tl = slab_headline(dev, args, world, rank, N, world, vs)
    kernels = kernel_table()
    # host/kernel split of the step: the library's event-timed kernel spans
    # (voxel, compaction, normals) per step on this rank, summed over the ranks
    # (on a shared GPU the ranks' kernels serialise, so the step is at least
    # their sum); host = the rest of the wall time (collectives, launches, syncs)
    k_ms = sum(v["avg_ms"] * v["launches"] for v in kernels.values()) / max(args.steps, 1)
    k_all = torch.tensor([k_ms], dtype=torch.float64, device=comm_dev(dev))
    dist.all_reduce(k_all, op=dist.ReduceOp.SUM)
    k_all = float(k_all.item())
    wall = elapsed / args.steps * 1e3
    shared = os.environ.get("O3DX_BENCH_SHARED_GPU") == "1"
    busy = k_all if shared else k_ms
    value = float(N) * args.steps / elapsed / 1e6
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "Mpoints/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"C2 per GPU: one uniform-random {world} x {n_per // 1_000_000}M-pt float32 cloud over "
                               f"[0,{world})x[0,1)^2 (C2's density) tiled over {world} GPUs as voxel-aligned x-slabs, "
                               "voxel_down_sample(vs=C2's (4/10M)^(1/3)) + estimate_normals(KNN30) with a verified "
                               "halo exchange of boundary representatives over RCCL",
                   "n_points": N, "points_per_gpu": n_per, "voxel_size": vs, "voxels": M, "knn": args.knn,
                   "parallelism": f"x-slab spatial tiling x{world}", "points_rank0": n_local},
        "roofline": (None if os.environ.get("O3DX_BENCH_SHARED_GPU") == "1"  # ranks sharing one GPU: no roofline
                     else roofline(kernels, M / world, N / world, args.pmc_json)),
        "cpu_baseline": None,
        "extra": {"kernels_rank0": kernels,
                  "world_size_observed": dist.get_world_size(), "backend": dist.get_backend(),
                  "step_breakdown": {"wall_ms": round(wall, 4), "kernel_ms_rank0": round(k_ms, 4),
                                     "kernel_ms_all_ranks": round(k_all, 4), "gpu_shared_by_ranks": shared,
                                     "host_frac": round(max(0.0, 1.0 - busy / wall), 4) if wall > 0 else None},
                  "collectives": "all_reduce (AABB + counts), all_to_all (halo representatives), all_gather "
                                 "(halo-proof verdict)",
                  "host_timeline_rank0_ms": tl,
                  "pipeline_algorithmic_GBs": round((12.0 * N + 28.0 * M) * args.steps / elapsed / 1e9, 2)},
    }
    if args.c4_n > 0:
        try:
            n4 = args.c4_n
            el4, m4, nl4, tl4 = slab_headline(dev, args, world, rank, n4, 1, synthetic.voxel_size_for(n4),
                                              timer_filter=["normals_stile"])
            line["extra"]["c4_strong"] = {"n": n4, "ranks": world, "voxels": m4, "points_rank0": nl4,
                                          "ms": round(el4 / args.steps * 1e3, 3),
                                          "value": round(n4 * args.steps / el4 / 1e6, 2), "unit": "Mpoints/s",
                                          "scaling": "strong", "host_timeline_rank0_ms": tl4}
        except RuntimeError as e:  # report, never hide
            line["extra"]["c4_error"] = str(e)
    torch.cuda.empty_cache()
    if not args.no_secondary and not args.scaling_child:
        for name, fn in (("icp_sharded", lambda: secondary_sharded_icp(dev, args, world, rank)),
                         ("c5", lambda: c5_sharded(dev, args, world, rank) if args.c5_n > 0 else {})):
            try:
                line["extra"].update(fn())
            except RuntimeError as e:  # report, never hide
                line["extra"][f"{name}_error"] = str(e)
            torch.cuda.empty_cache()
    if rank == 0:
        print(json.dumps(line), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def dry_run(args):
    """--dry-run: the launch plumbing without a GPU (gloo on the CPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    seen = 1
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        t = torch.ones(1, dtype=torch.int64)
        dist.all_reduce(t)
        seen = int(t.item())
    line = {"metric": METRIC, "value": float(seen), "unit": "Mpoints/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1.0, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "dry-run", "config": {"workload": "dry-run"},
            "roofline": None, "cpu_baseline": None,
            "extra": {"world_size_observed": seen, "scaling_child": args.scaling_child, "no_cpu": args.no_cpu,
                      "local_rank": os.environ.get("LOCAL_RANK"), "c4_single_gpu": {"Mpoints_per_s": 1.0},
                      "c4_strong": {"value": float(seen)}}}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _rank_counts(n: int):
    """1, 2, 4, ... below n, then n itself"""
    out, c = [1], 2
    while c < n:
        out.append(c)
        c *= 2
    return out + ([n] if n > 1 else [])


def _strip_gpus(argv):
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == "--gpus":
            skip = True
            continue
        if a.startswith("--gpus="):
            continue
        out.append(a)
    return out


def _run_ranks(n, argv, timeout_s):
    """One point of the curve: n fresh processes (one per GPU, LOCAL_RANK =
    rank, RCCL rendezvous on 127.0.0.1), rank 0's JSON line back.  A rank
    that fails or overruns ends the whole group (its PIDs, never a pattern)."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        if n > 1:
            env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        else:
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
                env.pop(k, None)
        cmd = [sys.executable, "-u", os.path.abspath(__file__), "--gpus", str(n)] + argv
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out0 = []
    import threading

    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    deadline = time.time() + timeout_s
    err = None
    while True:
        codes = [p.poll() for p in procs]
        if all(c is not None for c in codes):
            if any(codes):
                err = f"{n} ranks: exit codes {codes}"
            break
        if any(c not in (None, 0) for c in codes):
            err = f"{n} ranks: exit codes {codes} (the rest stopped)"
            break
        if time.time() > deadline:
            err = f"{n} ranks: over {timeout_s}s (stopped)"
            break
        time.sleep(0.5)
    if err:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
    reader.join(timeout=30)
    text = out0[0].decode() if out0 and out0[0] else ""
    lines = [ln for ln in text.splitlines() if ln.startswith("{")]
    if err or not lines:
        return None, err or f"{n} ranks: no result line"
    return json.loads(lines[-1]), None


def launch(args):
    """python bench.py --gpus N with no WORLD_SIZE: the 1 -> N scaling curve in
    one run.  This process never initialises a GPU (children only); it starts
    one fresh process per GPU for each rank count in turn (1, 2, 4, ... N),
    each rank count a separate rendezvous, and prints one line: the N-rank
    figures, `scaling_curve` (per count: value, ms, efficiency =
    value_n / (n x value_1)) and the CPU baseline, timed here after the GPU
    runs (reference precedent for one process per device:
    processors.py:204-208, :1088-1098)."""
    N = args.gpus
    base = _strip_gpus(sys.argv[1:])
    runs, errors = {}, []
    for n in _rank_counts(N):
        argv = list(base) + ["--no-cpu"] + ([] if n == N else ["--scaling-child"])
        log(f"bench launcher: {n} rank(s)")
        line, err = _run_ranks(n, argv, args.child_timeout)
        if err:
            errors.append(err)
            log("bench launcher:", err)
            break  # nothing more on the GPU after a failed run
        runs[n] = line
    if N in runs:
        line = runs[N]
    else:
        line = {"metric": METRIC, "value": None, "unit": "Mpoints/s", "n_gpus": N, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "f64", "data": "synthetic", "config": {}, "roofline": None,
                "cpu_baseline": None, "extra": {}}
    weak, c4 = {}, {}
    v1 = runs.get(1, {}).get("value")
    c41 = runs.get(1, {}).get("extra", {}).get("c4_single_gpu", {}).get("Mpoints_per_s")
    for n, ln in sorted(runs.items()):
        v = ln.get("value")
        weak[str(n)] = {"value": v, "ms_per_step": ln.get("ms_per_step"),
                        "efficiency": round(v / (n * v1), 4) if (v and v1) else None}
        cv = (ln.get("extra", {}).get("c4_single_gpu", {}).get("Mpoints_per_s") if n == 1
              else ln.get("extra", {}).get("c4_strong", {}).get("value"))
        c4[str(n)] = {"value": cv, "efficiency": round(cv / (n * c41), 4) if (cv and c41) else None}
    line["scaling_curve"] = {"unit": "Mpoints/s", "weak_c2_per_gpu": weak, "strong_c4_50M": c4,
                             "note": "1 rank = the single-GPU C2 step (one-call pipeline); n > 1 = the x-slab step "
                                     "with the halo exchange over RCCL; efficiency = value_n / (n x value_1)"}
    line["launcher"] = {"form": "bench.py --gpus N: fresh child processes per rank count, one per GPU",
                        "rank_counts": sorted(runs), "errors": errors}
    if not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args.cpu_n)
        if line.get("value") and line["cpu_baseline"]["value"] > 0:
            line.setdefault("extra", {})["gpu_over_cpu"] = round(line["value"] / line["cpu_baseline"]["value"], 1)
    print(json.dumps(line), flush=True)
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main() or 0)
