"""RCCL (torch.distributed backend "nccl") on the GPU box: the collective
patterns open3dpypro.distributed uses — SUM all-reduce of int64 fx digits in
place on the device, MAX all-reduce of float64 bounds, all-to-all with split
sizes (halo / target-row exchange), all-gather of a verdict vector — each
checked against its expected value.  Launch under torchrun (any world size;
one GPU per rank):
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/rccl_selftest.py"""
import json
import os

import torch
import torch.distributed as dist


def main():
    rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
    if os.environ.get("RCCL_SELFTEST_GLOO") == "1":  # the same checks on CPU (gloo): tests of this script
        dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    out = {"world": world, "backend": dist.get_backend()}
    # fx digits: exact integer sums, in place, stream-ordered
    d = torch.arange(64, dtype=torch.int64, device=dev) * (rank + 1) + (1 << 40)
    dist.all_reduce(d, op=dist.ReduceOp.SUM)
    exp = torch.arange(64, dtype=torch.int64) * (world * (world + 1) // 2) + world * (1 << 40)
    out["allreduce_int64"] = bool(torch.equal(d.cpu(), exp))
    # bounds: float64 MAX
    b = torch.tensor([float(rank), -float(rank), 0.5], dtype=torch.float64, device=dev)
    dist.all_reduce(b, op=dist.ReduceOp.MAX)
    out["allreduce_max_f64"] = b.cpu().tolist() == [float(world - 1), 0.0, 0.5]
    # all-to-all with split sizes: rank r sends (j + 1) rows of 7 floats to rank j
    ss = [j + 1 for j in range(world)]
    rs = [rank + 1] * world
    send = torch.cat([torch.full((j + 1, 7), float(100 * rank + j), device=dev) for j in range(world)])
    recv = torch.empty((sum(rs), 7), device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=rs, input_split_sizes=ss)
    exp_r = torch.cat([torch.full((rank + 1, 7), float(100 * j + rank)) for j in range(world)])
    out["all_to_all_splits"] = bool(torch.equal(recv.cpu(), exp_r))
    # verdict all-gather
    v = torch.tensor([rank, 1, 2, 3, 4], dtype=torch.int64, device=dev)
    g = [torch.empty_like(v) for _ in range(world)]
    dist.all_gather(g, v)
    out["all_gather"] = all(int(t[0]) == i for i, t in enumerate(g))
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    ok = all(v for k, v in out.items() if k not in ("world", "backend"))
    dist.destroy_process_group()
    raise SystemExit(0 if ok else 1)


if __name__ == "__main__":
    main()
