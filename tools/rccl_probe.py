"""RCCL sanity probe: all-reduce / all-gather / all-to-all across the ranks of one torchrun job
(one rank per GPU; on a one-GPU box every rank shares cuda:0).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tools/rccl_probe.py
"""
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % ndev)
    dist.init_process_group("nccl")
    x = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    g = [torch.empty(4, device="cuda") for _ in range(world)]
    dist.all_gather(g, torch.full((4,), float(rank), device="cuda"))
    a2a = torch.empty(world * 2, device="cuda")
    dist.all_to_all_single(a2a, torch.arange(world * 2, device="cuda", dtype=torch.float32) + 100 * rank)
    torch.cuda.synchronize()
    ok = bool(x[0].item() == world * (world + 1) / 2) and all(bool((t == i).all()) for i, t in enumerate(g))
    print(f"rank {rank}/{world} devices={ndev} allreduce={x[0].item()} gather_ok={ok} a2a={a2a.tolist()}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
