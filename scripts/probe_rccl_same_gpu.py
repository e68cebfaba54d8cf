"""Probe: can two RCCL ranks share one GPU (the 1-GPU box)?  Prints the outcome of one all_reduce."""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    t = torch.full((1 << 20,), float(rank + 1), device=dev)
    t0 = time.time()
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce ok value={t[0].item()} in {time.time()-t0:.3f}s", flush=True)
    out = torch.empty(2 << 20, device=dev)
    dist.all_gather_into_tensor(out, t)
    rs = torch.empty(1 << 19, device=dev)
    dist.reduce_scatter_tensor(rs, t)
    torch.cuda.synchronize()
    print(f"rank {rank}: ag/rs ok {out[0].item()} {rs[0].item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
