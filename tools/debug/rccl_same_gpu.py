"""Probe: can two ranks share one GPU under RCCL (for a 2-rank rehearsal of bench.py on a
1-GPU box)?  All-reduce + gather of a small tensor, ranks pinned to device 0."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((4,), float(rank + 1), device=dev)
dist.all_reduce(x)
lst = [torch.empty(4, device=dev) for _ in range(2)] if rank == 0 else None
dist.gather(x, lst, dst=0)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {x.tolist()} gather {[t.tolist() for t in lst] if lst else None}", flush=True)
dist.destroy_process_group()
