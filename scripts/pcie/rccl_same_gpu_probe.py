"""Can RCCL run two ranks on the box's one GPU?  (If so, bench.py's N > 1
legs can be rehearsed over the real "nccl" backend instead of gloo.)
torchrun --nproc-per-node 2 scripts/pcie/rccl_same_gpu_probe.py"""
import datetime
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=60))
x = torch.full((1 << 20,), float(rank + 1), device=dev)
dist.all_reduce(x)
ok_ar = bool((x == 3.0).all())
y = torch.full((1 << 20,), float(rank), device=dev)
z = torch.empty_like(y)
peer = 1 - rank
reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, y, peer), dist.P2POp(dist.irecv, z, peer)])
for r in reqs:
    r.wait()
torch.cuda.synchronize()
ok_p2p = bool((z == float(peer)).all())
print(f"rank {rank}: all_reduce {ok_ar} p2p {ok_p2p}", flush=True)
dist.destroy_process_group()
