"""Dev: can two RCCL ranks share one GPU on this box?  (world 2, both on cuda:0)."""
import os
import torch
import torch.distributed as dist
rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
t = torch.ones(4, device="cuda:0") * (rank + 1)
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce -> {t.tolist()}", flush=True)
dist.destroy_process_group()
