"""Diagnostic: one-rank RCCL process group under torch.distributed.run (env://),
an all_reduce and an all_gather_into_tensor; prints each step as it happens."""
import os
import sys
import time

import torch
import torch.distributed as dist


def log(*a):
    print("[%.1fs]" % (time.time() - T0), *a, flush=True)


T0 = time.time()
local = int(os.environ.get("LOCAL_RANK", "0"))
dev = torch.device("cuda", local)
torch.cuda.set_device(dev)
log("init", os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT"), os.environ.get("WORLD_SIZE"))
dist.init_process_group("nccl", device_id=dev)
log("initialised, world", dist.get_world_size())
t = torch.ones(4, device=dev)
dist.all_reduce(t)
torch.cuda.synchronize()
log("all_reduce", t.tolist())
o = torch.empty(4 * dist.get_world_size(), device=dev)
dist.all_gather_into_tensor(o, t)
torch.cuda.synchronize()
log("all_gather ok")
dist.barrier()
log("barrier ok")
dist.destroy_process_group()
log("done")
sys.exit(0)
