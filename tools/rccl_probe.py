#!/usr/bin/env python3
"""Can RCCL (backend "nccl") run two ranks on ONE GPU?  If it can, the RCCL device-tensor branch of
afm.sharded.Comm can be exercised on a one-GPU box.  Run under torch.distributed.run:

    timeout -k 10 120 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/rccl_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
print(f"[{rank}] init nccl", flush=True)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((4,), float(rank), device=dev)
out = torch.empty((world, 4), device=dev)
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
print(f"[{rank}] all_gather_into_tensor ok: {out[:, 0].tolist()}", flush=True)
y = torch.arange(world * 2, dtype=torch.float64, device=dev) + 100 * rank
z = torch.empty_like(y)
dist.all_to_all_single(z, y, output_split_sizes=[2] * world, input_split_sizes=[2] * world)
torch.cuda.synchronize()
print(f"[{rank}] all_to_all_single ok: {z.tolist()}", flush=True)
dist.barrier()
dist.destroy_process_group()
sys.exit(0)
