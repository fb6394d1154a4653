"""Probe: can two RCCL ranks share the one GPU of a gpurun box?

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 \
        tools/micro/rccl_two_ranks_one_gpu.py

Both ranks use cuda:0.  Prints one JSON line per rank: an eager all-reduce
result, then the same all-reduce captured in a hipGraph and replayed.
"""
import json
import os

import torch
import torch.distributed as dist

rank = int(os.environ['RANK'])
world = int(os.environ['WORLD_SIZE'])
torch.cuda.set_device(0)
dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
x = torch.full((1 << 20,), float(rank + 1), device='cuda')
dist.all_reduce(x)
torch.cuda.synchronize()
eager = x[0].item()
y = torch.full((1 << 20,), float(rank + 1), device='cuda')
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    dist.all_reduce(y)          # warm-up on the capture stream
torch.cuda.current_stream().wait_stream(s)
y.fill_(float(rank + 1))
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    dist.all_reduce(y)
y.fill_(float(rank + 1))
g.replay()
torch.cuda.synchronize()
print(json.dumps({'rank': rank, 'world': world, 'eager': eager,
                  'graph': y[0].item(),
                  'want': world * (world + 1) / 2}), flush=True)
dist.destroy_process_group()
