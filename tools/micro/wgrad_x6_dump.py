"""Diagnostic: dump the first staged LDS plane images of the bf16x6 weight
gradient (DGMC_X6_DEBUG=4) with X = column index; full rows 0 and 1."""
import os
import os.path as osp
import sys

import torch

os.environ['DGMC_X6_DEBUG'] = '4'
sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..', '..'))
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402

dev = 'cuda'
ops = _backend.ops()
P = 256
src = torch.arange(P, dtype=torch.int32, device=dev)
seg = torch.tensor([0, P], dtype=torch.int32, device=dev)
Cc = torch.arange(128, device=dev, dtype=torch.float32)[None].repeat(P, 1)
x3 = ops.split3(Cc)
print('split3 hi row 0 first 16:', x3[0, 0, :16].float().int().tolist())
part = ops.slot_wgrad_x6([x3], [x3], src, seg, 1)
img = part.view(-1).view(torch.bfloat16)[:6 * 16 * 128].float().view(
    6, 16, 128)
print('LDS X hi row 0:', img[0, 0].int().tolist())
print('LDS X hi row 1:', img[0, 1].int().tolist())
