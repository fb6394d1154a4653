"""Diagnostic: per-lane transposed fragments of the bf16x6 weight gradient
(DGMC_X6_DEBUG=8): run once with X = row index and once with X = column
index; lane l must hold rows 8 (l >> 5) + j of column l & 31."""
import os
import os.path as osp
import sys

import torch

os.environ['DGMC_X6_DEBUG'] = os.environ.get('XDBG', '8')
sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..', '..'))
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402

dev = 'cuda'
ops = _backend.ops()
P = 256
src = torch.arange(P, dtype=torch.int32, device=dev)
seg = torch.tensor([0, P], dtype=torch.int32, device=dev)
R = torch.arange(P, device=dev, dtype=torch.float32)[:, None].repeat(1, 128)
Cc = torch.arange(128, device=dev, dtype=torch.float32)[None].repeat(P, 1)
out = {}
for name, X in (('row', R), ('col', Cc)):
    part = ops.slot_wgrad_x6([ops.split3(X)], [ops.split3(X)], src, seg, 1)
    out[name] = part.view(-1).view(torch.bfloat16)[:64 * 16].float().view(
        64, 16)[:, 8:]
for l in (0, 1, 4, 5, 8, 12, 16, 31, 32, 48):
    print('lane %2d rows %s cols %s' % (l, out['row'][l].int().tolist(),
                                       out['col'][l].int().tolist()))
print('offX[0][0] lanes 0..15:', part.view(-1)[1024:1040].int().tolist())
print('offX[0][1] lanes 0..15:', part.view(-1)[1088:1104].int().tolist())
flat = part.view(-1)
print('tr address bytes lanes 0..15:', flat[1152:1168].long().tolist())
print('ring base bytes lane 0:', int(part.view(-1)[1216]))
pl = part.view(-1)[1280:1280 + 256].view(64, 4)
print('plain 8-B read at each lane address (last run), lanes 0..7:',
      pl[:8].int().tolist())
