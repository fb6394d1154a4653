"""Diagnostic: operand-pairing map of the bf16x6 weight gradient.
X = identity rows, G[p][c] = p (+ 0.5 c for c < 2): dW[i][c] must equal
G[i][c]; prints the first rows / columns of what comes out."""
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..', '..'))
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402

dev = 'cuda'
ops = _backend.ops()
P = 256
src = torch.arange(P, dtype=torch.int32, device=dev)
seg = torch.tensor([0, P], dtype=torch.int32, device=dev)
X = torch.zeros(P, 128, device=dev)
X[torch.arange(128), torch.arange(128)] = 1.0
G = torch.arange(P, device=dev, dtype=torch.float32)[:, None].repeat(1, 128)
G = G + torch.arange(128, device=dev)[None] * 0.0
G[:, 1] += 1000.0
w = ops.slot_wgrad_x6([ops.split3(X)], [ops.split3(G)], src, seg, 1)[0]
ref = X.t() @ G
print('max err', float((w - ref).abs().max()))
torch.set_printoptions(linewidth=200)
print('dW[0:40, 0] (want 0..39):', w[:40, 0].tolist())
print('dW[0:8, 1] (want 1000..1007):', w[:8, 1].tolist())
print('dW[5, 0:40] (want 5, 1005, 5, ...):', w[5, :40].tolist())
