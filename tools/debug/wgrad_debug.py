"""Layout debugging for csrc/hip/slot_wgrad.hip (identity operator, one-hot
operands: dW must be a single 1 at (c0, o0))."""
import os
import sys
sys.path.insert(0, os.getcwd())
import torch
from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops.sparse import (SparseOperator,
                                                          slot_weight_grad)
assert _backend.hip_available()
dev = 'cuda'
C, N = 128, 32
ar = torch.arange(N, device=dev)
op = SparseOperator.from_coo(ar, ar, torch.ones(N, device=dev), N, N)
for p0, c0, o0 in [(0, 0, 0), (1, 0, 0), (2, 0, 0), (4, 0, 0), (8, 0, 0),
                   (16, 0, 0), (0, 1, 0), (0, 4, 0), (0, 8, 0), (0, 16, 0),
                   (0, 0, 1), (0, 0, 4), (0, 0, 8), (0, 0, 16), (5, 3, 7)]:
    X = torch.zeros(N, C, device=dev)
    G = torch.zeros(N, C, device=dev)
    X[p0, c0] = 1
    G[p0, o0] = 1
    dW = slot_weight_grad(X.bfloat16(), G.bfloat16(), op, 1, 1, nsplit=1)[0]
    nz = dW.nonzero().tolist()
    print((p0, c0, o0), '->', nz[:6], [dW[i, j].item() for i, j in nz[:6]])
