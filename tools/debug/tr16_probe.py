import os, sys
sys.path.insert(0, os.getcwd())
import torch
from deep_graph_matching_consensus_amd.ops import _backend
assert _backend.hip_available()
o = _backend.ops().tr16_probe(torch.empty(1, device='cuda')).cpu()
for l in range(0, 64):
    print(l, o[l].tolist())
