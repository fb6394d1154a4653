"""Cold top-k filter on the DBP15K zh_en shape, a few calls (a short driver
for rocprofv3 counter passes: tools/gpu_r6_ae.sh)."""
import os.path as osp
import sys

sys.path.insert(0, osp.dirname(osp.dirname(osp.dirname(osp.abspath(
    __file__)))))

import torch  # noqa: E402

from deep_graph_matching_consensus_amd.ops import sparse_corr  # noqa: E402

g = torch.Generator(device='cuda').manual_seed(0)
Ns, Nt, C = 19388, 19572, 256
h_s = torch.randn(1, Ns, C, device='cuda', generator=g)
h_t = torch.randn(1, Nt, C, device='cuda', generator=g)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    sparse_corr.top_k(h_s, h_t, 10)
torch.cuda.synchronize()
print('ok')
