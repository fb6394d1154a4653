"""psi_1's large weight gradients (``[1024 x 6656]``, ``[256 x 6656]`` over
K = 11k rows): the MFMA TN kernel (``dense_wgrad``, split over row chunks)
vs the library path (``matmul_tn_fp32``: hipBLASLt, split-K when small)."""
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))
from deep_graph_matching_consensus_amd.ops import dense as D
from deep_graph_matching_consensus_amd.ops.gemm import matmul_tn_fp32
def t(f, n=10):
    for _ in range(3): f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(n): f()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1000
for K, M, N in [(11008, 1024, 6656), (11008, 256, 6656), (10304, 1024, 6656)]:
    x = torch.randn(K, M, device='cuda').bfloat16()
    g = torch.randn(K, N, device='cuda').bfloat16()
    ref = matmul_tn_fp32(x, g)
    us0 = t(lambda: matmul_tn_fp32(x, g))
    res = {}
    for ns in (1, 2, 3):
        out = D.dense_wgrad([x], [g], nsplit=ns)
        err = (out - ref).abs().max().item() / ref.abs().max().item()
        res[ns] = (t(lambda: D.dense_wgrad([x], [g], nsplit=ns)), err)
    rest = ' '.join('dw%d %.1f us (err %.1e)' % (k, v[0], v[1])
                    for k, v in res.items())
    print(K, M, N, 'lib %.1f us' % us0, rest, flush=True)
