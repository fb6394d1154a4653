"""Split-K sweep for the long-K weight-gradient GEMMs ``a^T b`` (fp32 out).

    python tools/bench_wgrad_tn.py

Shapes: the loop-shared consensus weight gradient (10 uses x 9.2k nodes,
384 x 128) and psi_1's two SplineConv weight gradients.
"""
import json
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))
from deep_graph_matching_consensus_amd.ops import _backend


def timeit(fn, iters=30, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def split(a, b, s, swap=False):
    K, M = a.shape
    N = b.shape[1]
    k = K // s
    if swap:
        a, b, M, N = b, a, N, M
    a3 = a[:k * s].view(s, k, M).transpose(1, 2)
    b3 = b[:k * s].view(s, k, N)
    part = torch.bmm(a3, b3, out_dtype=torch.float32)
    out = torch.empty(M, N, device=a.device)
    _backend.ops().reduce_add_rows(part, out, False)
    return out


def main():
    dev = 'cuda'
    assert _backend.hip_available()
    res = {}
    for name, K, M, N in (('consensus_fold', 92160, 384, 128),
                          ('psi1_l2', 11008, 256, 6656),
                          ('psi1_l1', 11008, 1024, 6656)):
        a = torch.randn(K, M, device=dev).bfloat16()
        b = torch.randn(K, N, device=dev).bfloat16()
        row = {}
        row['mm'] = timeit(lambda: torch.mm(a.t(), b,
                                            out_dtype=torch.float32))
        for s in (2, 4, 8, 16, 32, 64, 128):
            if K // s < 256:
                continue
            row['s%d' % s] = timeit(lambda: split(a, b, s))
            row['s%d_swap' % s] = timeit(lambda: split(a, b, s, True))
        res[name] = {k: round(v, 1) for k, v in row.items()}
        print(json.dumps({name: res[name]}), flush=True)


if __name__ == '__main__':
    main()
