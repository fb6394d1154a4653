"""Micro-benchmark of the per-pair dense kernels (csrc/hip/dense_consensus.hip)
at PascalVOC bench shapes, swept over the number of pairs B (fixed cost vs
per-block cost).  GPU only.

    python tools/bench_pair_kernels.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                '..'))
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000.0


def main():
    assert _backend.hip_available()
    ops = _backend.ops()
    dev = 'cuda'
    R, N = 128, 19
    for B in (1, 8, 64, 256, 512, 1024, 2048):
        n = torch.randint(5, N + 1, (B, ))
        n[0] = N
        ptr = torch.zeros(B + 1, dtype=torch.int32)
        ptr[1:] = torch.cumsum(n, 0)
        ptr = ptr.to(dev)
        rows = int(ptr[-1])
        S_hat = torch.randn(B, N, N, device=dev)
        P = torch.randn(rows, R, device=dev).bfloat16()
        Q = torch.randn(rows, R, device=dev).bfloat16()
        b1 = torch.randn(R, device=dev)
        w2 = torch.randn(R, device=dev)
        b2 = torch.randn(1, device=dev)
        G = torch.randn(B, N, N, device=dev)
        r_s = torch.randn(rows, R, device=dev).bfloat16()
        t = {}
        t['cons_fwd'] = timeit(lambda: ops.dense_consensus(
            S_hat, P, Q, b1, w2, b2, ptr, ptr))
        t['cons_bwd'] = timeit(lambda: ops.dense_consensus_bwd(
            G, P, Q, b1, w2, ptr, ptr, None))
        S, r_t = ops.dense_softmax_transport(S_hat, r_s, ptr, ptr, rows, False)
        t['trans_fwd'] = timeit(lambda: ops.dense_softmax_transport(
            S_hat, r_s, ptr, ptr, rows, True))
        t['trans_bwd'] = timeit(lambda: ops.dense_softmax_transport_bwd(
            S, r_s, r_t, ptr, ptr))
        t['fused_fwd'] = timeit(lambda: ops.dense_consensus_transport(
            S_hat, P, Q, b1, w2, b2, r_s, ptr, ptr, rows))
        t['fused_bwd'] = timeit(lambda: ops.dense_transport_consensus_bwd(
            S, r_s, r_t, G, P, Q, b1, w2, ptr, ptr, None))
        t['empty_like'] = timeit(lambda: torch.empty_like(S_hat).fill_(0))
        print('B=%5d ' % B + ' '.join('%s=%.1fus' % kv for kv in t.items()),
              flush=True)


if __name__ == '__main__':
    main()
