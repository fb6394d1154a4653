"""Timing of the folded projection's NT GEMM: exact-f32 MFMA kernel vs
bf16x6 (dense_nt_f32 / dense_nt_x6) on the PascalVOC shapes.

    python tools/micro/bench_dense_nt.py
"""
import json
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..', '..'))
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / reps, 2)


def main():
    ops = _backend.ops()
    for M, parts, Nn in ((10944, 3, 128), (10944, 1, 384)):
        ps = [torch.randn(M, 128, device='cuda') for _ in range(parts)]
        bt = torch.randn(Nn, 128 * parts, device='cuda')
        b3 = ops.split3(bt)
        print(json.dumps({'M': M, 'K': 128 * parts, 'N': Nn,
                          'f32_us': timeit(lambda: ops.dense_nt_f32(ps, bt)),
                          'x6_us': timeit(lambda: ops.dense_nt_x6(ps, bt)),
                          'x6_b3_us': timeit(lambda: ops.dense_nt_x6(ps, bt,
                                                                     b3))}))


if __name__ == '__main__':
    main()
