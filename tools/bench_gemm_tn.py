"""Micro-benchmark of the split-K TN GEMM (csrc/hip/gemm_tn.hip) on the
DBP15K psi_1 weight-gradient shapes against torch's fp32 product and the
dense_wgrad_f32 kernel where it applies.

    python tools/bench_gemm_tn.py [--reps 50] [--json out.json]
"""
import argparse
import json
import os.path as osp
import sys

sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))

import torch  # noqa: E402

from deep_graph_matching_consensus_amd.ops import _backend, gemm  # noqa

SHAPES = [
    ('relconv_l0_dW', 38960, [768], [300]),
    ('relconv_l12_dW', 38960, [768], [256]),
    ('final_linear_dW', 38960, [256], [300, 256, 256, 256]),
    ('pascal_l0_like', 9216, [256], [256]),
]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1000.0 * a.elapsed_time(b) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--reps', type=int, default=50)
    p.add_argument('--json', default=None)
    p.add_argument('--cfgs', type=int, nargs='+', default=[0, 4])
    p.add_argument('--only', default=None, help='one shape name')
    p.add_argument('--no-torch', action='store_true')
    args = p.parse_args()
    dev = torch.device('cuda')
    out = {}
    for name, K, wa, wb in SHAPES:
        if args.only and name != args.only:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        a = [torch.randn(K, w, device=dev, generator=g) for w in wa]
        b = [torch.randn(K, w, device=dev, generator=g) for w in wb]
        A, B = torch.cat(a, 1), torch.cat(b, 1)
        M, N = A.size(1), B.size(1)
        flop = 2.0 * K * M * N
        row = {'K': K, 'M': M, 'N': N}
        for x6 in (True, False):
            for cfg in args.cfgs:
                us = timeit(lambda: gemm.tn_f32(a, b, x6=x6, cfg=cfg),
                            args.reps)
                row['tn_{}_cfg{}'.format('x6' if x6 else 'f32', cfg)] = \
                    round(us, 1)
        row['tn_x6'] = row['tn_x6_cfg{}'.format(args.cfgs[0])]
        if not args.no_torch:
            row['torch_fp32_us'] = round(timeit(lambda: A.t() @ B,
                                                args.reps), 1)
        if gemm._dense_tn_f32_ok(A, B) and not args.no_torch:
            from deep_graph_matching_consensus_amd.ops.dense import _seg01
            seg = _seg01(K, dev)
            row['dense_wgrad_f32_us'] = round(timeit(
                lambda: _backend.ops().dense_wgrad_f32([A], 1, [B], seg),
                args.reps), 1)
        row['tn_x6_tflops'] = round(flop / row['tn_x6'] / 1e6, 1)
        out[name] = row
        print(name, row, flush=True)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
