"""Micro-benchmark of the chunked NT GEMM (csrc/hip/gemm_f32.hip) on the
DBP15K psi_1 shapes: bf16x6 with and without the scheduled fragment
splits (``sched``), exact f32, torch fp32.

    python tools/bench_gemm_nt.py [--reps 30] [--json out.json]
"""
import argparse
import json
import os.path as osp
import sys

sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))

import torch  # noqa: E402

from deep_graph_matching_consensus_amd.ops import gemm  # noqa: E402

# name: (M, part widths, Nn)
SHAPES = [
    ('relconv_l0_map', 38960, [300], 768),
    ('relconv_l12_map', 38960, [256], 768),
    ('final_linear', 38960, [300, 256, 256, 256], 256),
    ('relconv_dx', 38960, [768], 256),
    ('final_dx', 38960, [256], 768),
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
    return round(1000.0 * a.elapsed_time(b) / reps, 1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--reps', type=int, default=30)
    p.add_argument('--json', default=None)
    args = p.parse_args()
    dev = torch.device('cuda')
    out = {}
    for name, M, widths, Nn in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        parts = [torch.randn(M, w, device=dev, generator=g) for w in widths]
        K = sum(widths)
        bt = torch.randn(Nn, K, device=dev, generator=g)
        row = {'M': M, 'K': K, 'Nn': Nn}
        y0 = gemm.nt_f32(parts, bt, sched=0)
        y1 = gemm.nt_f32(parts, bt, sched=1)
        row['sched_bit_identical'] = bool(torch.equal(y0, y1))
        row['x6_us'] = timeit(lambda: gemm.nt_f32(parts, bt, sched=0),
                              args.reps)
        row['x6_sched_us'] = timeit(lambda: gemm.nt_f32(parts, bt, sched=1),
                                    args.reps)
        row['f32_us'] = timeit(lambda: gemm.nt_f32(parts, bt, x6=False),
                               args.reps)
        x = torch.cat(parts, 1)
        row['torch_us'] = timeit(lambda: x @ bt.t(), args.reps)
        out[name] = row
        print(name, row, flush=True)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
