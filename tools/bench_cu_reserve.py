"""CU contention under data parallelism: the bf16x6
GEMMs run persistent grids sized to every CU; RCCL's channel kernels,
launched from the backward hooks, hold some CUs at the same time.  This
times psi_1 layer 0's pieces-sized weight gradient and forward (the
PascalVOC static-batch operator, 1024 -> 256) alone and next to a side-stream
kernel that occupies ``--hog`` CUs for the whole measurement
(``cu_hog``: one spinning workgroup per CU, bounded by the wall clock), with
the grids sized to all CUs (reserve 0) and to ``CUs - reserve``.

    python tools/bench_cu_reserve.py [--hog 8 16] [--reserve 8 16] [--json f]

(round 6: the input-gradient kernel added - the reserve is applied only
from the step's first gradient all-reduce launch to its end.)
"""
import argparse
import json
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..'))

from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    PASCAL_VOC_CATEGORIES, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.datasets.static_batch import \
    StaticPairBatcher  # noqa: E402
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402
from deep_graph_matching_consensus_amd.ops import slot_gemm as sg  # noqa
from deep_graph_matching_consensus_amd.ops.plans import spline_plan  # noqa


def timed(fn, reps, hog_blocks, side):
    """Mean us per call of ``fn`` on the current stream; with
    ``hog_blocks`` a CU hog runs on ``side`` across the whole window."""
    ops = _backend.ops()
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    if hog_blocks:
        # Long enough to cover every call (sized from an uncontended run).
        t = timed(fn, 3, 0, None)
        with torch.cuda.stream(side):
            ops.cu_hog(torch.empty(1, device='cuda'), hog_blocks,
                       min(3.0 * t * (reps + 4) + 200.0, 5e5))
        torch.cuda._sleep(1000)     # let the hog occupy its CUs first
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / reps, 2)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--hog', type=int, nargs='+', default=[8, 16])
    p.add_argument('--reserve', type=int, nargs='+', default=[8, 16])
    p.add_argument('--reps', type=int, default=20)
    p.add_argument('--json', default=None)
    args = p.parse_args()
    dev = torch.device('cuda')
    groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, graphs=128,
                                    feature_dim=16, seed=0)
    store = GraphStore(groups, dev, valid_pairs=True)
    b = StaticPairBatcher(store, 512, seed=0)
    assert b.load()
    b.materialize()
    N = b.cap_s + b.cap_t
    op = spline_plan(b.v['ei'], b.v['ea_val'], N, (5, 5), (1, 1), 1,
                     root=True)
    plan = sg.compact_plan(op, 26)
    P = plan.src.numel()
    ops = _backend.ops()
    cin, cout = 1024, 256
    x = torch.randn(N, cin, device=dev)
    w = torch.randn(25, cin, cout, device=dev) / cin ** 0.5
    r = torch.randn(cin, cout, device=dev) / cin ** 0.5
    dy = torch.randn(P, cout, device=dev)
    x3 = ops.split3(x)
    wt3 = ops.slot_weight_x3(w, r, True)
    w3 = ops.slot_weight_x3(w, r, False)
    kernels = {
        'fwd_1024x256': lambda: ops.slot_gemm_x6(x, plan.src, plan.seg, wt3,
                                                 True, None),
        # the input gradient (persistent like the forward; runs in the
        # backward next to the gradient all-reduces)
        'dx_1024x256': lambda: ops.slot_gemm_x6(dy, plan.src, plan.seg, w3,
                                                False, None),
        'wgrad_1024x256': lambda: ops.slot_wgrad_x6(
            [x3], [dy], plan.src, plan.seg, sg._x6_rounds(16)),
    }
    side = torch.cuda.Stream()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    out = {'cus': cus, 'rows': N, 'compact_rows': int(plan.seg[-1]),
           'results': []}
    for name, fn in kernels.items():
        for hog in [0] + args.hog:
            for res in sorted({0, *args.reserve}):
                if res and not hog:
                    continue
                _backend.set_cu_reserve(res)
                us = timed(fn, args.reps, hog, side)
                out['results'].append({'kernel': name, 'hog_cus': hog,
                                       'reserve_cus': res, 'us': us})
                print(json.dumps(out['results'][-1]), flush=True)
    _backend.set_cu_reserve(0)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
