"""Micro-benchmark of the fp32 slot GEMM kernels (csrc/hip/slot_gemm.hip) on
a PascalVOC-shaped static batch operator: forward (gathered NN), dX (W^T),
row-mapped SpMM and the TN weight gradient for the psi_1 (1024 -> 256,
256 -> 256) and psi_2 (128 -> 128) shapes.

    python tools/bench_slot_gemm.py [--reps 20]
"""
import argparse
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


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / reps


def slot_ids(plan, used):
    seg = plan.seg.long()
    rows = torch.arange(used, device=seg.device)
    return torch.searchsorted(seg[1:], rows, right=True)


def rel(a, ref):
    return float((a.double() - ref).abs().max() / ref.abs().max())


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--reps', type=int, default=20)
    p.add_argument('--only', default=None)
    args = p.parse_args()
    dev = torch.device('cuda')
    groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, graphs=128,
                                    feature_dim=16, seed=0)
    store = GraphStore(groups, dev, valid_pairs=True)
    b = StaticPairBatcher(store, 512, seed=0)
    assert b.load()
    b.materialize()
    # The union graph as the training step sees it (static assembled
    # operator from the plan provider).
    N = b.cap_s + b.cap_t
    ei, ea = b.v['ei'], b.v['ea_val']
    op = spline_plan(ei, ea, N, (5, 5), (1, 1), 1, root=True)
    S = 26
    plan = sg.compact_plan(op, S)
    used = int(plan.seg[-1])
    print('N %d, nnz %d, used compact rows %d (P_cap %d)' % (
        N, int(op.rowptr[-1]), used, plan.P_cap))
    ops = _backend.ops()
    At = op.t()
    for cin, cout, uses in ((128, 128, 10), (256, 256, 1), (1024, 256, 1)):
        if args.only and args.only != str(cin):
            continue
        x = torch.randn(N, cin, device=dev)
        w = torch.randn(25, cin, cout, device=dev) / cin ** 0.5
        r = torch.randn(cin, cout, device=dev) / cin ** 0.5
        g = torch.randn(N, cout, device=dev)
        flop = 2.0 * used * cin * cout
        t = timeit(lambda: ops.slot_gemm(x, plan.src, plan.seg, w, r, False),
                   args.reps)
        print('%4d->%-4d fwd   %8.1f us  %6.1f TF/s' % (cin, cout, t,
                                                       flop / t / 1e6))
        valid = plan.src[:used] >= 0
        y1 = ops.slot_gemm(x, plan.src, plan.seg, w, r, False)[:used][valid]
        wt = ops.slot_weight_t(w, r)
        y2 = ops.slot_gemm2(x, plan.src, plan.seg, wt, None, True)
        y2 = y2[:used][valid]
        if cin * cout <= 256 * 256:      # (fp64 oracle memory)
            ref = (x.double()[plan.src[:used][valid].long()].unsqueeze(1) @ (
                torch.cat([w, r[None]]).double()[slot_ids(plan, used)[valid]])
            ).squeeze(1)
            print('    v1 err %.2e  v2 err %.2e (rel. to max |Y|)' % (
                rel(y1, ref), rel(y2, ref)))
        t = timeit(lambda: ops.slot_gemm2(x, plan.src, plan.seg, wt, None,
                                          True), args.reps)
        print('%4d->%-4d fwd2  %8.1f us  %6.1f TF/s' % (cin, cout, t,
                                                       flop / t / 1e6))
        t = timeit(lambda: ops.slot_weight_t(w, r), args.reps)
        print('%4d->%-4d W^T   %8.1f us' % (cin, cout, t))
        dyc = ops.slot_spmm_rowmap(At.rowptr, At.col, At.val, plan.cinv, g,
                                   plan.seg)
        t = timeit(lambda: ops.slot_spmm_rowmap(At.rowptr, At.col, At.val,
                                                plan.cinv, g, plan.seg),
                   args.reps)
        print('%4d->%-4d rowmap %7.1f us' % (cin, cout, t))
        rg = ops.slot_rowmap_ranges(At.rowptr, plan.cinv)
        d2 = ops.slot_spmm_rowmap(At.rowptr, At.col, At.val, plan.cinv, g,
                                  plan.seg, rg)
        assert torch.equal(d2[:used], dyc[:used])
        t = timeit(lambda: ops.slot_spmm_rowmap(At.rowptr, At.col, At.val,
                                                plan.cinv, g, plan.seg, rg),
                   args.reps)
        print('%4d->%-4d rowmap+ranges %7.1f us' % (cin, cout, t))
        t = timeit(lambda: ops.slot_gemm(dyc, plan.src, plan.seg, w, r,
                                         True), args.reps)
        print('%4d->%-4d dX    %8.1f us  %6.1f TF/s' % (cin, cout, t,
                                                       flop / t / 1e6))
        if cin * cout <= 256 * 256:      # (fp64 oracle memory)
            z1 = ops.slot_gemm(dyc, plan.src, plan.seg, w, r, True)[:used]
            z2 = ops.slot_gemm2(dyc, plan.src, plan.seg, w, r, False)[:used]
            ref = (dyc[:used].double().unsqueeze(1) @ torch.cat(
                [w, r[None]]).double()[slot_ids(plan, used)].transpose(1, 2)
            ).squeeze(1)
            print('    v1 err %.2e  v2 err %.2e' % (rel(z1, ref),
                                                  rel(z2, ref)))
        t = timeit(lambda: ops.slot_gemm2(dyc, plan.src, plan.seg, w, r,
                                          False), args.reps)
        print('%4d->%-4d dX2   %8.1f us  %6.1f TF/s' % (cin, cout, t,
                                                       flop / t / 1e6))
        xs, ds = [x] * uses, [dyc] * uses
        t = timeit(lambda: sg.weight_grad(xs, ds, plan, cin, cout),
                   max(args.reps // 4, 2))
        print('%4d->%-4d wgrad %8.1f us  %6.1f TF/s  (%d uses)' % (
            cin, cout, t, uses * flop / t / 1e6, uses))


if __name__ == '__main__':
    main()
