"""Timing + error of the bf16x6 slot GEMM (csrc/hip/slot_gemm_x6.hip) against
the exact-f32 MFMA kernels on the PascalVOC-shaped static batch operator.

    python tools/bench_slot_gemm_x6.py [--reps 20] [--json out.json]

Per shape (psi_2 128->128, psi_1 256->256 and 1024->256): forward (gathered
X W_s) and input gradient (dY_c W_s^T) in us per call - operands as bf16
planes or fp32 (split in the kernel) - plus the split kernels' cost, the
weight gradient, and the max error of both against fp64.
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
    return round(t0.elapsed_time(t1) * 1e3 / reps, 2)


def main():
    p = argparse.ArgumentParser()
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
    used = int(plan.seg[-1])
    P = plan.src.numel()
    ops = _backend.ops()
    out = {'N': N, 'compact_rows': used, 'P_cap': P, 'shapes': []}
    seg = plan.seg.cpu().tolist()
    src = plan.src.long()
    for cin, cout in ((128, 128), (256, 256), (1024, 256)):
        x = torch.randn(N, cin, device=dev)
        w = torch.randn(25, cin, cout, device=dev) / cin ** 0.5
        r = torch.randn(cin, cout, device=dev) / cin ** 0.5
        dy = torch.randn(P, cout, device=dev)
        wt = ops.slot_weight_t(w, r)
        x3 = ops.split3(x)
        dy3 = ops.split3(dy)
        wt3 = ops.slot_weight_x3(w, r, True)
        w3 = ops.slot_weight_x3(w, r, False)
        flop = 2.0 * used * cin * cout
        rec = {'cin': cin, 'cout': cout}
        rec['fwd_f32_us'] = timeit(lambda: ops.slot_gemm2(
            x, plan.src, plan.seg, wt, None, True), args.reps)
        rec['fwd_x6_us'] = timeit(lambda: ops.slot_gemm_x6(
            x3, plan.src, plan.seg, wt3, True, None), args.reps)
        rec['fwd_x6_f32x_us'] = timeit(lambda: ops.slot_gemm_x6(
            x, plan.src, plan.seg, wt3, True, None), args.reps)
        rec['split_x_us'] = timeit(lambda: ops.split3(x), args.reps)
        def f32dx():
            if cout >= 256:
                return ops.slot_gemm2(dy, plan.src, plan.seg, w, r, False)
            return ops.slot_gemm(dy, plan.src, plan.seg, w, r, True, None)
        rec['dx_f32_us'] = timeit(f32dx, args.reps)
        rec['dx_x6_us'] = timeit(lambda: ops.slot_gemm_x6(
            dy3, plan.src, plan.seg, w3, False, None), args.reps)
        rec['dx_x6_f32dy_us'] = timeit(lambda: ops.slot_gemm_x6(
            dy, plan.src, plan.seg, w3, False, None), args.reps)
        rec['split_dy_us'] = timeit(lambda: ops.split3(dy), args.reps)
        rec['weight_x3_us'] = timeit(lambda: ops.slot_weight_x3(w, r, True),
                                     args.reps)
        uses = 10 if cin == 128 else 1
        rounds = 1 if cin == 128 else (2 if cin == 256 else 6)
        xs = [x] * uses
        dys = [dy] * uses
        x3s = [x3] * uses
        dy3s = [dy3] * uses
        rec['wgrad_uses'] = uses
        rec['wgrad_f32_us'] = timeit(lambda: ops.slot_wgrad_f32(
            xs, dys, plan.src, plan.seg, rounds), args.reps)
        rec['wgrad_x6_us'] = timeit(lambda: ops.slot_wgrad_x6(
            x3s, dy3s, plan.src, plan.seg, rounds), args.reps)
        rec['wgrad_x6_f32dy_us'] = timeit(lambda: ops.slot_wgrad_x6(
            x3s, dys, plan.src, plan.seg, rounds), args.reps)
        rec['wgrad_x6_f32xdy_us'] = timeit(lambda: ops.slot_wgrad_x6(
            xs, dys, plan.src, plan.seg, rounds), args.reps)
        rec['fwd_x6_tflops'] = round(flop / rec['fwd_x6_us'] / 1e6, 1)
        rec['fwd_f32_tflops'] = round(flop / rec['fwd_f32_us'] / 1e6, 1)
        # errors vs fp64
        W = torch.cat([w, r[None]], 0).double()
        ref = torch.zeros(P, cout, dtype=torch.float64, device=dev)
        refz = torch.zeros(P, cin, dtype=torch.float64, device=dev)
        for s in range(26):
            a, bb = seg[s], seg[s + 1]
            rows = src[a:bb]
            ok = rows >= 0
            ref[a:bb][ok] = x.double()[rows[ok]] @ W[s]
            refz[a:bb] = dy.double()[a:bb] @ W[s].t()
        valid = src >= 0
        y6 = ops.slot_gemm_x6(x3, plan.src, plan.seg, wt3, True, None)
        y32 = ops.slot_gemm2(x, plan.src, plan.seg, wt, None, True)
        rec['fwd_err_x6'] = float((y6.double() - ref)[valid].abs().max())
        rec['fwd_err_f32'] = float((y32.double() - ref)[valid].abs().max())
        vr = torch.zeros(P, dtype=torch.bool, device=dev)
        vr[:used] = True
        z6 = ops.slot_gemm_x6(dy3, plan.src, plan.seg, w3, False, None)
        z32 = f32dx()
        rec['dx_err_x6'] = float((z6.double() - refz)[vr].abs().max())
        rec['dx_err_f32'] = float((z32.double() - refz)[vr].abs().max())
        print(json.dumps(rec), flush=True)
        out['shapes'].append(rec)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
