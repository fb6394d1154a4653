"""Micro-benchmark: fused slot conv (csrc/hip/slot_conv.hip) vs the unfused
GEMM + SpMM SplineConv on a PascalVOC-shaped static batch (psi_2 layer,
128 -> 128, 26 slots).

    python tools/bench_slot_conv.py [--reps 50]
"""
import argparse
import json
import os
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))

from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    PASCAL_VOC_CATEGORIES, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.datasets.static_batch import \
    StaticPairBatcher  # noqa: E402
from deep_graph_matching_consensus_amd.ops import _backend, plans  # noqa
from deep_graph_matching_consensus_amd.ops.sparse import (  # noqa: E402
    slot_conv_error, slot_conv_image, slot_tile_plan)


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--reps', type=int, default=50)
    p.add_argument('--only-fwd', action='store_true',
                   help='time the fused forward only (counter runs)')
    args = p.parse_args()
    dev = torch.device('cuda')
    groups = make_keypoint_datasets(categories=PASCAL_VOC_CATEGORIES,
                                    graphs=128, visible_prob=0.75, seed=0)
    store = GraphStore(groups, dev, x_dtype=torch.bfloat16, valid_pairs=True)
    b = StaticPairBatcher(store, 512, seed=0)
    assert b.load()
    b.materialize()
    N = b.cap_s + b.cap_t
    ea = b.edge_attr.index_select(0, b.v['ea'])
    plans.register_plan_provider(b.v['ei'], ea, b._assembler)
    op = plans.spline_plan(b.v['ei'], ea, N, (5, 5), (1, 1), 1, True)
    assert getattr(op, 'tile_flag', None) is not None
    S, C = 26, 128
    ops = _backend.ops()
    x = torch.randn(N, C, device=dev).bfloat16()
    g = torch.randn(N, C, device=dev).bfloat16()
    w_lp = (torch.randn(C, S * C, device=dev) / C ** 0.5).bfloat16()
    bias = torch.randn(C, device=dev)
    img_f = slot_conv_image(w_lp, C, False)
    img_b = slot_conv_image(w_lp, C, True)
    err = slot_conv_error(dev)
    dy = torch.empty(N * S, C, dtype=torch.bfloat16, device=dev)
    opt = op.t()

    res = {'N': N, 'S': S, 'tiles': (N + op.tile_window - 1) // op.tile_window,
           'debug': int(os.environ.get('DGMC_SC_DEBUG', '0'))}
    pl = slot_tile_plan(op, S)
    res['plan_us'] = timeit(lambda: ops.slot_tile_plan(
        op.tile_flag, op.rowptr, op.col, op.val, op.tile_window, S, err),
        args.reps)
    res['fused_fwd_us'] = timeit(lambda: ops.slot_conv(
        x, *pl, S, img_f, False, bias, True, torch.bfloat16, None), args.reps)
    if args.only_fwd:
        print(json.dumps(res))
        return
    res['fused_bwd_dy_us'] = timeit(lambda: ops.slot_conv(
        g, *pl, S, img_b, True, None, False, torch.bfloat16, dy), args.reps)
    res['fused_bwd_us'] = timeit(lambda: ops.slot_conv(
        g, *pl, S, img_b, True, None, False, torch.bfloat16, None),
        args.reps)

    def unfused_fwd():
        y = (x @ w_lp).view(-1, C)
        return ops.spmm_csr(op.rowptr, op.col, op.val, y, None, None, bias,
                            True, torch.bfloat16)

    def unfused_bwd():
        ops.spmm_csr_out(opt.rowptr, opt.col, opt.val, g, None, None, None,
                         False, dy)
        return dy.view(N, -1) @ w_lp.t()
    res['unfused_fwd_us'] = timeit(unfused_fwd, args.reps)
    res['unfused_bwd_us0'] = timeit(unfused_bwd, args.reps)
    # dX GEMM alone ([N, S*C] x [S*C, C], 172 output tiles) and split-K.
    dY = dy.view(N, -1)
    wt = w_lp.t()
    res['dx_gemm_us'] = timeit(lambda: dY @ wt, args.reps)
    for sk in (2, 4, 8):
        kk = dY.size(1) // sk
        a3 = dY.view(N, sk, kk).transpose(0, 1)
        b3 = wt.contiguous().view(sk, kk, C)
        part = torch.empty(sk, N, C, device=dev)
        out = torch.empty(N, C, device=dev)

        def split():
            torch.bmm(a3, b3, out_dtype=torch.float32, out=part)
            ops.reduce_add_rows(part, out, False)
        res['dx_splitk%d_us' % sk] = timeit(split, args.reps)
    res['y_gemm_us'] = timeit(lambda: x @ w_lp, args.reps)
    res['unfused_bwd_us'] = timeit(unfused_bwd, args.reps)
    # Weight gradient over 10 loop uses: slot_wgrad vs dY stack + GEMM.
    from deep_graph_matching_consensus_amd.ops.sparse import (
        slot_pair_lists, slot_weight_grad)
    from deep_graph_matching_consensus_amd.ops.gemm import matmul_tn_fp32
    U = 10
    Xs = torch.randn(U * N, C, device=dev).bfloat16()
    Gs = torch.randn(U * N, C, device=dev).bfloat16()
    slot_pair_lists(op, S)
    res['pair_lists_us'] = timeit(lambda: (op.__dict__.pop('_slot_pairs',
                                                           None),
                                           slot_pair_lists(op, S)), 10)
    for ns in (40, 64, 96):
        res['wgrad_slot_s%d_us' % ns] = timeit(
            lambda: slot_weight_grad(Xs, Gs, op, S, U, nsplit=ns), 10)
    dYs = torch.randn(U * N, S * C, device=dev).bfloat16()
    res['wgrad_gemm_us'] = timeit(lambda: matmul_tn_fp32(Xs, dYs), 10)
    res['err'] = int(err)
    if res['debug'] & 8:
        # Stamps of the last launch (unfused ran after: re-run fwd once).
        ops.slot_conv(x, *pl, S, img_f, False, bias, True, torch.bfloat16,
                      None)
        torch.cuda.synchronize()
        st = ops.slot_conv_stamps().tolist()
        for w in range(2):
            b = st[8 * w:8 * w + 5]
            res['stamps_us_wg%d' % w] = [round((v - b[0]) / 100.0, 2)
                                         for v in b]
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v)
                      for k, v in res.items()}))


if __name__ == '__main__':
    main()
