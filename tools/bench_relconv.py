"""Per-kernel timing of the fused RelCNN consensus encoder
(csrc/hip/relconv.hip) on the full-size DBP15K-shaped joint graph
(19,388 + 19,572 entities): layer forward, layer forward + projection,
projection backward, layer backward, partial fold - and one whole fused
consensus step forward + backward.

    python tools/bench_relconv.py [--reps 50] [--json out.json]
"""
import argparse
import json
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..'))

from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair  # noqa
from deep_graph_matching_consensus_amd.models import RelCNN  # noqa: E402
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402
from deep_graph_matching_consensus_amd.ops import relconv as rc  # noqa


def timeit(fn, reps):
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
    p = argparse.ArgumentParser()
    p.add_argument('--reps', type=int, default=50)
    p.add_argument('--json', default=None)
    p.add_argument('--hub-sweep', type=int, nargs='*', default=[],
                   help='also time fwd / bwd with these hub thresholds')
    p.add_argument('--scale', type=float, default=1.0)
    p.add_argument('--no-gemm', action='store_true')
    args = p.parse_args()
    dev = torch.device('cuda')
    d = make_kg_pair('zh_en', seed=0, scale=args.scale)
    n_s, n_t = d.x1.size(0), d.x2.size(0)
    N = n_s + n_t
    ei = torch.cat([d.edge_index1, d.edge_index2 + n_s], 1).to(dev)
    plan = rc.rel_plan(ei, N)
    ops = _backend.ops()
    torch.manual_seed(0)
    psi_2 = RelCNN(32, 32, 3, cat=True, lin=True).to(dev)
    mlp0 = torch.nn.Linear(32, 32).to(dev)
    conv = psi_2.convs[1]
    w = [conv.lin1.weight.detach(), conv.lin2.weight.detach(),
         conv.root.weight.detach()]
    b = conv.root.bias.detach()
    feat = torch.randn(N, 128, device=dev).relu_()
    fold = torch.randn(32, 128, device=dev) / 11
    pq = torch.empty(N, 32, device=dev)
    dfeat = torch.randn(N, 128, device=dev)
    dpq = torch.randn(N, 32, device=dev)
    part = torch.zeros(plan.n_tiles, rc.PART, device=dev)
    partf = torch.zeros(plan.n_tiles, 4096, device=dev)
    outs = [torch.empty(rc.PART, device=dev) for _ in range(3)] + \
        [torch.empty(4096, device=dev)]
    fa, ba = plan.fwd_args(), plan.bwd_args()
    res = {'N': N, 'nnz': int(plan.col_f.numel()),
           'hub_rows': int(plan.hub.sum()), 'tiles': plan.n_tiles}
    res['fwd_us'] = timeit(lambda: ops.relconv_fwd(
        *fa, feat[:, 32:64], None, *w, b, True, feat[:, 64:96], None, None,
        None, None), args.reps)
    res['fwd_proj_us'] = timeit(lambda: ops.relconv_fwd(
        *fa, feat[:, 64:96], None, *w, b, True, feat[:, 96:128], None,
        feat[:, 0:96], fold, pq), args.reps)
    res['proj_bwd_us'] = timeit(lambda: ops.rel_proj_bwd(
        dpq, feat, fold, dfeat, partf, True), args.reps)
    res['bwd_us'] = timeit(lambda: ops.relconv_bwd(
        *ba, dfeat[:, 64:96], feat[:, 32:64], None, *w, dfeat[:, 32:64],
        dfeat[:, 32:64], 0, True, part, True), args.reps)
    res['fold_us'] = timeit(lambda: ops.rel_fold(
        [part, part, part, partf], outs), args.reps)
    for T in args.hub_sweep:
        pt = rc.RelPlan(ei, N, hub_threshold=T)
        fa2, ba2 = pt.fwd_args(), pt.bwd_args()
        res['hub%d_rows' % T] = int(pt.hub.sum())
        res['hub%d_fwd_us' % T] = timeit(lambda: ops.relconv_fwd(
            *fa2, feat[:, 32:64], None, *w, b, True, feat[:, 64:96], None,
            None, None, None), args.reps)
        res['hub%d_bwd_us' % T] = timeit(lambda: ops.relconv_bwd(
            *ba2, dfeat[:, 64:96], feat[:, 32:64], None, *w,
            dfeat[:, 32:64], dfeat[:, 32:64], 0, True, part, True),
            args.reps)
    # node GEMMs of psi_1 (exact-f32 chunked kernel vs torch / hipBLASLt)
    tiny = torch.zeros(1, device=dev)
    res['launch_floor_us'] = timeit(lambda: tiny.add_(1), args.reps)
    for K, Nn in (() if args.no_gemm else
                  ((300, 768), (256, 768), (1068, 256))):
        xg = torch.randn(N, K, device=dev)
        wg = torch.randn(Nn, K, device=dev)
        res['gemm_%dx%d_us' % (K, Nn)] = timeit(
            lambda: ops.gemm_nt_f32([xg], wg, None, False, None), 10)
        res['torch_%dx%d_us' % (K, Nn)] = timeit(lambda: xg @ wg.t(), 10)
    r_s = torch.randn(n_s, 32, device=dev)
    r_t = torch.randn(n_t, 32, device=dev, requires_grad=True)

    def step():
        out = rc.psi2_fold(psi_2, mlp0.weight, plan, r_s, r_t, ('bench', 0))
        torch.autograd.grad(out, [r_t] + list(psi_2.parameters())[:12] +
                            [mlp0.weight], dpq, allow_unused=True)
    res['step_fwd_bwd_us'] = timeit(step, max(args.reps // 5, 3))
    print(json.dumps(res), flush=True)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
