"""Weight gradient with dY_c gathered in the kernel's staging (from the
node gradient and the rowmap entry table) vs the rowmap SpMM writing dY_c
plus the weight gradient reading it, on the PascalVOC-shaped static batch
(psi_2 128 -> 128 with 10 uses, psi_1 256 -> 256 and 1024 -> 256).

    python tools/bench_wgrad_gather.py
"""
import json
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402
from deep_graph_matching_consensus_amd.ops import slot_gemm as sg  # noqa
from deep_graph_matching_consensus_amd.ops.plans import spline_plan  # noqa
from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    PASCAL_VOC_CATEGORIES, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.datasets.static_batch import \
    StaticPairBatcher  # noqa: E402

DEV = 'cuda'


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1000 / reps, 1)


def main():
    ops = _backend.ops()
    groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, graphs=64,
                                    feature_dim=16, seed=0)
    store = GraphStore(groups, DEV, valid_pairs=True)
    b = StaticPairBatcher(store, 512, seed=0)
    assert b.load()
    b.materialize()
    N = b.cap_s + b.cap_t
    op = spline_plan(b.v['ei'], b.v['ea_val'], N, (5, 5), (1, 1), 1,
                     root=True)
    plan = sg.compact_plan(op, 26)
    At = op.t()
    ell = sg.rowmap_ranges(plan, At)
    n = ell.view(-1, 8)[:, 3]
    rec = {'N': N, 'P_cap': plan.src.numel(),
           'rows_gt3': int((n > 3).sum()), 'rows_used': int(plan.seg[-1])}
    for cin, cout, uses in ((128, 128, 10), (256, 256, 1), (1024, 256, 1)):
        xs = [ops.split3(torch.randn(N, cin, device=DEV))
              for _ in range(uses)]
        gs = [torch.randn(N, cout, device=DEV) for _ in range(uses)]
        rounds = 1 if cin == 128 else (2 if cin == 256 else 6)

        def rowmaps():
            return [ops.slot_spmm_rowmap(At.rowptr, At.col, At.val, plan.cinv,
                                         g, plan.seg, ell, False) for g in gs]
        dys = rowmaps()
        key = '%dx%d_u%d' % (cin, cout, uses)
        rec[key + '_rowmaps_us'] = timeit(rowmaps)
        rec[key + '_wgrad_dyc_us'] = timeit(lambda: ops.slot_wgrad_x6(
            xs, dys, plan.src, plan.seg, rounds))
        rec[key + '_wgrad_gathered_us'] = timeit(lambda: ops.slot_wgrad_x6(
            xs, gs, plan.src, plan.seg, rounds, ell, At.col, At.val))
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
