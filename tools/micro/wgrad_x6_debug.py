"""Diagnostic: bf16x6 weight gradient vs exact-f32 on the headline plan,
per slot (relative error, scale ratio)."""
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..', '..'))
from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    PASCAL_VOC_CATEGORIES, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.datasets.static_batch import \
    StaticPairBatcher  # noqa: E402
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402
from deep_graph_matching_consensus_amd.ops import slot_gemm as sg  # noqa
from deep_graph_matching_consensus_amd.ops.plans import spline_plan  # noqa

dev = 'cuda'
groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, graphs=64,
                                feature_dim=16, seed=0)
store = GraphStore(groups, dev, valid_pairs=True)
b = StaticPairBatcher(store, 512, seed=0)
assert b.load()
b.materialize()
N = b.cap_s + b.cap_t
op = spline_plan(b.v['ei'], b.v['ea_val'], N, (5, 5), (1, 1), 1, root=True)
plan = sg.compact_plan(op, 26)
ops = _backend.ops()
P = plan.src.numel()
used = int(plan.seg[-1])
for cin, uses in ((128, 1), (128, 3)):
    xs = [torch.randn(N, cin, device=dev) for _ in range(uses)]
    dys = []
    for _ in range(uses):
        d = torch.randn(P, cin, device=dev)
        d[used:] = 0
        d[plan.src.long() < 0] = 0
        dys.append(d)
    w6 = ops.slot_wgrad_x6([ops.split3(x) for x in xs],
                           [ops.split3(d) for d in dys], plan.src, plan.seg, 1)
    w32 = ops.slot_wgrad_f32(xs, dys, plan.src, plan.seg, 1)
    print('uses', uses, 'max |w32|', float(w32.abs().max()),
          'max |w6 - w32|', float((w6 - w32).abs().max()))
    for s in range(0, 26, 5):
        a, bb = w6[s], w32[s]
        print(' slot', s, 'rel', float((a - bb).norm() / bb.norm()),
              'ratio', float((a * bb).sum() / (bb * bb).sum()))
    # element pattern of slot 0: where is it wrong
    e = (w6[0] - w32[0]).abs()
    print(' slot0 err rows (first 8 i):', e.max(1).values[:8].tolist())
    print(' slot0 err cols (first 8 c):', e.max(0).values[:8].tolist())
    # transpose check
    print(' slot0 rel vs transposed', float((w6[0] - w32[0].t()).norm() /
                                              w32[0].norm()))
