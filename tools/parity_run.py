"""Accuracy parity of the native fp32 / bf16 paths against the reference
expression (``--impl reference``: eager PyTorch, reference semantics, fp32)
on the PascalVOC-shaped flagship: same seed, same synthetic data, same number
of Adam steps; reports the training-loss curve and held-out Hits@1 / Hits@10
of S_L (``/root/reference/examples/pascal.py:80-99``).

    python tools/parity_run.py --steps 200 \
        --out profiles/accuracy_parity_r3.json
"""
import argparse
import json
import os.path as osp
import sys
import time

import torch

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
sys.path.insert(0, ROOT)

from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    PASCAL_VOC_CATEGORIES, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN  # noqa
from deep_graph_matching_consensus_amd.runtime import reference_mode  # noqa
from deep_graph_matching_consensus_amd.train import PairTrainer  # noqa


def run(impl, dtype, args, device):
    torch.manual_seed(args.seed)
    reference = impl == 'reference'
    bf16 = dtype == 'bf16'
    groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, graphs=128,
                                    visible_prob=0.75, seed=args.seed)
    x_dtype = torch.bfloat16 if bf16 else torch.float32
    store = GraphStore(groups, device, x_dtype=x_dtype, valid_pairs=True)
    test_groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, graphs=32,
                                         visible_prob=0.75, seed=args.seed,
                                         split='test')
    test_store = GraphStore(test_groups, device, x_dtype=x_dtype)
    torch.manual_seed(args.seed)
    model = DGMC(SplineCNN(1024, 256, 2, 2, cat=False, dropout=0.5),
                 SplineCNN(128, 128, 2, 2, cat=True, dropout=0.0),
                 num_steps=10).to(device)
    mode = 'eager' if reference else 'graph'
    trainer = PairTrainer(model, store, 512, lr=1e-3, mode=mode, bf16=bf16,
                          seed=args.seed)
    curve = []
    t0 = time.time()
    with reference_mode(reference):
        for step in range(1, args.steps + 1):
            trainer.step()
            if step % args.log_every == 0:
                st = trainer.read_stats()
                curve.append({'step': step,
                              'loss': round(st['loss_sum'] /
                                            args.log_every, 4),
                              'hits@1_train': round(st['hits@1'], 4)})
                print(impl, dtype, curve[-1], flush=True)
        hits = trainer.evaluate(test_store, args.eval_pairs, seed=7)
    return {'impl': impl, 'dtype': dtype, 'steps': args.steps,
            'wall_s': round(time.time() - t0, 1), 'curve': curve,
            'hits@1_test': round(hits[1], 4),
            'hits@10_test': round(hits[10], 4)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--steps', type=int, default=200)
    p.add_argument('--log-every', type=int, default=20)
    p.add_argument('--eval-pairs', type=int, default=4000)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--runs', default='native:fp32,reference:fp32,native:bf16')
    p.add_argument('--out', default=None)
    args = p.parse_args()
    device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
    results = []
    for spec in args.runs.split(','):
        impl, dtype = spec.split(':')
        results.append(run(impl, dtype, args, device))
    by = {(r['impl'], r['dtype']): r for r in results}
    out = {'config': 'PascalVOC-shaped SplineCNN DGMC, batch 512, L=10, '
                     'Adam 1e-3, seed {}'.format(args.seed),
           'eval_pairs': args.eval_pairs, 'runs': results}
    nf, rf = by.get(('native', 'fp32')), by.get(('reference', 'fp32'))
    if nf and rf:
        out['delta_hits@1_native_fp32_vs_reference'] = round(
            nf['hits@1_test'] - rf['hits@1_test'], 4)
    nb = by.get(('native', 'bf16'))
    if nf and nb:
        out['delta_hits@1_native_bf16_vs_fp32'] = round(
            nb['hits@1_test'] - nf['hits@1_test'], 4)
    line = json.dumps(out, indent=1)
    print(line)
    if args.out:
        with open(args.out, 'w') as f:
            f.write(line + '\n')


if __name__ == '__main__':
    main()
