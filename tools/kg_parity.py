"""DBP15K-shaped two-phase accuracy parity: native fp32 (captured KGTrainer
phases, HIP kernels) against the reference expression (``reference_mode``:
eager PyTorch, reference semantics, fp32) on the same synthetic KG pair,
same seed, the reference schedule (``/root/reference/examples/dbp15k.py:
63-76``: epochs 1-100 initial matching, 101-200 refinement with
``num_steps`` consensus steps and a detached psi_1).  Also reports the
raw-feature nearest-neighbour Hits@1 the trained model must beat.

    python tools/kg_parity.py --scale 0.25 --out profiles/kg_parity_r4.json
"""
import argparse
import json
import os.path as osp
import sys
import time

import torch

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
sys.path.insert(0, ROOT)

from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair  # noqa
from deep_graph_matching_consensus_amd.models import DGMC, RelCNN  # noqa
from deep_graph_matching_consensus_amd.runtime import reference_mode  # noqa
from deep_graph_matching_consensus_amd.train import KGTrainer  # noqa


def raw_nn_hits1(data):
    """Hits@1 of matching test sources to their nearest target by the raw
    feature inner product (no training)."""
    src, dst = data.test_y
    s = data.x1[src] @ data.x2.t()
    return float((s.argmax(-1) == dst).float().mean())


def run(impl, args, device):
    reference = impl == 'reference'
    torch.manual_seed(args.seed)
    data = make_kg_pair(args.category, scale=args.scale,
                        seed=args.seed).to(device)
    torch.manual_seed(args.seed)
    psi_1 = RelCNN(data.x1.size(-1), args.dim, args.num_layers,
                   batch_norm=False, cat=True, lin=True, dropout=0.5)
    psi_2 = RelCNN(args.rnd_dim, args.rnd_dim, args.num_layers,
                   batch_norm=False, cat=True, lin=True, dropout=0.0)
    model = DGMC(psi_1, psi_2, num_steps=None, k=args.k).to(device)
    trainer = KGTrainer(model, data, lr=1e-3, graph=not reference)
    curve = []
    half = args.epochs // 2
    t0 = time.time()
    with reference_mode(reference):
        model.num_steps = 0
        for epoch in range(1, args.epochs + 1):
            if epoch == half + 1:
                model.num_steps, model.detach = args.num_steps, True
            trainer.step()
            if epoch % args.log_every == 0 or epoch == args.epochs:
                h1, h10 = trainer.evaluate()
                curve.append({'epoch': epoch,
                              'loss': round(float(trainer.last_loss), 4),
                              'hits@1': round(h1, 4),
                              'hits@10': round(h10, 4)})
                print(impl, curve[-1], flush=True)
    return {'impl': impl, 'dtype': 'fp32',
            'wall_s': round(time.time() - t0, 1), 'curve': curve,
            'hits@1': curve[-1]['hits@1'],
            'hits@10': curve[-1]['hits@10'], 'raw_nn_hits@1': round(
                raw_nn_hits1(data), 4)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--category', default='zh_en')
    p.add_argument('--scale', type=float, default=0.25)
    p.add_argument('--dim', type=int, default=256)
    p.add_argument('--rnd_dim', type=int, default=32)
    p.add_argument('--num_layers', type=int, default=3)
    p.add_argument('--num_steps', type=int, default=10)
    p.add_argument('--k', type=int, default=10)
    p.add_argument('--epochs', type=int, default=200)
    p.add_argument('--log-every', type=int, default=20)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--runs', default='native,reference')
    p.add_argument('--out', default=None)
    args = p.parse_args()
    device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
    results = [run(impl, args, device) for impl in args.runs.split(',')]
    by = {r['impl']: r for r in results}
    out = {'config': 'DBP15K-shaped {} KG pair, scale {}, RelCNN dim {} '
                     'rnd_dim {} L={}, k={}, two-phase {} epochs, Adam 1e-3, '
                     'seed {}'.format(args.category, args.scale, args.dim,
                                      args.rnd_dim, args.num_layers, args.k,
                                      args.epochs, args.seed),
           'runs': results}
    if 'native' in by and 'reference' in by:
        for m in ('hits@1', 'hits@10'):
            out['delta_{}_native_vs_reference'.format(m)] = round(
                by['native'][m] - by['reference'][m], 4)
    line = json.dumps(out, indent=1)
    print(line)
    if args.out:
        with open(args.out, 'w') as f:
            f.write(line + '\n')


if __name__ == '__main__':
    main()
