"""DBP15K cross-lingual KG alignment (reference: examples/dbp15k.py).

Synthetic DBP15K-shaped KG pair (same entity/triple/alignment counts as the
chosen category).  Two-phase schedule of the reference: epochs 1-100 train
the initial feature matching (num_steps=0), epochs 101-200 refine with
num_steps consensus iterations and a detached psi_1.

    python examples/dbp15k.py --category zh_en
"""
import argparse
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..'))

from deep_graph_matching_consensus_amd.datasets.kg import (  # noqa: E402
    DBP15K_SIZES, make_kg_pair)
from deep_graph_matching_consensus_amd.models import DGMC, RelCNN  # noqa
from deep_graph_matching_consensus_amd.train import KGTrainer  # noqa: E402

parser = argparse.ArgumentParser()
parser.add_argument('--category', type=str, required=True,
                    choices=sorted(DBP15K_SIZES))
parser.add_argument('--dim', type=int, default=256)
parser.add_argument('--rnd_dim', type=int, default=32)
parser.add_argument('--num_layers', type=int, default=3)
parser.add_argument('--num_steps', type=int, default=10)
parser.add_argument('--k', type=int, default=10)
parser.add_argument('--epochs', type=int, default=200)
parser.add_argument('--scale', type=float, default=1.0)
parser.add_argument('--no_graph', action='store_true')
parser.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'],
                    help='fp32 = reference precision')
parser.add_argument('--checkpoint', default=None,
                    help='save / resume the trainer state here')
args = parser.parse_args()

device = 'cuda' if torch.cuda.is_available() else 'cpu'
data = make_kg_pair(args.category, scale=args.scale).to(device)

psi_1 = RelCNN(data.x1.size(-1), args.dim, args.num_layers, batch_norm=False,
               cat=True, lin=True, dropout=0.5)
psi_2 = RelCNN(args.rnd_dim, args.rnd_dim, args.num_layers, batch_norm=False,
               cat=True, lin=True, dropout=0.0)
model = DGMC(psi_1, psi_2, num_steps=None, k=args.k).to(device)
trainer = KGTrainer(model, data, lr=0.001, graph=not args.no_graph,
                    bf16=args.dtype == 'bf16')
start = 1
if args.checkpoint and osp.exists(args.checkpoint):
    trainer.load(args.checkpoint)
    start = trainer.step_count + 1

print('Optimize initial feature matching...')
half = args.epochs // 2
if start <= half:
    model.num_steps = 0
for epoch in range(start, args.epochs + 1):
    if epoch == half + 1:
        print('Refine correspondence matrix...')
        model.num_steps = args.num_steps
        model.detach = True
    trainer.step()
    if args.checkpoint:
        trainer.save(args.checkpoint)
    if epoch % 10 == 0 or epoch > half:
        hits1, hits10 = trainer.evaluate()
        loss = float(trainer.last_loss)
        print(f'{epoch:03d}: Loss: {loss:.4f}, Hits@1: {hits1:.4f}, '
              f'Hits@10: {hits10:.4f}')
