"""PascalPF-style matching trained on random point sets
(reference: examples/pascal_pf.py).

Training data is the reference's own synthetic generator (30-60 inliers,
0-20 outliers, KNN(8) graphs with Cartesian attributes, constant node
features).  The real PascalPF test pairs are not available offline, so the
model is tested on held-out random pairs from the same generator.

    python examples/pascal_pf.py
"""
import argparse
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..'))

from deep_graph_matching_consensus_amd.datasets.random_graphs import (  # noqa
    RandomGraphDataset, pascal_pf_transform)
from deep_graph_matching_consensus_amd.graph import DataLoader  # noqa: E402
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN  # noqa

parser = argparse.ArgumentParser()
parser.add_argument('--dim', type=int, default=256)
parser.add_argument('--rnd_dim', type=int, default=64)
parser.add_argument('--num_layers', type=int, default=2)
parser.add_argument('--num_steps', type=int, default=10)
parser.add_argument('--lr', type=float, default=0.001)
parser.add_argument('--batch_size', type=int, default=64)
parser.add_argument('--epochs', type=int, default=32)
parser.add_argument('--test_pairs', type=int, default=256)
parser.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'],
                    help='fp32 = reference precision; bf16 = encoder GEMMs '
                         'under autocast')
args = parser.parse_args()

transform = pascal_pf_transform()
train_dataset = RandomGraphDataset(30, 60, 0, 20, transform=transform)
train_loader = DataLoader(train_dataset, args.batch_size, shuffle=True,
                          follow_batch=['x_s', 'x_t'])
test_dataset = RandomGraphDataset(30, 60, 0, 20, transform=transform,
                                  length=args.test_pairs)

device = 'cuda' if torch.cuda.is_available() else 'cpu'
psi_1 = SplineCNN(1, args.dim, 2, args.num_layers, cat=False, dropout=0.0)
psi_2 = SplineCNN(args.rnd_dim, args.rnd_dim, 2, args.num_layers, cat=True,
                  dropout=0.0)
model = DGMC(psi_1, psi_2, num_steps=args.num_steps).to(device)
optimizer = torch.optim.Adam(model.parameters(), lr=args.lr)


def autocast():
    return torch.autocast(device_type='cuda' if device == 'cuda' else 'cpu',
                          dtype=torch.bfloat16,
                          enabled=args.dtype == 'bf16' and device == 'cuda',
                          cache_enabled=False)


def train():
    model.train()
    total_loss = torch.zeros((), device=device)
    correct = torch.zeros((), device=device)
    examples = 0
    for data in train_loader:
        optimizer.zero_grad()
        data = data.to(device)
        with autocast():
            S_0, S_L = model(data.x_s, data.edge_index_s, data.edge_attr_s,
                             data.x_s_batch, data.x_t, data.edge_index_t,
                             data.edge_attr_t, data.x_t_batch)
        y = torch.stack([data.y_index_s, data.y_t], dim=0)
        loss = model.loss(S_0, y)
        loss = model.loss(S_L, y) + loss if model.num_steps > 0 else loss
        loss.backward()
        optimizer.step()
        total_loss += loss.detach()
        correct += model.correct(S_L.detach(), y)
        examples += y.size(1)
    return total_loss.item() / len(train_loader), correct.item() / examples


@torch.no_grad()
def test():
    model.eval()
    correct = num_examples = 0
    for i in range(len(test_dataset)):
        pair = test_dataset[i].to(device)
        with autocast():
            _, S_L = model(pair.x_s, pair.edge_index_s, pair.edge_attr_s,
                           None, pair.x_t, pair.edge_index_t,
                           pair.edge_attr_t, None)
        y = torch.stack([pair.y_index_s, pair.y_t], dim=0)
        correct += model.acc(S_L, y, reduction='sum')
        num_examples += y.size(1)
    return correct / num_examples


for epoch in range(1, args.epochs + 1):
    loss, acc = train()
    print(f'Epoch: {epoch:02d}, Loss: {loss:.4f}, Acc: {acc:.2f}, '
          f'Test: {100 * test():.1f}')
