"""BASELINE config 1: synthetic Erdos-Renyi pairs, GIN encoders, L=10
(plumbing check; runs on CPU).

    python examples/er_gin.py [--nodes 20] [--iters 200]
"""
import argparse
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..'))

from deep_graph_matching_consensus_amd.datasets.random_graphs import (  # noqa
    make_er_pair)
from deep_graph_matching_consensus_amd.models import DGMC, GIN  # noqa: E402

parser = argparse.ArgumentParser()
parser.add_argument('--nodes', type=int, default=20)
parser.add_argument('--p', type=float, default=0.2)
parser.add_argument('--dim', type=int, default=32)
parser.add_argument('--rnd_dim', type=int, default=16)
parser.add_argument('--num_steps', type=int, default=10)
parser.add_argument('--iters', type=int, default=200)
parser.add_argument('--lr', type=float, default=0.001)
args = parser.parse_args()

device = 'cpu'
model = DGMC(GIN(32, args.dim, 2), GIN(args.rnd_dim, args.rnd_dim, 2),
             num_steps=args.num_steps).to(device)
optimizer = torch.optim.Adam(model.parameters(), lr=args.lr)

for it in range(1, args.iters + 1):
    s, t, y = make_er_pair(args.nodes, args.p, seed=it)
    model.train()
    optimizer.zero_grad()
    S_0, S_L = model(s.x, s.edge_index, None, None, t.x, t.edge_index, None,
                     None)
    loss = model.loss(S_0, y) + model.loss(S_L, y)
    loss.backward()
    optimizer.step()
    if it % 20 == 0:
        model.eval()
        s, t, y = make_er_pair(args.nodes, args.p, seed=10 ** 6 + it)
        with torch.no_grad():
            _, S_L = model(s.x, s.edge_index, None, None, t.x, t.edge_index,
                           None, None)
        print(f'iter {it:04d} loss {loss.item():.4f} '
              f'test Hits@1 {model.acc(S_L, y):.3f}')
