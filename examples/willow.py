"""WILLOW-ObjectClass matching with PascalVOC pre-training
(reference: /root/reference/examples/willow.py).

Protocol of the reference driver, on synthetic data (datasets/keypoints.py):

* pre-train on PascalVOC-shaped graphs (``ValidPairDataset(sample=True)``
  batches, ``willow.py:86-91``) and snapshot the state dict;
* every run (``willow.py:143-167``): shuffle each WILLOW-shaped category
  (40 graphs, exactly 10 keypoints, all visible), fine-tune a fresh Adam from
  the snapshot for ``--epochs`` EPOCHS over ``PairDataset(sample=False)`` of
  the first 20 graphs per category (all 20 x 20 ordered pairs, concatenated
  over categories, shuffled DataLoader with ``follow_batch``), with the
  identity ground truth over the 10 keypoints (``generate_y``, ``:94-97``);
* test (``:121-140``): two independently shuffled loaders over the same
  category's held-out graphs, zipped, identity ground truth, until
  ``--test_samples`` ground truths are seen;
* report per-category mean +- std over ``--runs``.

``--dtype fp32`` (default) is the reference precision; ``bf16`` runs the
encoder GEMMs under autocast.

    python examples/willow.py [--runs 20] [--dtype fp32]
"""
import argparse
import copy
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..'))

from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    PASCAL_VOC_CATEGORIES, WILLOW_CATEGORIES, GraphStore, keypoint_transform,
    make_keypoint_datasets)
from deep_graph_matching_consensus_amd.graph import DataLoader  # noqa: E402
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN  # noqa
from deep_graph_matching_consensus_amd.train import PairTrainer  # noqa: E402
from deep_graph_matching_consensus_amd.utils import PairDataset  # noqa: E402

parser = argparse.ArgumentParser()
parser.add_argument('--isotropic', action='store_true')
parser.add_argument('--dim', type=int, default=256)
parser.add_argument('--rnd_dim', type=int, default=128)
parser.add_argument('--num_layers', type=int, default=2)
parser.add_argument('--num_steps', type=int, default=10)
parser.add_argument('--lr', type=float, default=0.001)
parser.add_argument('--batch_size', type=int, default=512)
parser.add_argument('--pre_epochs', type=int, default=15)
parser.add_argument('--epochs', type=int, default=15)
parser.add_argument('--runs', type=int, default=20)
parser.add_argument('--test_samples', type=int, default=100)
parser.add_argument('--graphs', type=int, default=128,
                    help='synthetic PascalVOC graphs per category')
parser.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'])
args = parser.parse_args()

device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
bf16 = args.dtype == 'bf16' and device.type == 'cuda'
x_dtype = torch.bfloat16 if bf16 else torch.float32
mode = 'graph' if device.type == 'cuda' else 'eager'
transform = keypoint_transform(args.isotropic)

pre_store = GraphStore(make_keypoint_datasets(
    PASCAL_VOC_CATEGORIES, args.graphs, transform=transform), device,
    x_dtype=x_dtype)
willow = make_keypoint_datasets(WILLOW_CATEGORIES, 40, visible_prob=1.0,
                                transform=transform, seed=7)

psi_1 = SplineCNN(1024, args.dim, 2, args.num_layers, cat=False, dropout=0.5)
psi_2 = SplineCNN(args.rnd_dim, args.rnd_dim, 2, args.num_layers, cat=True,
                  dropout=0.0)
model = DGMC(psi_1, psi_2, num_steps=args.num_steps).to(device)


def autocast():
    return torch.autocast(device_type=device.type, dtype=torch.bfloat16,
                          enabled=bf16, cache_enabled=False)


print('Pretraining model on PascalVOC...')
pre = PairTrainer(model, pre_store, args.batch_size, lr=args.lr, mode=mode,
                  bf16=bf16)
steps = max(pre_store.num_graphs // args.batch_size, 1)
for epoch in range(1, args.pre_epochs + 1):
    for _ in range(steps):
        pre.step()
    stats = pre.read_stats()
    print(f'Epoch: {epoch:02d}, Loss: {stats["loss_sum"] / steps:.4f}')
state_dict = copy.deepcopy(model.state_dict())
print('Done!')


def generate_y(num_nodes, batch_size):
    """Identity ground truth over ``num_nodes`` keypoints per pair
    (``willow.py:94-97``)."""
    row = torch.arange(num_nodes * batch_size, device=device)
    col = row[:num_nodes].view(1, -1).repeat(batch_size, 1).view(-1)
    return torch.stack([row, col], dim=0)


def _to(data):
    return data.to(device) if x_dtype == torch.float32 else \
        data.to(device).apply(lambda t: t.to(x_dtype)
                              if t.is_floating_point() else t, 'x', 'x_s',
                              'x_t')


def train(loader, optimizer):
    model.train()
    total = torch.zeros((), device=device)
    for data in loader:
        optimizer.zero_grad()
        data = _to(data)
        with autocast():
            S_0, S_L = model(data.x_s, data.edge_index_s, data.edge_attr_s,
                             data.x_s_batch, data.x_t, data.edge_index_t,
                             data.edge_attr_t, data.x_t_batch)
        num_graphs = data.num_graphs
        y = generate_y(10, num_graphs)
        loss = model.loss(S_0, y)
        loss = model.loss(S_L, y) + loss if model.num_steps > 0 else loss
        loss.backward()
        optimizer.step()
        total += loss.detach() * num_graphs
    return float(total) / len(loader.dataset)


@torch.no_grad()
def test(dataset, seed):
    model.eval()
    g1 = torch.Generator().manual_seed(2 * seed)
    g2 = torch.Generator().manual_seed(2 * seed + 1)
    loader1 = DataLoader(dataset, args.batch_size, shuffle=True, generator=g1)
    loader2 = DataLoader(dataset, args.batch_size, shuffle=True, generator=g2)
    correct = torch.zeros((), dtype=torch.long, device=device)
    num_examples = 0
    while num_examples < args.test_samples:
        for data_s, data_t in zip(loader1, loader2):
            data_s, data_t = _to(data_s), _to(data_t)
            with autocast():
                _, S_L = model(data_s.x, data_s.edge_index, data_s.edge_attr,
                               data_s.batch, data_t.x, data_t.edge_index,
                               data_t.edge_attr, data_t.batch)
            y = generate_y(10, data_t.num_graphs)
            correct += model.correct(S_L, y)
            num_examples += y.size(1)
            if num_examples >= args.test_samples:
                break
    return float(correct) / num_examples


def run(i):
    gen = torch.Generator().manual_seed(i)
    train_sets, test_sets = [], []
    for ds in willow:
        perm = torch.randperm(len(ds), generator=gen).tolist()
        train_sets.append([ds[j] for j in perm[:20]])
        test_sets.append([ds[j] for j in perm[20:]])
    train_dataset = torch.utils.data.ConcatDataset(
        [PairDataset(t, t, sample=False) for t in train_sets])
    loader = DataLoader(train_dataset, args.batch_size, shuffle=True,
                        follow_batch=['x_s', 'x_t'],
                        generator=torch.Generator().manual_seed(100 + i))
    model.load_state_dict(state_dict)
    optimizer = torch.optim.Adam(model.parameters(), lr=args.lr)
    for _ in range(1, 1 + args.epochs):
        train(loader, optimizer)
    accs = [100 * test(t, 1000 * i + c) for c, t in enumerate(test_sets)]
    print(f'Run {i:02d}:')
    print(' '.join([c.ljust(13) for c, _ in WILLOW_CATEGORIES]))
    print(' '.join([f'{acc:.2f}'.ljust(13) for acc in accs]))
    return accs


accs = torch.tensor([run(i) for i in range(1, 1 + args.runs)])
print('-' * 14 * 5)
mean, std = accs.mean(dim=0), accs.std(dim=0)
print(' '.join([c.ljust(13) for c, _ in WILLOW_CATEGORIES]))
print(' '.join([f'{a:.2f} ± {s:.2f}'.ljust(13) for a, s in zip(mean, std)]))
