"""PascalVOC keypoint matching (reference: examples/pascal.py).

Same flags and model as the reference driver; data are synthetic
PascalVOC-shaped keypoint graphs (20 categories, Delaunay + Cartesian/
Distance), trained with the HBM-resident loader and (on GPU) a
hipGraph-captured step.  Multi-GPU: launch with torch.distributed.run.

    python examples/pascal.py [--epochs 15] [--batch_size 512] [--dtype fp32]
"""
import argparse
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..'))

from deep_graph_matching_consensus_amd import parallel  # noqa: E402
from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    PASCAL_VOC_CATEGORIES, GraphStore, keypoint_transform,
    make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN  # noqa
from deep_graph_matching_consensus_amd.train import (  # noqa: E402
    MetricsLogger, PairTrainer)

parser = argparse.ArgumentParser()
parser.add_argument('--isotropic', action='store_true')
parser.add_argument('--dim', type=int, default=256)
parser.add_argument('--rnd_dim', type=int, default=128)
parser.add_argument('--num_layers', type=int, default=2)
parser.add_argument('--num_steps', type=int, default=10)
parser.add_argument('--lr', type=float, default=0.001)
parser.add_argument('--batch_size', type=int, default=512)
parser.add_argument('--epochs', type=int, default=15)
parser.add_argument('--test_samples', type=int, default=1000)
parser.add_argument('--graphs', type=int, default=256,
                    help='synthetic training graphs per category')
parser.add_argument('--mode', default=None, choices=['graph', 'static',
                                                     'eager'])
parser.add_argument('--normalization', default='softmax',
                    choices=['softmax', 'sinkhorn'],
                    help='extension: Sinkhorn instead of the reference '
                         'row softmax (dense path)')
parser.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'],
                    help='fp32 = reference precision; bf16 = encoder GEMMs '
                         'under autocast')
parser.add_argument('--checkpoint', default=None)
parser.add_argument('--log', default=None, help='JSONL metrics file')
args = parser.parse_args()

device = parallel.init_distributed()
transform = keypoint_transform(args.isotropic)
train_groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, args.graphs,
                                      transform=transform, split='train')
test_groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES,
                                     max(args.graphs // 4, 8),
                                     transform=transform, split='test')
bf16 = args.dtype == 'bf16' and device.type == 'cuda'
dtype = torch.bfloat16 if bf16 else torch.float32
store = GraphStore(train_groups, device, x_dtype=dtype)
test_stores = [GraphStore([g], device, x_dtype=dtype) for g in test_groups]

num_node_features = train_groups[0].num_node_features
num_edge_features = train_groups[0].num_edge_features
psi_1 = SplineCNN(num_node_features, args.dim, num_edge_features,
                  args.num_layers, cat=False, dropout=0.5)
psi_2 = SplineCNN(args.rnd_dim, args.rnd_dim, num_edge_features,
                  args.num_layers, cat=True, dropout=0.0)
model = DGMC(psi_1, psi_2, num_steps=args.num_steps,
             normalization=args.normalization).to(device)
mode = args.mode or ('graph' if device.type == 'cuda' else 'eager')
trainer = PairTrainer(model, store, args.batch_size, lr=args.lr, mode=mode,
                      bf16=bf16)
logger = MetricsLogger(args.log)
if args.checkpoint and osp.exists(args.checkpoint):
    trainer.load(args.checkpoint)

steps_per_epoch = max(store.num_graphs // (args.batch_size *
                                           parallel.world_size()), 1)
for epoch in range(1, args.epochs + 1):
    for _ in range(steps_per_epoch):
        trainer.step()
    stats = trainer.read_stats()
    loss = stats['loss_sum'] / (steps_per_epoch * parallel.world_size())
    accs = [100 * trainer.evaluate(s, args.test_samples)[1]
            for s in test_stores]
    accs += [sum(accs) / len(accs)]
    logger.log(epoch=epoch, loss=loss, acc=accs[-1])
    if parallel.rank() == 0:
        print(f'Epoch: {epoch:02d}, Loss: {loss:.4f}')
        print(' '.join([c[:5].ljust(5) for c, _ in PASCAL_VOC_CATEGORIES] +
                       ['mean']))
        print(' '.join([f'{acc:.1f}'.ljust(5) for acc in accs]))
    if args.checkpoint:
        trainer.save(args.checkpoint)
parallel.shutdown()
