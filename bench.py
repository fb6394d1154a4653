#!/usr/bin/env python
"""Training-throughput benchmark (driver contract).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config pascal]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Headline (BASELINE.json): graph-pairs/sec of DGMC training on
PascalVOC-shaped keypoint graphs with SplineCNN encoders, exactly the
reference driver's model (``/root/reference/examples/pascal.py:46-52``):
psi_1 = SplineCNN(1024, 256, dim=2, 2 layers, cat=False, dropout=0.5),
psi_2 = SplineCNN(128, 128, dim=2, 2 layers, cat=True), num_steps=10, k=-1
(dense), Adam(lr=1e-3), loss = NLL(S_0) + NLL(S_L), 512 pairs per GPU per
step (weak scaling: global batch = 512 * N).  Data: synthetic
PascalVOC-shaped graphs (20 categories, 6-19 keypoints, ~9 visible nodes per
graph, Delaunay + Cartesian), random-init weights.  Every timed step runs the
full forward (10 consensus iterations), backward, gradient all-reduce and the
Adam update.

Rank 0 prints ONE JSON line.  ``--impl reference`` measures the eager
PyTorch expression of the reference algorithm (fp32, oracle ops, reference
host syncs) used as the BASELINE.md denominator.
"""
import argparse
import json
import os
import os.path as osp
import sys
import time

import torch

ROOT = osp.dirname(osp.abspath(__file__))
sys.path.insert(0, ROOT)

from deep_graph_matching_consensus_amd import parallel  # noqa: E402
from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    PASCAL_VOC_CATEGORIES, WILLOW_CATEGORIES, DevicePairLoader, GraphStore,
    make_keypoint_datasets)
from deep_graph_matching_consensus_amd.datasets.static_batch import (  # noqa
    StaticPairBatcher)
from deep_graph_matching_consensus_amd.runtime import GraphedStep  # noqa
from deep_graph_matching_consensus_amd.models import (  # noqa: E402
    DGMC, SplineCNN)
from deep_graph_matching_consensus_amd.runtime import reference_mode  # noqa

BASELINE_FILE = osp.join(ROOT, 'profiles', 'reference_equivalent.json')

CONFIGS = {
    # name: (categories, visible_prob, rnd_dim, metric description)
    'pascal': dict(categories=PASCAL_VOC_CATEGORIES, visible_prob=0.75,
                   model='DGMC-SplineCNN PascalVOC (psi_1 SplineCNN(1024,256,'
                         'dim=2,L=2,cat=False,dropout=0.5), psi_2 SplineCNN('
                         '128,128,dim=2,L=2,cat=True), num_steps=10, k=-1)'),
    'willow': dict(categories=WILLOW_CATEGORIES, visible_prob=1.0,
                   model='DGMC-SplineCNN WILLOW (psi_1 SplineCNN(1024,256,'
                         'dim=2,L=2,cat=False,dropout=0.5), psi_2 SplineCNN('
                         '128,128,dim=2,L=2,cat=True), num_steps=10, k=-1)'),
}


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--config', default='pascal', choices=sorted(CONFIGS))
    p.add_argument('--batch-size', type=int, default=512)
    p.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    p.add_argument('--impl', default='native',
                   choices=['native', 'reference'])
    p.add_argument('--graphs-per-category', type=int, default=128)
    p.add_argument('--num-steps', type=int, default=10)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--no-overlap', action='store_true')
    p.add_argument('--no-graph', action='store_true',
                   help='disable hipGraph capture of the training step')
    p.add_argument('--json-out', default=None)
    return p.parse_args(argv)


def build_model(cfg, args, num_node_features, num_edge_features, device):
    psi_1 = SplineCNN(num_node_features, 256, num_edge_features, 2,
                      cat=False, dropout=0.5)
    psi_2 = SplineCNN(128, 128, num_edge_features, 2, cat=True, dropout=0.0)
    return DGMC(psi_1, psi_2, num_steps=args.num_steps).to(device)


def main(argv=None):
    args = parse_args(argv)
    device = parallel.init_distributed()
    rank, world = parallel.rank(), parallel.world_size()
    cfg = CONFIGS[args.config]
    torch.manual_seed(args.seed)
    reference = args.impl == 'reference'
    use_bf16 = args.dtype == 'bf16' and not reference

    groups = make_keypoint_datasets(
        cfg['categories'], graphs=args.graphs_per_category,
        visible_prob=cfg['visible_prob'], seed=args.seed)
    store = GraphStore(groups, device,
                       x_dtype=torch.bfloat16 if use_bf16 else torch.float32,
                       valid_pairs=True)
    shard = torch.arange(store.num_graphs)[rank::world].numpy()
    use_graph = (device.type == 'cuda' and not reference and
                 not args.no_graph)

    model = build_model(cfg, args, groups[0].num_node_features,
                        groups[0].num_edge_features, device)
    model.train()
    reducer = parallel.GradBucketAllReducer(
        model, overlap=not (args.no_overlap or use_graph))
    fused = device.type == 'cuda'
    optimizer = torch.optim.Adam(model.parameters(), lr=1e-3, fused=fused,
                                 capturable=use_graph)
    stats = torch.zeros(3, dtype=torch.float64, device=device)
    autocast = dict(device_type=device.type, dtype=torch.bfloat16,
                    enabled=use_bf16, cache_enabled=False)

    def forward_loss(batch, rows, mask):
        with torch.autocast(**autocast):
            S_0, S_L = model(batch.x_s, batch.edge_index_s,
                             batch.edge_attr_s, batch.x_s_batch, batch.x_t,
                             batch.edge_index_t, batch.edge_attr_t,
                             batch.x_t_batch)
        y = torch.stack([rows, batch.y], dim=0)
        loss = model.loss(S_0, y, mask=mask)
        if model.num_steps > 0:
            loss = model.loss(S_L, y, mask=mask) + loss
        loss.backward()
        stats[0] += loss.detach().double()
        stats[1] += model.correct(S_L.detach(), y, mask).double()
        stats[2] += y.size(1) if mask is None else mask.sum().double()

    overflows = 0
    if use_graph:
        # Static shapes + whole-step hipGraph (zero-grad, gather, forward,
        # backward and - on one GPU - the optimizer update).
        batcher = StaticPairBatcher(store, args.batch_size, sources=shard,
                                    seed=args.seed + 1000 * rank)
        rows = torch.arange(batcher.cap_s, device=device)

        def body():
            reducer.flat.zero_()
            batch = batcher.materialize()
            forward_loss(batch, rows, batch.y_mask)
            if world == 1:
                optimizer.step()

        step_graph = GraphedStep(body, warmup=3)

        def train_step():
            while not batcher.load():
                pass
            step_graph()
            if world > 1:
                reducer.finish()
                optimizer.step()
    else:
        loader = DevicePairLoader(store, args.batch_size, sources=shard,
                                  seed=args.seed + 1000 * rank)
        batches = loader.forever()

        def train_step():
            batch = next(batches)
            reducer.zero_grad()
            rows = torch.arange(batch.y.numel(), device=device)
            forward_loss(batch, rows, None)
            reducer.finish()
            optimizer.step()

    def sync():
        if device.type == 'cuda':
            torch.cuda.synchronize()

    with reference_mode(reference):
        for _ in range(args.warmup):
            train_step()
        stats.zero_()
        parallel.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            train_step()
        sync()
        parallel.barrier()
        elapsed = time.perf_counter() - t0
    if use_graph:
        overflows = batcher.overflows

    elapsed = parallel.all_reduce_max(elapsed, device)
    parallel.all_reduce_sum(stats)
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    pairs = args.batch_size * world * args.steps
    value = pairs / elapsed
    hits1 = float(stats[1] / stats[2]) if stats[2] > 0 else None
    mean_loss = float(stats[0] / (args.steps * world))

    baseline = None
    if osp.exists(BASELINE_FILE) and not reference:
        with open(BASELINE_FILE) as f:
            ref = json.load(f)
        entry = ref.get(args.config, {})
        baseline = entry.get('value')
    nodes = store.node_ptr[1:] - store.node_ptr[:-1]
    out = {
        'metric': 'graph-pairs/sec training, PascalVOC-shaped SplineCNN DGMC'
                  if args.config == 'pascal' else
                  'graph-pairs/sec training, {}-shaped SplineCNN DGMC'.format(
                      args.config),
        'value': round(value, 2),
        'unit': 'pairs/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms_per_step, 3),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': round(value / baseline, 3) if baseline else None,
        'dtype': 'fp32' if not use_bf16 else 'bf16',
        'data': 'synthetic ({} categories x {} graphs, mean {:.1f} nodes/'
                'graph, Delaunay+Cartesian), random-init weights'.format(
                    len(cfg['categories']), args.graphs_per_category,
                    float(nodes.mean())),
        'config': {
            'model': cfg['model'],
            'global_batch': args.batch_size * world,
            'seq_len': int(nodes.max()),
            'parallelism': 'dp{}'.format(world),
            'impl': args.impl,
            'consensus_steps': args.num_steps,
            'hipgraph': bool(use_graph),
        },
        'hits@1_train': round(hits1, 4) if hits1 is not None else None,
        'loss': round(mean_loss, 4),
        'capacity_overflows': overflows,
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, 'w') as f:
                f.write(line + '\n')
    parallel.shutdown()
    return 0


if __name__ == '__main__':
    sys.exit(main())
