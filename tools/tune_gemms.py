#!/usr/bin/env python
"""Tune the library GEMMs of the benchmark configs with TunableOp (GPU box).

Runs one eager training step per static-batch size bucket for every rank of
every world size the driver benchmarks (1, 2, 4, 8: each rank samples its own
source shard, so its bucket capacities - the GEMMs' M - differ), plus the
DBP15K-shaped KG steps, with online tuning on; writes the union of results to
``deep_graph_matching_consensus_amd/runtime/tuned/gemm_gfx950.csv`` (or
``--out``).  Single process; ranks are simulated by their source shards.

    python tools/tune_gemms.py [--configs pascal willow dbp15k] [--out F]
"""
import argparse
import os
import os.path as osp
import sys
import time

import numpy as np
import torch

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.runtime import tuning  # noqa: E402
from deep_graph_matching_consensus_amd.train import PairTrainer  # noqa: E402


def tune_pairs(cfg_name, worlds, device, batch_size=512):
    cfg = bench.CONFIGS[cfg_name]
    args = bench.parse_args([])
    groups = make_keypoint_datasets(cfg['categories'],
                                    graphs=args.graphs_per_category,
                                    visible_prob=cfg['visible_prob'],
                                    seed=args.seed)
    store = GraphStore(groups, device, x_dtype=torch.bfloat16,
                       valid_pairs=True)
    for world in worlds:
        for rank in range(world):
            torch.manual_seed(0)
            model = bench.build_model(cfg, args, groups[0].num_node_features,
                                      groups[0].num_edge_features, device)
            sources = np.arange(store.num_graphs)[rank::world]
            tr = PairTrainer(model, store, batch_size, mode='graph',
                             seed=args.seed + 1000 * rank, sources=sources)
            for i, b in enumerate(tr.batchers):
                for _ in range(10000):
                    s, t = tr.batcher.next_ids()
                    if b.fits(s, t) and b.load(s, t):
                        break
                tr._static_body(i)
            torch.cuda.synchronize()
            print('{} world {} rank {}: caps {}, {} results'.format(
                cfg_name, world, rank, [b.caps for b in tr.batchers],
                len(torch.cuda.tunable.get_results())), flush=True)
            del tr, model


def tune_kg(device):
    args = bench.parse_args(['--config', 'dbp15k', '--steps', '1',
                             '--warmup', '1', '--no-graph'])
    out = bench.bench_kg(args, bench.CONFIGS['dbp15k'], device)
    print('dbp15k: {} ms/step, {} results'.format(
        out['ms_per_step'], len(torch.cuda.tunable.get_results())),
        flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--configs', nargs='+',
                   default=['pascal', 'willow', 'dbp15k'])
    p.add_argument('--worlds', nargs='+', type=int, default=[1, 2, 4, 8])
    p.add_argument('--out', default=tuning.TUNED_FILE)
    p.add_argument('--max-ms', type=int, default=15)
    args = p.parse_args()
    os.environ['DGMC_AMD_TUNED_GEMMS'] = '0'
    device = torch.device('cuda')
    tmp = args.out + '.partial'
    tuning.start_tuning(tmp, args.max_ms)
    t0 = time.time()
    for name in args.configs:
        if name == 'dbp15k':
            tune_kg(device)
        else:
            tune_pairs(name, args.worlds, device)
        tuning.write_results(tmp)
    os.makedirs(osp.dirname(args.out), exist_ok=True)
    n = tuning.write_results(args.out)
    print('wrote {} results to {} in {:.0f} s'.format(n, args.out,
                                                      time.time() - t0))


if __name__ == '__main__':
    main()
