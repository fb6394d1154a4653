"""Per-step wall times of the flagship training loop (first steps after
capture), with the size bucket each step used.

    python tools/step_times.py [--steps 30]
"""
import argparse
import os.path as osp
import sys
import time

import torch

sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))
import bench  # noqa: E402
from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.train import PairTrainer  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--steps', type=int, default=30)
    p.add_argument('--spin-ms', type=float, default=0)
    p.add_argument('--event-steps', type=int, default=0)
    a = p.parse_args()
    args = bench.parse_args([])
    cfg = bench.CONFIGS['pascal']
    dev = torch.device('cuda')
    torch.manual_seed(0)
    groups = make_keypoint_datasets(cfg['categories'], graphs=128,
                                    visible_prob=cfg['visible_prob'], seed=0)
    store = GraphStore(groups, dev, x_dtype=torch.bfloat16, valid_pairs=True)
    model = bench.build_model(cfg, args, groups[0].num_node_features,
                              groups[0].num_edge_features, dev)
    tr = PairTrainer(model, store, 512, mode='graph', seed=0)
    orig = tr._load_next
    last = {}

    def spy():
        last['b'] = orig()
        return last['b']
    tr._load_next = spy
    for i in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step()
        torch.cuda.synchronize()
        print('step %2d bucket %d  %.3f ms' % (
            i, last.get('b', -1), 1e3 * (time.perf_counter() - t0)),
            flush=True)
    if a.spin_ms > 0:
        x = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < a.spin_ms / 1e3:
            for _ in range(10):
                y = x @ x
            torch.cuda.synchronize()
            n += 10
        print('spin: %d GEMMs in %.0f ms' % (n, 1e3 * (time.perf_counter() -
                                                       t0)))
        del x, y
    # GPU time per step from events (no host synchronisation in between).
    evs = []
    for i in range(a.event_steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        tr.step()
        e1.record()
        evs.append((e0, e1, last.get('b', -1)))
    torch.cuda.synchronize()
    for i, (e0, e1, b) in enumerate(evs):
        print('event step %2d bucket %d  %.3f ms gpu' % (i, b,
                                                       e0.elapsed_time(e1)))
    # Host time split: batch staging vs graph replay.
    import collections
    acc = collections.defaultdict(float)
    lo = tr._load_next
    graphs = tr._graphs

    def timed_load():
        h0 = time.perf_counter()
        b = lo()
        acc['load'] += time.perf_counter() - h0
        return b
    tr._load_next = timed_load
    orig_calls = [g.__call__ for g in graphs]

    class _T(object):
        def __init__(self, g):
            self.g = g

        def __call__(self):
            h0 = time.perf_counter()
            self.g()
            acc['replay'] += time.perf_counter() - h0
    tr._graphs = [_T(g) for g in graphs]
    torch.cuda.synchronize()
    for i in range(40):
        tr.step()
    torch.cuda.synchronize()
    print('host per step: load %.3f ms, replay %.3f ms' % (
        1e3 * acc['load'] / 40, 1e3 * acc['replay'] / 40))
    tr._graphs = graphs
    tr._load_next = lo
    # Unsynchronised windows: host issue time vs wall time per step.
    for w in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host = 0.0
        for i in range(20):
            h0 = time.perf_counter()
            tr.step()
            host += time.perf_counter() - h0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print('window %d: %.3f ms/step wall, %.3f ms/step host issue' % (
            w, 1e3 * wall / 20, 1e3 * host / 20), flush=True)


if __name__ == '__main__':
    main()
