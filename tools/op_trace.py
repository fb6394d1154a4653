"""Ordered list of the device ops of one static training step, each with the
innermost frame of this package that issued it (forward) or the autograd
node it came from (backward) - maps the rocprof kernel sequence
(tools/prof_quick.sh -> seq.txt) back to source lines.

    python tools/op_trace.py [--out gpurun_out/op_trace.txt]
"""
import argparse
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from deep_graph_matching_consensus_amd import parallel  # noqa: E402
from deep_graph_matching_consensus_amd.datasets import (  # noqa: E402
    GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.train import PairTrainer  # noqa: E402

PKG = os.path.join(ROOT, 'deep_graph_matching_consensus_amd')
SKIP = ('aten.detach', 'aten.view', 'aten._unsafe_view', 'aten.slice',
        'aten.select', 'aten.t.', 'aten.transpose', 'aten.expand',
        'aten.unsqueeze', 'aten.squeeze', 'aten.alias', 'aten.as_strided',
        'aten.permute', 'aten.split', 'aten.narrow', 'aten.unbind',
        'aten.lift_fresh', 'aten.empty', 'aten._to_copy.default?',
        'aten.is_same_size', 'aten.sym_', 'aten._local_scalar_dense')


def _where():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if fr.filename.startswith(PKG):
            return '{}:{} {}'.format(os.path.relpath(fr.filename, ROOT),
                                     fr.lineno, fr.name)
    return '(autograd engine)'


class Trace(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if not name.startswith(SKIP):
            shapes = [tuple(a.shape) for a in args
                      if isinstance(a, torch.Tensor)][:3]
            self.rows.append('{:<48s} {:<40s} {}'.format(
                name, str(shapes)[:40], _where()))
        return func(*args, **(kwargs or {}))


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--out', default=None)
    p.add_argument('--batch-size', type=int, default=512)
    p.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'])
    args = p.parse_args()
    bf16 = args.dtype == 'bf16'
    device = parallel.init_distributed()
    torch.manual_seed(0)
    cfg = bench.CONFIGS['pascal']
    groups = make_keypoint_datasets(cfg['categories'], graphs=128,
                                    visible_prob=cfg['visible_prob'], seed=0)
    store = GraphStore(groups, device,
                       x_dtype=torch.bfloat16 if bf16 else torch.float32,
                       valid_pairs=True)
    bargs = bench.parse_args([])
    model = bench.build_model(cfg, bargs, groups[0].num_node_features,
                              groups[0].num_edge_features, device)
    trainer = PairTrainer(model, store, args.batch_size, mode='static',
                          bf16=bf16 and device.type == 'cuda', buckets=False)
    for _ in range(2):
        trainer.step()
    bucket = trainer._load_next()
    tr = Trace()
    with tr:
        trainer._static_body(bucket)
    if device.type == 'cuda':
        torch.cuda.synchronize()
    text = '\n'.join('{:4d} {}'.format(i, r) for i, r in enumerate(tr.rows))
    if args.out:
        with open(args.out, 'w') as f:
            f.write(text + '\n')
    else:
        print(text)


if __name__ == '__main__':
    main()
