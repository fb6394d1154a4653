"""Device ops of one DBP15K-shaped KG training step (refinement phase:
num_steps=10, detach=True, k=10), counted per (op, issuing source line) -
the KG counterpart of tools/op_trace.py, for finding glue kernels.

    python tools/op_trace_kg.py [--out gpurun_out/op_trace_kg.txt]
"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

from op_trace import SKIP, _where  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
from deep_graph_matching_consensus_amd import parallel  # noqa: E402
from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair  # noqa
from deep_graph_matching_consensus_amd.models import DGMC, RelCNN  # noqa
from deep_graph_matching_consensus_amd.train import KGTrainer  # noqa: E402


class Count(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if not name.startswith(SKIP):
            self.rows[(name, _where())] += 1
        return func(*args, **(kwargs or {}))


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--out', default=None)
    p.add_argument('--scale', type=float, default=1.0)
    args = p.parse_args()
    device = parallel.init_distributed()
    torch.manual_seed(0)
    data = make_kg_pair('zh_en', scale=args.scale, seed=0).to(device)
    psi_1 = RelCNN(data.x1.size(-1), 256, 3, batch_norm=False, cat=True,
                   lin=True, dropout=0.5)
    psi_2 = RelCNN(32, 32, 3, batch_norm=False, cat=True, lin=True,
                   dropout=0.0)
    model = DGMC(psi_1, psi_2, num_steps=10, k=10, detach=True).to(device)
    trainer = KGTrainer(model, data, graph=False)
    for _ in range(2):
        trainer.step()
    tr = Count()
    with tr:
        trainer._body_static()
    if device.type == 'cuda':
        torch.cuda.synchronize()
    lines = ['{:5d}  {:<44s} {}'.format(n, op, where)
             for (op, where), n in tr.rows.most_common()]
    text = 'total ops: {}\n'.format(sum(tr.rows.values())) + '\n'.join(lines)
    if args.out:
        with open(args.out, 'w') as f:
            f.write(text + '\n')
    print(text[:6000])


if __name__ == '__main__':
    main()
