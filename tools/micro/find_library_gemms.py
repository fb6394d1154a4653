"""List the torch GEMM calls (addmm / mm / matmul / linear) that reach the
library in one eager PascalVOC-shaped training step of bench.py's model,
with their shapes and the first package frame that issued them.

    python tools/micro/find_library_gemms.py
"""
import collections
import os.path as osp
import sys
import traceback

import torch

ROOT = osp.dirname(osp.dirname(osp.dirname(osp.abspath(__file__))))
sys.path.insert(0, ROOT)

seen = collections.Counter()


def _where():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if 'deep_graph_matching_consensus_amd' in fr.filename:
            return '{}:{}'.format(fr.filename.split(
                'deep_graph_matching_consensus_amd/')[-1], fr.lineno)
    return '?'


def wrap(mod, name):
    orig = getattr(mod, name)

    def f(*a, **k):
        shp = tuple(tuple(t.shape) for t in a if torch.is_tensor(t))
        seen[(name, shp, _where())] += 1
        return orig(*a, **k)
    setattr(mod, name, f)


for n in ('addmm', 'mm', 'matmul', 'bmm', 'baddbmm'):
    wrap(torch, n)
wrap(torch.nn.functional, 'linear')
torch.Tensor.__matmul__ = lambda s, o: torch.matmul(s, o)

import bench  # noqa: E402

sys.argv = (['bench.py', '--steps', '1', '--warmup', '1', '--eval-pairs',
             '0'] + sys.argv[1:])
try:
    bench.main()
except SystemExit:
    pass
for (name, shp, where), c in sorted(seen.items(), key=lambda t: -t[1]):
    print('{:4d} x {:8s} {:40s} {}'.format(c, name, str(shp), where))
