"""Repeat psi_1 RelCNN forward + backward (DBP15K shape, scale 0.25) and
report parameters whose gradients differ between repetitions (bitwise) or
from the fp64 reference expression beyond 4x the fp32 one.

    python tools/micro/relcnn_determinism.py [reps]
"""
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..', '..'))
from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair  # noqa
from deep_graph_matching_consensus_amd.models import RelCNN  # noqa: E402
from deep_graph_matching_consensus_amd.runtime import reference_mode  # noqa


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = 'cuda'
    data = make_kg_pair('zh_en', scale=0.25, seed=0).to(dev)
    x = torch.cat([data.x1, data.x2], 0)
    n1 = data.x1.size(0)
    ei = torch.cat([data.edge_index1, data.edge_index2 + n1], 1)
    torch.manual_seed(0)
    model = RelCNN(x.size(1), 256, 3, batch_norm=False, cat=True, lin=True,
                   dropout=0.0).to(dev)
    go = torch.randn(x.size(0), 256, device=dev)
    names = [n for n, _ in model.named_parameters()
             if not n.startswith('batch_norms')]
    params = [dict(model.named_parameters())[n] for n in names]

    def run():
        out = model(x, ei)
        return [out] + list(torch.autograd.grad(out, params, go))

    m2 = RelCNN(x.size(1), 256, 3, batch_norm=False, cat=True, lin=True,
                dropout=0.0).to(dev).double()
    m2.load_state_dict({k: v.double() for k, v in model.state_dict().items()})
    with reference_mode(True):
        o = m2(x.double(), ei)
        p2 = dict(m2.named_parameters())
        ref = [o] + list(torch.autograd.grad(o, [p2[n] for n in names],
                                             go.double()))
    first = run()
    torch.cuda.synchronize()
    for r in range(reps):
        cur = run()
        torch.cuda.synchronize()
        for n, a, b, f in zip(['out'] + names, cur, first, ref):
            if not torch.equal(a, b):
                print('rep %d: %s differs from rep 0 by %.3g (vs fp64 %.3g / '
                      '%.3g)' % (r, n, float((a - b).abs().max()),
                                 float((a.double() - f).abs().max()),
                                 float((b.double() - f).abs().max())),
                      flush=True)
    print('done', flush=True)


if __name__ == '__main__':
    main()
