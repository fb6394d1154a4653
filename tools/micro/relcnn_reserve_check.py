"""psi_1 RelCNN forward + backward (DBP15K shape, scale 0.25) against the
fp64 reference expression under different DP CU reserves (the persistent
NT GEMM picks its tile shape from the usable CU count).

    python tools/micro/relcnn_reserve_check.py
"""
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.join(osp.dirname(osp.abspath(__file__)), '..', '..'))
from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair  # noqa
from deep_graph_matching_consensus_amd.models import RelCNN  # noqa: E402
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402
from deep_graph_matching_consensus_amd.runtime import reference_mode  # noqa


def main():
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

    def oracle(dtype):
        m2 = RelCNN(x.size(1), 256, 3, batch_norm=False, cat=True, lin=True,
                    dropout=0.0).to(dev).to(dtype)
        m2.load_state_dict({k: v.to(dtype)
                            for k, v in model.state_dict().items()})
        with reference_mode(True):
            o = m2(x.to(dtype), ei)
            p2 = dict(m2.named_parameters())
            return [o] + list(torch.autograd.grad(
                o, [p2[n] for n in names], go.to(dtype)))

    r64, r32 = oracle(torch.float64), oracle(torch.float32)
    for res in (0, 4, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192):
        _backend.set_cu_reserve(res)
        out = model(x, ei)
        got = [out] + list(torch.autograd.grad(out, params, go))
        worst = []
        for n, a, b32, b64 in zip(['out'] + names, got, r32, r64):
            e = float((a.detach().double() - b64).abs().max())
            e32 = float((b32.double() - b64).abs().max())
            lim = 4 * e32 + 1e-6 * float(b64.abs().max())
            if e > lim:
                worst.append('%s %.3g > %.3g' % (n, e, lim))
        print('reserve %d: %s' % (res, '; '.join(worst) if worst else 'ok'),
              flush=True)
    _backend.set_cu_reserve(0)


if __name__ == '__main__':
    main()
