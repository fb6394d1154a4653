"""Loop-shared gradient accumulation (runtime/loopgrad.py) == plain
autograd."""
import pytest
import torch

from deep_graph_matching_consensus_amd.datasets import (
    DevicePairLoader, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, RelCNN, SplineCNN
from deep_graph_matching_consensus_amd.runtime import loopgrad


def _grads(model, args, y, seed, enabled, autocast=False):
    model.zero_grad(set_to_none=True)
    old = loopgrad.ENABLED
    loopgrad.ENABLED = enabled
    try:
        torch.manual_seed(seed)
        dev = args[0].device.type
        with torch.autocast(dev, dtype=torch.bfloat16, enabled=autocast):
            S0, SL = model(*args, y=y)
            loss = model.loss(S0, y) + model.loss(SL, y)
        loss.backward()
    finally:
        loopgrad.ENABLED = old
    return loss.detach(), {n: p.grad.detach().clone()
                           for n, p in model.named_parameters()
                           if p.grad is not None}


def _batch(device, feat=16, bs=12):
    groups = make_keypoint_datasets(graphs=6, feature_dim=feat, seed=3)
    store = GraphStore(groups, device)
    b = next(iter(DevicePairLoader(store, batch_size=bs, seed=0)))
    args = (b.x_s, b.edge_index_s, b.edge_attr_s, b.x_s_batch, b.x_t,
            b.edge_index_t, b.edge_attr_t, b.x_t_batch)
    return args, b.y


def _compare(model, args, y, rtol, autocast=False):
    l0, g0 = _grads(model, args, y, 5, enabled=False, autocast=autocast)
    l1, g1 = _grads(model, args, y, 5, enabled=True, autocast=autocast)
    assert torch.allclose(l0, l1, rtol=1e-5, atol=1e-6)
    assert g0.keys() == g1.keys()
    for n in g0:
        err = (g0[n] - g1[n]).abs().max().item()
        scale = g0[n].abs().max().item() + 1e-12
        # (psi_2.final.bias cancels in P_i - Q_j: its gradient is ~0.)
        assert err <= rtol * scale + 1e-6, (n, err, scale)
    # Every psi_2 / MLP parameter actually received a gradient.
    assert any(n.startswith('psi_2.') for n in g1)
    assert 'mlp.0.weight' in g1


def test_loop_grads_match_dense_spline_cpu():
    args, y = _batch('cpu')
    torch.manual_seed(0)
    model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                 SplineCNN(8, 8, 2, 2, cat=True), num_steps=3)
    _compare(model, args, y, rtol=1e-5)


def test_loop_grads_match_sparse_rel_cpu():
    args, y = _batch('cpu')
    torch.manual_seed(0)
    model = DGMC(RelCNN(16, 16, 2), RelCNN(8, 8, 2), num_steps=3, k=4)
    args = (args[0], args[1], None, args[3], args[4], args[5], None,
            args[7])
    _compare(model, args, y, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('autocast', [False, True])
def test_loop_grads_match_dense_spline_gpu(autocast):
    args, y = _batch('cuda', feat=32, bs=16)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(32, 32, 2, 2, cat=False),
                 SplineCNN(16, 16, 2, 2, cat=True), num_steps=4).cuda()
    _compare(model, args, y, rtol=2e-2 if autocast else 1e-4,
             autocast=autocast)
