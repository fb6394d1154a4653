"""Opt-in Sinkhorn normalisation (extension; the reference uses softmax)."""
import torch

from deep_graph_matching_consensus_amd.datasets import (
    DevicePairLoader, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
from deep_graph_matching_consensus_amd.ops import reference as ref


def test_masked_sinkhorn_doubly_stochastic_on_valid_block():
    torch.manual_seed(0)
    B, N = 3, 7
    S_hat = torch.randn(B, N, N)
    n = torch.tensor([7, 5, 3])
    mask = ref.count_mask(n, n, N, N)
    S = ref.masked_sinkhorn(S_hat, mask, num_iters=50)
    assert torch.isfinite(S).all()
    assert (S[~mask] == 0).all()
    for b in range(B):
        blk = S[b, :n[b], :n[b]]
        assert torch.allclose(blk.sum(-1), torch.ones(n[b]), atol=1e-5)
        assert torch.allclose(blk.sum(-2), torch.ones(n[b]), atol=1e-3)
    # Zero iterations degenerate to the masked softmax.
    assert torch.allclose(ref.masked_sinkhorn(S_hat, mask, num_iters=0),
                          ref.masked_softmax(S_hat, mask), atol=1e-6)


def test_dgmc_sinkhorn_forward_backward():
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=1)
    store = GraphStore(groups, 'cpu')
    b = next(iter(DevicePairLoader(store, batch_size=6, seed=0)))
    torch.manual_seed(0)
    model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                 SplineCNN(8, 8, 2, 2, cat=True), num_steps=2,
                 normalization='sinkhorn', sinkhorn_iters=5)
    S_0, S_L = model(b.x_s, b.edge_index_s, b.edge_attr_s, b.x_s_batch,
                     b.x_t, b.edge_index_t, b.edge_attr_t, b.x_t_batch)
    assert torch.allclose(S_L.sum(-1), torch.ones(S_L.size(0)), atol=1e-5)
    y = torch.stack([torch.arange(b.y.numel()), b.y])
    loss = model.loss(S_0, y) + model.loss(S_L, y)
    loss.backward()
    assert all(p.grad is not None for p in model.mlp.parameters())
