"""CPU: native-path == reference-mode (fused pair encoding, index packing)."""
import torch

from deep_graph_matching_consensus_amd.datasets import (
    DevicePairLoader, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
from deep_graph_matching_consensus_amd.runtime import reference_mode


def test_native_equals_reference_mode_cpu():
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=1)
    store = GraphStore(groups, 'cpu')
    batch = next(iter(DevicePairLoader(store, batch_size=12, seed=0)))
    torch.manual_seed(0)
    model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                 SplineCNN(8, 8, 2, 2, cat=True), num_steps=2)
    args = (batch.x_s, batch.edge_index_s, batch.edge_attr_s,
            batch.x_s_batch, batch.x_t, batch.edge_index_t,
            batch.edge_attr_t, batch.x_t_batch)
    torch.manual_seed(1)
    a0, aL = model(*args)
    with reference_mode():
        torch.manual_seed(1)
        b0, bL = model(*args)
    assert torch.allclose(a0, b0, atol=1e-5)
    assert torch.allclose(aL, bL, atol=1e-5)
