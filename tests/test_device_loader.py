"""The HBM-resident pair loader must reproduce Python pair collation."""
import numpy as np
import torch

from deep_graph_matching_consensus_amd.datasets import (
    DevicePairLoader, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.datasets import device_loader as dl
from deep_graph_matching_consensus_amd.graph import Batch
from deep_graph_matching_consensus_amd.graph.meta import lookup_batch_info
from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.utils import ValidPairDataset
from deep_graph_matching_consensus_amd.utils.data import PairData


def _datasets():
    return make_keypoint_datasets(graphs=6, feature_dim=16, seed=3)


def test_native_collate_matches_numpy():
    store = GraphStore(_datasets(), 'cpu')
    rng = np.random.default_rng(0)
    s = rng.integers(0, store.num_graphs, 9)
    t = store.sample_partners(s, rng)
    ref = dl._collate_numpy(store, s, t)
    if _backend.host_available():
        out = store._collate_host(s, t)
        for a, b in zip(out, ref):
            assert torch.equal(a, b)


def test_store_batch_equals_python_collation():
    groups = _datasets()
    store = GraphStore(groups, 'cpu')
    s_ids = np.array([0, 7, 13])
    rng = np.random.default_rng(1)
    t_ids = store.sample_partners(s_ids, rng)
    batch = store.collate(s_ids, t_ids)

    flat = [g for grp in groups for g in grp]
    pairs = []
    for s, t in zip(s_ids, t_ids):
        ds = ValidPairDataset([flat[s]], [flat[t]])
        assert len(ds) == 1  # partner is valid
        pairs.append(ds[0])
    ref = Batch.from_data_list(pairs, follow_batch=['x_s', 'x_t'])
    for key in ['x_s', 'x_t', 'edge_index_s', 'edge_index_t', 'edge_attr_s',
                'edge_attr_t', 'x_s_batch', 'x_t_batch', 'y']:
        assert torch.equal(batch[key], ref[key]), key
    assert isinstance(pairs[0], PairData)
    info = lookup_batch_info(batch.x_s_batch)
    assert info is not None and info.num_graphs == 3


def test_loader_epoch():
    store = GraphStore(_datasets(), 'cpu')
    loader = DevicePairLoader(store, batch_size=16, seed=0)
    n = 0
    for batch in loader:
        assert batch.num_graphs == 16
        assert (batch.y >= 0).all()
        n += 1
    assert n == len(loader) == store.num_graphs // 16
