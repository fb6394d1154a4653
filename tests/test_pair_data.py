"""Port of ``/root/reference/test/utils/test_data.py`` + collation checks."""
import torch

from deep_graph_matching_consensus_amd.graph import Data, DataLoader
from deep_graph_matching_consensus_amd.graph.meta import lookup_batch_info
from deep_graph_matching_consensus_amd.utils import (PairDataset,
                                                     ValidPairDataset)

REPR = 'Data(edge_index=[2, 30], x=[10, 16])'
REPR_Y = 'Data(edge_index=[2, 30], x=[10, 16], y=[10])'


def test_pair_dataset():
    x = torch.randn(10, 16)
    edge_index = torch.randint(x.size(0), (2, 30), dtype=torch.long)
    data = Data(x=x, edge_index=edge_index)

    for sample, length in [(True, 2), (False, 4)]:
        dataset = PairDataset([data, data], [data, data], sample=sample)
        assert dataset.__repr__() == (
            'PairDataset([{0}, {0}], [{0}, {0}], sample={1})'.format(
                REPR, sample))
        assert len(dataset) == length
        pair = dataset[0]
        assert len(pair) == 4
        assert torch.allclose(pair.x_s, x)
        assert pair.edge_index_s.tolist() == edge_index.tolist()
        assert torch.allclose(pair.x_t, x)
        assert pair.edge_index_t.tolist() == edge_index.tolist()


def test_valid_pair_dataset():
    x = torch.randn(10, 16)
    edge_index = torch.randint(x.size(0), (2, 30), dtype=torch.long)
    y = torch.randperm(x.size(0))
    data = Data(x=x, edge_index=edge_index, y=y)

    for sample, length in [(True, 2), (False, 4)]:
        dataset = ValidPairDataset([data, data], [data, data], sample=sample)
        assert dataset.__repr__() == (
            'ValidPairDataset([{0}, {0}], [{0}, {0}], sample={1})'.format(
                REPR_Y, sample))
        assert len(dataset) == length
        pair = dataset[0]
        assert len(pair) == 5
        assert torch.allclose(pair.x_s, x)
        assert pair.edge_index_s.tolist() == edge_index.tolist()
        assert torch.allclose(pair.x_t, x)
        assert pair.edge_index_t.tolist() == edge_index.tolist()
        assert pair.y.tolist() == torch.arange(x.size(0)).tolist()


def test_valid_pairs_subset_rule():
    def g(labels):
        labels = torch.tensor(labels)
        n = labels.numel()
        return Data(x=torch.randn(n, 2), edge_index=torch.zeros(2, 0).long(),
                    y=labels)
    a, b, c = g([0, 1]), g([2, 1, 0]), g([1, 2])
    ds = ValidPairDataset([a, b, c], [a, b, c])
    # a <= a, a <= b; b <= b; c <= b, c <= c
    assert ds.pairs == [[0, 0], [0, 1], [1, 1], [2, 1], [2, 2]]
    pair = ds[1]  # a -> b
    assert pair.y.tolist() == [2, 1]


def test_pair_collation_follow_batch():
    g1 = Data(x=torch.randn(3, 4), edge_index=torch.tensor([[0, 1], [1, 2]]),
              y=torch.tensor([0, 1, 2]))
    g2 = Data(x=torch.randn(2, 4), edge_index=torch.tensor([[0], [1]]),
              y=torch.tensor([1, 0]))
    ds = ValidPairDataset([g1, g2], [g1, g2])
    loader = DataLoader(ds, batch_size=len(ds), follow_batch=['x_s', 'x_t'])
    batch = next(iter(loader))
    assert batch.num_graphs == len(ds)
    # index_s offset by x_s rows, y stays local.
    assert batch.edge_index_s.max() < batch.x_s.size(0)
    assert batch.y.max() < 3
    assert batch.x_s_batch.tolist() == sorted(batch.x_s_batch.tolist())
    info = lookup_batch_info(batch.x_s_batch)
    assert info is not None and info.num_nodes == batch.x_s.size(0)
    moved = batch.to('cpu')
    assert lookup_batch_info(moved.x_t_batch) is not None
