"""Ports of the reference encoder tests (``/root/reference/test/models``)."""
from itertools import product

import torch

from deep_graph_matching_consensus_amd.models import (GIN, MLP, RelCNN,
                                                      SplineCNN)


def test_mlp():
    model = MLP(16, 32, num_layers=2, batch_norm=True, dropout=0.5)
    assert model.__repr__() == ('MLP(16, 32, num_layers=2, batch_norm=True'
                                ', dropout=0.5)')
    out = model(torch.randn(100, 16))
    assert out.size() == (100, 32)


def test_gin():
    model = GIN(16, 32, num_layers=2, batch_norm=True, cat=True, lin=True)
    assert model.__repr__() == ('GIN(16, 32, num_layers=2, batch_norm=True, '
                                'cat=True, lin=True)')
    x = torch.randn(100, 16)
    edge_index = torch.randint(100, (2, 400), dtype=torch.long)
    for cat, lin in product([False, True], [False, True]):
        model = GIN(16, 32, 2, True, cat, lin)
        out = model(x, edge_index)
        assert out.size() == (100, 16 + 2 * 32 if not lin and cat else 32)
        assert out.size() == (100, model.out_channels)


def test_rel():
    model = RelCNN(16, 32, num_layers=2, batch_norm=True, cat=True, lin=True,
                   dropout=0.5)
    assert model.__repr__() == ('RelCNN(16, 32, num_layers=2, batch_norm=True'
                                ', cat=True, lin=True, dropout=0.5)')
    assert model.convs[0].__repr__() == 'RelConv(16, 32)'
    x = torch.randn(100, 16)
    edge_index = torch.randint(100, (2, 400), dtype=torch.long)
    for cat, lin in product([False, True], [False, True]):
        model = RelCNN(16, 32, 2, True, cat, lin, 0.5)
        out = model(x, edge_index)
        assert out.size() == (100, 16 + 2 * 32 if not lin and cat else 32)
        assert out.size() == (100, model.out_channels)


def test_spline():
    model = SplineCNN(16, 32, dim=3, num_layers=2, cat=True, lin=True,
                      dropout=0.5)
    assert model.__repr__() == ('SplineCNN(16, 32, dim=3, num_layers=2, '
                                'cat=True, lin=True, dropout=0.5)')
    x = torch.randn(100, 16)
    edge_index = torch.randint(100, (2, 400), dtype=torch.long)
    edge_attr = torch.rand((400, 3))
    for cat, lin in product([False, True], [False, True]):
        model = SplineCNN(16, 32, 3, 2, cat, lin, 0.5)
        out = model(x, edge_index, edge_attr)
        assert out.size() == (100, 16 + 2 * 32 if not lin and cat else 32)
        assert out.size() == (100, model.out_channels)
