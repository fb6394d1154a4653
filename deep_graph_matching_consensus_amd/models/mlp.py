"""Multi-layer perceptron encoder
(API of ``/root/reference/dgmc/models/mlp.py``).

Layer schedule (``mlp.py:31-39``): every hidden ``Linear`` is followed by ReLU
and, if ``batch_norm``, BatchNorm1d; dropout is applied only to the input of
the *last* ``Linear``.  BatchNorm modules are always constructed so the
checkpoint carries ``batch_norms.i.*`` keys even with ``batch_norm=False``.
"""
import torch
import torch.nn.functional as F
from torch.nn import BatchNorm1d, Linear, ModuleList

from ..ops.gemm import linear


class MLP(torch.nn.Module):
    def __init__(self, in_channels, out_channels, num_layers,
                 batch_norm=False, dropout=0.0):
        super(MLP, self).__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_layers = num_layers
        self.batch_norm = batch_norm
        self.dropout = dropout

        widths = [in_channels] + [out_channels] * num_layers
        self.lins = ModuleList(
            [Linear(a, b) for a, b in zip(widths[:-1], widths[1:])])
        self.batch_norms = ModuleList(
            [BatchNorm1d(out_channels) for _ in range(num_layers)])
        self.reset_parameters()

    def reset_parameters(self):
        for module in list(self.lins) + list(self.batch_norms):
            module.reset_parameters()

    def forward(self, x, *args):
        last = self.num_layers - 1
        for depth in range(self.num_layers):
            lin = self.lins[depth]
            if depth == last:
                x = F.dropout(x, p=self.dropout, training=self.training)
                x = linear(x, lin.weight, lin.bias)
                break
            x = F.relu(linear(x, lin.weight, lin.bias))
            if self.batch_norm:
                x = self.batch_norms[depth](x)
        return x

    def __repr__(self):
        return '{}({}, {}, num_layers={}, batch_norm={}, dropout={})'.format(
            type(self).__name__, self.in_channels, self.out_channels,
            self.num_layers, self.batch_norm, self.dropout)
