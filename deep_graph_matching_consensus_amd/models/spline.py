"""SplineCNN encoder (API of ``/root/reference/dgmc/models/spline.py``).

``num_layers`` x ``SplineConv(kernel_size=5)`` each followed by ReLU (fused
into the aggregation kernel's epilogue here), optional concatenation,
dropout applied ONCE to the (concatenated) features (``spline.py:52``), then
the optional final ``Linear``.
"""
import torch
import torch.nn.functional as F
from torch.nn import ModuleList

from ..nn.conv import SplineConv
from ..ops import _backend, slot_gemm
from .encoder import StackedEncoder


class SplineCNN(StackedEncoder):
    def __init__(self, in_channels, out_channels, dim, num_layers, cat=True,
                 lin=True, dropout=0.0):
        super(SplineCNN, self).__init__()
        self.dim = dim
        self.dropout = dropout
        widths = [in_channels] + [out_channels] * num_layers
        self.convs = ModuleList([
            SplineConv(a, out_channels, dim, kernel_size=5)
            for a in widths[:-1]
        ])
        self._init_head(in_channels, out_channels, num_layers, cat, lin)
        self.reset_parameters()

    def reset_parameters(self):
        for conv in self.convs:
            conv.reset_parameters()
        if self.lin:
            self.final.reset_parameters()

    def takes_x6_planes(self, x):
        """Whether the first conv reads ``x`` (fp32) on the bf16x6 slot path:
        a producer may then hand it the operand planes as well (attached as
        ``x._dgmc_x6``; ops/slot_gemm.py)."""
        conv = self.convs[0] if len(self.convs) else None
        return (conv is not None and slot_gemm.X6 and
                slot_gemm.ENABLED and x.dtype == torch.float32 and
                conv.in_channels % 128 == 0 and conv.out_channels % 128 == 0
                and _backend.use_hip(x))

    def forward(self, x, edge_index, edge_attr, *args):
        xs = [x]
        last = len(self.convs) - 1
        for i, conv in enumerate(self.convs):
            # (a non-last layer's output feeds the next conv: on the fp32
            # bf16x6 path its aggregation also writes the operand planes)
            kw = {'planes_out': True} if i < last else {}
            if (self.cat and xs[-1].requires_grad and
                    torch.is_grad_enabled()):
                # xs[-1] also feeds the concatenation: route that consumer
                # through the conv's alias so both gradients meet inside
                # the conv backward (no separate add kernel).
                out, xs[-1] = conv(xs[-1], edge_index, edge_attr, act='relu',
                                   passthrough=True, **kw)
            else:
                out = conv(xs[-1], edge_index, edge_attr, act='relu', **kw)
            xs.append(out)
        parts = self._parts_out(xs)
        if parts is not None:
            return parts
        h = F.dropout(self._head(xs), p=self.dropout, training=self.training)
        return self._project(h)

    def __repr__(self):
        return ('{}({}, {}, dim={}, num_layers={}, cat={}, lin={}, '
                'dropout={})').format(type(self).__name__, self.in_channels,
                                      self.out_channels, self.dim,
                                      self.num_layers, self.cat, self.lin,
                                      self.dropout)
