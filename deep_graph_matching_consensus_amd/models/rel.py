"""Relational encoder (API of ``/root/reference/dgmc/models/rel.py``).

``RelConv`` (``rel.py:7-38``) computes
``root(x) + mean_{j->i} lin1(x)_j + mean_{i->j} lin2(x)_j`` by running
message passing twice with a mutated ``flow``.  Here the three linear maps are
stacked into ONE GEMM (``x @ [lin1 | lin2 | root]^T``) and both aggregation
directions plus the root term are a single sparse operator
(:func:`~..ops.plans.relational_plan`) evaluated by one gather-reduce kernel
(ReLU fused when the encoder has no BatchNorm).  Checkpoint keys are kept
(``lin1.weight``, ``lin2.weight``, ``root.weight``, ``root.bias``).
"""
import torch
import torch.nn.functional as F
from torch.nn import BatchNorm1d, Linear, ModuleList

from ..ops.gemm import compute_dtype
from ..ops.plans import relational_plan
from ..ops.sparse import gemm_spmm
from ..runtime.cache import cached
from .encoder import StackedEncoder


class RelConv(torch.nn.Module):
    def __init__(self, in_channels, out_channels):
        super(RelConv, self).__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.lin1 = Linear(in_channels, out_channels, bias=False)
        self.lin2 = Linear(in_channels, out_channels, bias=False)
        self.root = Linear(in_channels, out_channels)
        self.reset_parameters()

    def reset_parameters(self):
        for lin in (self.lin1, self.lin2, self.root):
            lin.reset_parameters()

    def stacked_weight(self):
        """``[in, 3 * out]`` fp32 operand ``[lin1 | lin2 | root]^T``,
        memoised per forward scope."""
        return cached(('rel_w', id(self)), lambda: torch.cat(
            [self.lin1.weight, self.lin2.weight, self.root.weight],
            dim=0).t())

    def forward(self, x, edge_index, act=None, passthrough=False):
        plan = relational_plan(edge_index, x.size(0))
        dtype = compute_dtype(x)
        w = self.stacked_weight()
        # (fp32: the GEMM reads the stacked weight in place - no copy)
        w_lp = w if dtype == w.dtype else cached(
            ('rel_w_lp', id(self), dtype),
            lambda: w.detach().to(dtype,
                                  memory_format=torch.contiguous_format))
        # root.bias enters through the root slot (coefficient 1) = output bias.
        return gemm_spmm(plan, x, w, w_lp, self.out_channels,
                         bias=self.root.bias, relu=(act == 'relu'),
                         loop_key=(id(self), x.size(0), plan.num_cols),
                         passthrough=passthrough)

    def __repr__(self):
        return '{}({}, {})'.format(type(self).__name__, self.in_channels,
                                   self.out_channels)


class RelCNN(StackedEncoder):
    def __init__(self, in_channels, out_channels, num_layers,
                 batch_norm=False, cat=True, lin=True, dropout=0.0):
        super(RelCNN, self).__init__()
        self.batch_norm = batch_norm
        self.dropout = dropout
        widths = [in_channels] + [out_channels] * num_layers
        self.convs = ModuleList(
            [RelConv(a, out_channels) for a in widths[:-1]])
        self.batch_norms = ModuleList(
            [BatchNorm1d(out_channels) for _ in range(num_layers)])
        self._init_head(in_channels, out_channels, num_layers, cat, lin)
        self.reset_parameters()

    def reset_parameters(self):
        for conv, bn in zip(self.convs, self.batch_norms):
            conv.reset_parameters()
            bn.reset_parameters()
        if self.lin:
            self.final.reset_parameters()

    def forward(self, x, edge_index, *args):
        xs = [x]
        for conv, bn in zip(self.convs, self.batch_norms):
            kw = {}
            if (self.cat and xs[-1].requires_grad and
                    torch.is_grad_enabled()):
                # xs[-1] also feeds the concatenation: that consumer reads
                # the conv's alias, so both gradients meet in the conv
                # backward (added in its dx GEMM epilogue).  'cat': the
                # alias feeds only _head's torch.cat (in-place accumulation
                # into that gradient slice is safe).
                kw = {'passthrough': 'cat'}
            if self.batch_norm:
                h = conv(xs[-1], edge_index, **kw)
                if kw:
                    h, xs[-1] = h
                h = bn(F.relu(h))
            else:
                h = conv(xs[-1], edge_index, act='relu', **kw)
                if kw:
                    h, xs[-1] = h
            xs.append(F.dropout(h, p=self.dropout, training=self.training))
        return self._head_project(xs)

    def __repr__(self):
        return ('{}({}, {}, num_layers={}, batch_norm={}, cat={}, lin={}, '
                'dropout={})').format(type(self).__name__, self.in_channels,
                                      self.out_channels, self.num_layers,
                                      self.batch_norm, self.cat, self.lin,
                                      self.dropout)
