"""Shared skeleton of the stacked GNN encoders (GIN, SplineCNN, RelCNN).

All three reference encoders (``/root/reference/dgmc/models/gin.py``,
``spline.py``, ``rel.py``) share the same output rule
(``gin.py:25-34``): features of all layers are optionally concatenated
(``cat``, including the input) and optionally projected by a final
``Linear`` (``lin``)::

    out_channels = out            if lin
                 = in + L * out   if cat and not lin
                 = out            otherwise

``pair_fusable`` tells :class:`~..models.dgmc.DGMC` that encoding the source
and target graphs in ONE call on their disjoint union gives the same result as
two calls (true unless BatchNorm runs in training mode), which halves the
kernel launches and doubles GEMM sizes on the hot path.
"""
import contextlib

import torch
from torch.nn import Linear

from ..ops.gemm import linear, linear_parts


class CatParts(object):
    """The concatenation ``torch.cat(parts, -1)`` left unformed: a consumer
    that reads the parts directly (``ops/dense.py::cat_matmul``) skips the
    copy; :meth:`cat` forms it for any other consumer."""

    def __init__(self, parts):
        self.parts = list(parts)

    def cat(self):
        return torch.cat(self.parts, dim=-1)

    def size(self, dim=None):
        n = self.parts[0].size(0)
        c = sum(p.size(-1) for p in self.parts)
        return torch.Size([n, c]) if dim is None else (n, c)[dim]

    @property
    def dtype(self):
        return self.parts[0].dtype


class StackedEncoder(torch.nn.Module):
    def _init_head(self, in_channels, out_channels, num_layers, cat, lin):
        self.in_channels = in_channels
        self.num_layers = num_layers
        self.cat = cat
        self.lin = lin
        width = in_channels + num_layers * out_channels if cat \
            else out_channels
        if lin:
            self.out_channels = out_channels
            self.final = Linear(width, out_channels)
        else:
            self.out_channels = width

    def _head(self, xs):
        x = torch.cat(xs, dim=-1) if self.cat else xs[-1]
        return x

    def _project(self, x):
        if not self.lin or getattr(self, '_features_only', False):
            return x
        return linear(x, self.final.weight, self.final.bias)

    def _head_project(self, xs):
        """``_project(_head(xs))``; with ``cat`` and the final Linear the
        layer features are read in place by one GEMM (no concatenation)."""
        if self.cat and self.lin and not getattr(self, '_features_only',
                                                 False):
            return linear_parts(xs, self.final.weight, self.final.bias)
        return self._project(self._head(xs))

    @contextlib.contextmanager
    def features_only(self):
        """Inside the block ``forward`` returns the features BEFORE the final
        ``Linear`` (callers that fold the projection into a following linear
        map, e.g. DGMC's consensus MLP)."""
        prev = getattr(self, '_features_only', False)
        self._features_only = True
        try:
            yield self
        finally:
            self._features_only = prev

    @contextlib.contextmanager
    def features_parts(self):
        """Like :meth:`features_only`, and with ``cat=True`` (and no active
        dropout) ``forward`` returns the layer features as a
        :class:`CatParts` instead of concatenating them."""
        prev = getattr(self, '_features_parts', False)
        self._features_parts = True
        try:
            with self.features_only():
                yield self
        finally:
            self._features_parts = prev

    def _parts_out(self, xs):
        """:class:`CatParts` of ``xs`` when :meth:`features_parts` applies."""
        if (getattr(self, '_features_parts', False) and self.cat and
                (getattr(self, 'dropout', 0.0) == 0.0 or not self.training)):
            return CatParts(xs)
        return None

    @property
    def pair_fusable(self):
        for m in self.modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and \
                    m.training and getattr(self, 'batch_norm', False):
                return False
        return True
