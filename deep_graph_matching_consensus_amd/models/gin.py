"""GIN encoder (API of ``/root/reference/dgmc/models/gin.py``).

``num_layers`` GIN convolutions, each wrapping a 2-layer :class:`MLP`
(``train_eps=True``).  As in the reference there is **no** activation between
convolutions (``gin.py:48-49``); ``edge_attr`` is ignored.
"""
from torch.nn import ModuleList

from ..nn.conv import GINConv
from .encoder import StackedEncoder
from .mlp import MLP


class GIN(StackedEncoder):
    def __init__(self, in_channels, out_channels, num_layers,
                 batch_norm=False, cat=True, lin=True):
        super(GIN, self).__init__()
        self.batch_norm = batch_norm
        widths = [in_channels] + [out_channels] * num_layers
        self.convs = ModuleList([
            GINConv(MLP(a, out_channels, 2, batch_norm, dropout=0.0),
                    train_eps=True) for a in widths[:-1]
        ])
        self._init_head(in_channels, out_channels, num_layers, cat, lin)
        self.reset_parameters()

    def reset_parameters(self):
        for conv in self.convs:
            conv.reset_parameters()
        if self.lin:
            self.final.reset_parameters()

    def forward(self, x, edge_index, *args):
        xs = [x]
        for conv in self.convs:
            xs.append(conv(xs[-1], edge_index))
        return self._project(self._head(xs))

    def __repr__(self):
        return ('{}({}, {}, num_layers={}, batch_norm={}, cat={}, '
                'lin={})').format(type(self).__name__, self.in_channels,
                                  self.out_channels, self.num_layers,
                                  self.batch_norm, self.cat, self.lin)
