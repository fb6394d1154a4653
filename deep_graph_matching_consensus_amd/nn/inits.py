"""Parameter initialisers (PyG ``torch_geometric.nn.inits`` semantics).

``reset`` is used by ``DGMC.reset_parameters``
(``/root/reference/dgmc/models/dgmc.py:5,83``); ``uniform`` is the
SplineConv initialiser (``U(+-1/sqrt(in * K))``).
"""
import math


def uniform(size, tensor):
    bound = 1.0 / math.sqrt(size)
    if tensor is not None:
        tensor.data.uniform_(-bound, bound)


def reset(nn):
    def _reset(item):
        if hasattr(item, 'reset_parameters'):
            item.reset_parameters()

    if nn is not None:
        if hasattr(nn, 'children') and len(list(nn.children())) > 0:
            for item in nn.children():
                _reset(item)
        else:
            _reset(nn)
