"""Graph containers: ``Data`` (one graph / one pair) and ``Batch`` (collated).

The reference builds on PyTorch-Geometric 1.4's ``Data``/``Batch``
(``/root/reference/dgmc/utils/data.py:6``, ``examples/pascal.py:7``).  PyG is
not a dependency of this framework; this module re-implements the subset of
its semantics the matching pipeline relies on:

* attribute-style storage, ``keys`` (sorted, ``None`` values skipped),
  ``len(data)`` = number of keys, PyG-style ``repr`` (``Data(x=[10, 16])``);
* ``__cat_dim__`` (-1 for ``*index*``/``face`` keys, else 0) and ``__inc__``
  (``num_nodes`` for ``*index*``/``face`` keys, else 0) used by collation;
* ``Batch.from_data_list(..., follow_batch=[...])`` producing ``batch`` and
  ``<key>_batch`` assignment vectors plus host-side ``ptr`` metadata.

Beyond PyG, collation records the per-graph node counts on the host
(:mod:`.meta`) so that the device forward never has to synchronise to learn
``B``/``N_max`` (the reference pays two host syncs per ``to_dense_batch``,
SURVEY.md N7).
"""
import re

import torch

from .meta import register_batch_info


def _size_repr(value):
    if torch.is_tensor(value):
        return list(value.size())
    if isinstance(value, (int, float, bool)):
        return value
    if isinstance(value, (list, tuple)):
        return [len(value)]
    if isinstance(value, dict):
        return '{...}'
    return value


class Data(object):
    r"""A plain attribute container for one graph (or one graph pair).

    Args mirror PyG: ``x``, ``edge_index``, ``edge_attr``, ``y``, ``pos``,
    ``norm``, ``face`` plus arbitrary keyword attributes.
    """

    def __init__(self, x=None, edge_index=None, edge_attr=None, y=None,
                 pos=None, norm=None, face=None, **kwargs):
        self.x = x
        self.edge_index = edge_index
        self.edge_attr = edge_attr
        self.y = y
        self.pos = pos
        self.norm = norm
        self.face = face
        for key, item in kwargs.items():
            if key == 'num_nodes':
                self.__num_nodes__ = item
            else:
                self[key] = item

    # -- dict-like interface -------------------------------------------------
    def __getitem__(self, key):
        return getattr(self, key, None)

    def __setitem__(self, key, value):
        setattr(self, key, value)

    @property
    def keys(self):
        keys = [key for key in self.__dict__.keys()
                if self[key] is not None and not key.startswith('__')]
        return sorted(keys)

    def __len__(self):
        return len(self.keys)

    def __contains__(self, key):
        return key in self.keys

    def __iter__(self):
        for key in self.keys:
            yield key, self[key]

    def __call__(self, *keys):
        for key in sorted(self.keys) if not keys else keys:
            if key in self:
                yield key, self[key]

    # -- collation rules -----------------------------------------------------
    def __cat_dim__(self, key, value):
        return -1 if bool(re.search('(index|face)', key)) else 0

    def __inc__(self, key, value):
        return self.num_nodes if bool(re.search('(index|face)', key)) else 0

    # -- shape helpers -------------------------------------------------------
    @property
    def num_nodes(self):
        if hasattr(self, '__num_nodes__'):
            return self.__num_nodes__
        for key, item in self('x', 'pos', 'norm'):
            return item.size(0)
        if self.edge_index is not None and self.edge_index.numel() > 0:
            return int(self.edge_index.max()) + 1
        return None

    @num_nodes.setter
    def num_nodes(self, num_nodes):
        self.__num_nodes__ = num_nodes

    @property
    def num_edges(self):
        for key, item in self('edge_index', 'edge_attr'):
            return item.size(self.__cat_dim__(key, item))
        return None

    @property
    def num_node_features(self):
        if self.x is None:
            return 0
        return 1 if self.x.dim() == 1 else self.x.size(1)

    @property
    def num_features(self):
        return self.num_node_features

    @property
    def num_edge_features(self):
        if self.edge_attr is None:
            return 0
        return 1 if self.edge_attr.dim() == 1 else self.edge_attr.size(1)

    # -- device movement -----------------------------------------------------
    def apply(self, func, *keys):
        for key, item in self(*keys):
            if torch.is_tensor(item):
                self[key] = func(item)
        return self

    def to(self, device, *keys, **kwargs):
        return self.apply(lambda x: x.to(device, **kwargs), *keys)

    def clone(self):
        out = self.__class__.__new__(self.__class__)
        for key, item in self.__dict__.items():
            out.__dict__[key] = item.clone() if torch.is_tensor(item) else item
        return out

    def __repr__(self):
        info = ['{}={}'.format(key, _size_repr(item)) for key, item in self]
        return '{}({})'.format(self.__class__.__name__, ', '.join(info))


class Batch(Data):
    r"""A batch of graphs collated into one big disconnected graph.

    ``batch`` maps nodes to graphs; ``<key>_batch`` vectors are created for
    every key in ``follow_batch``.  Host-side ``ptr`` offsets are registered
    with :func:`register_batch_info` so that downstream dense packing is
    sync-free.
    """

    def __init__(self, batch=None, **kwargs):
        super(Batch, self).__init__(**kwargs)
        self.batch = batch
        self.__data_class__ = Data
        self.__slices__ = None

    @staticmethod
    def from_data_list(data_list, follow_batch=[]):
        keys = sorted(set.union(*[set(data.keys) for data in data_list]))
        assert 'batch' not in keys

        batch = Batch()
        batch.__data_class__ = data_list[0].__class__
        for key in keys + ['batch']:
            batch[key] = []
        for key in follow_batch:
            batch['{}_batch'.format(key)] = []

        cumsum = {key: 0 for key in keys}
        counts = {key: [] for key in follow_batch}
        num_nodes_list = []
        for i, data in enumerate(data_list):
            for key in data.keys:
                item = data[key]
                if torch.is_tensor(item) and item.dtype != torch.bool:
                    inc = cumsum[key]
                    item = item + inc if inc != 0 else item
                batch[key].append(item)
                cumsum[key] = cumsum[key] + data.__inc__(key, item)
            for key in follow_batch:
                size = data[key].size(data.__cat_dim__(key, data[key]))
                counts[key].append(size)
                batch['{}_batch'.format(key)].append(
                    torch.full((size, ), i, dtype=torch.long))
            num_nodes = data.num_nodes
            num_nodes_list.append(num_nodes)
            if num_nodes is not None:
                batch.batch.append(
                    torch.full((num_nodes, ), i, dtype=torch.long))

        if num_nodes_list and num_nodes_list[0] is None:
            batch.batch = None

        for key in batch.keys:
            item = batch[key]
            if not isinstance(item, list) or len(item) == 0:
                continue
            if torch.is_tensor(item[0]):
                batch[key] = torch.cat(
                    item, dim=data_list[0].__cat_dim__(key, item[0]))
            elif isinstance(item[0], (int, float)):
                batch[key] = torch.tensor(item)

        batch.__num_graphs__ = len(data_list)
        for key in follow_batch:
            register_batch_info(batch['{}_batch'.format(key)], counts[key])
        if batch.batch is not None and None not in num_nodes_list:
            register_batch_info(batch.batch, num_nodes_list)
        return batch.contiguous()

    def contiguous(self):
        return self.apply(lambda x: x.contiguous())

    def apply(self, func, *keys):
        from .meta import transfer_batch_info
        for key, item in self(*keys):
            if torch.is_tensor(item):
                new = func(item)
                if new is not item:
                    transfer_batch_info(item, new)
                self[key] = new
        return self

    @property
    def num_graphs(self):
        if hasattr(self, '__num_graphs__'):
            return self.__num_graphs__
        return int(self.batch[-1]) + 1

    @property
    def keys(self):
        keys = [key for key in self.__dict__.keys()
                if self[key] is not None and not key.startswith('__')]
        return sorted(keys)
