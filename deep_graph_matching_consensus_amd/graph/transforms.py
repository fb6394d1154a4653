"""Geometric graph transforms used by the reference drivers.

Re-implements (host-side, once per graph) the PyG 1.4 transforms the
reference composes:

* ``Delaunay`` + ``FaceToEdge`` + ``Cartesian``/``Distance`` for keypoint
  graphs (``/root/reference/examples/pascal.py:24-29``, ``willow.py:30-35``);
* ``Constant`` + ``KNNGraph(k=8)`` + ``Cartesian`` for PascalPF
  (``/root/reference/examples/pascal_pf.py:68-72``).

Delaunay triangulation uses scipy's qhull (as PyG does).  Pseudo-coordinates
follow PyG 1.4's sign convention ``pos[col] - pos[row]`` normalised into
``[0, 1]^D`` so they can index open B-spline kernels directly.
"""
import numpy as np
import scipy.spatial
import torch


class Compose(object):
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data

    def __repr__(self):
        args = ['    {},'.format(t) for t in self.transforms]
        return '{}([\n{}\n])'.format(self.__class__.__name__, '\n'.join(args))


def coalesce_undirected(edge_index, num_nodes):
    """``to_undirected`` + ``coalesce``: symmetric, sorted (row, col),
    unique."""
    row, col = edge_index
    row, col = torch.cat([row, col]), torch.cat([col, row])
    key = torch.unique(row * num_nodes + col)
    return torch.stack([key // num_nodes, key % num_nodes], dim=0)


class Delaunay(object):
    r"""Computes the Delaunay triangulation of ``pos`` into ``face``."""

    def __call__(self, data):
        pos = data.pos
        n = pos.size(0)
        if n < 2:
            data.edge_index = torch.empty((2, 0), dtype=torch.long)
        elif n == 2:
            data.edge_index = torch.tensor([[0, 1], [1, 0]])
        elif n == 3:
            data.face = torch.tensor([[0], [1], [2]])
        else:
            tri = scipy.spatial.Delaunay(pos.detach().cpu().numpy(),
                                         qhull_options='QJ')
            face = torch.from_numpy(tri.simplices.astype(np.int64))
            data.face = face.t().contiguous()
        return data

    def __repr__(self):
        return '{}()'.format(self.__class__.__name__)


class FaceToEdge(object):
    r"""Converts triangle faces ``[3, F]`` into undirected ``edge_index``."""

    def __init__(self, remove_faces=True):
        self.remove_faces = remove_faces

    def __call__(self, data):
        if data.face is not None:
            face = data.face
            edge_index = torch.cat([face[:2], face[1:], face[::2]], dim=1)
            data.edge_index = coalesce_undirected(edge_index, data.num_nodes)
            if self.remove_faces:
                data.face = None
        return data

    def __repr__(self):
        return '{}()'.format(self.__class__.__name__)


class Cartesian(object):
    r"""Saves relative Cartesian coordinates of linked nodes in ``edge_attr``.

    ``norm=True`` maps them into ``[0, 1]^D`` via ``c / (2 max|c|) + 0.5``.
    """

    def __init__(self, norm=True, max_value=None, cat=True):
        self.norm, self.max, self.cat = norm, max_value, cat

    def __call__(self, data):
        (row, col), pos, pseudo = data.edge_index, data.pos, data.edge_attr
        cart = pos[col] - pos[row]
        cart = cart.view(-1, 1) if cart.dim() == 1 else cart
        if self.norm and cart.numel() > 0:
            max_value = cart.abs().max() if self.max is None else self.max
            cart = cart / (2 * max_value) + 0.5
        if pseudo is not None and self.cat:
            pseudo = pseudo.view(-1, 1) if pseudo.dim() == 1 else pseudo
            data.edge_attr = torch.cat([pseudo, cart.type_as(pseudo)], -1)
        else:
            data.edge_attr = cart
        return data

    def __repr__(self):
        return '{}(norm={}, max_value={})'.format(self.__class__.__name__,
                                                  self.norm, self.max)


class Distance(object):
    r"""Saves the (normalised) Euclidean distance of linked nodes."""

    def __init__(self, norm=True, max_value=None, cat=True):
        self.norm, self.max, self.cat = norm, max_value, cat

    def __call__(self, data):
        (row, col), pos, pseudo = data.edge_index, data.pos, data.edge_attr
        dist = torch.norm(pos[col] - pos[row], p=2, dim=-1).view(-1, 1)
        if self.norm and dist.numel() > 0:
            dist = dist / (dist.max() if self.max is None else self.max)
        if pseudo is not None and self.cat:
            pseudo = pseudo.view(-1, 1) if pseudo.dim() == 1 else pseudo
            data.edge_attr = torch.cat([pseudo, dist.type_as(pseudo)], -1)
        else:
            data.edge_attr = dist
        return data

    def __repr__(self):
        return '{}(norm={}, max_value={})'.format(self.__class__.__name__,
                                                  self.norm, self.max)


class Constant(object):
    r"""Adds a constant node feature (``x = value``, concatenated if
    ``cat``)."""

    def __init__(self, value=1, cat=True):
        self.value, self.cat = value, cat

    def __call__(self, data):
        c = torch.full((data.num_nodes, 1), float(self.value))
        if data.x is not None and self.cat:
            x = data.x.view(-1, 1) if data.x.dim() == 1 else data.x
            data.x = torch.cat([x, c.to(x.dtype)], dim=-1)
        else:
            data.x = c
        return data

    def __repr__(self):
        return '{}(value={})'.format(self.__class__.__name__, self.value)


def knn_graph(pos, k, loop=False):
    """Edges ``neighbour -> centre`` (``source_to_target`` flow)."""
    n = pos.size(0)
    if n <= 1:
        return torch.empty((2, 0), dtype=torch.long)
    dist = torch.cdist(pos, pos)
    if not loop:
        dist.fill_diagonal_(float('inf'))
    kk = min(k, n if loop else n - 1)
    nbr = dist.topk(kk, dim=1, largest=False).indices  # [n, kk]
    centre = torch.arange(n).view(-1, 1).expand(-1, kk)
    return torch.stack([nbr.reshape(-1), centre.reshape(-1)], dim=0)


class KNNGraph(object):
    r"""Creates a k-NN graph from ``pos`` (``edge_attr`` is reset)."""

    def __init__(self, k=6, loop=False, force_undirected=False):
        self.k, self.loop, self.force_undirected = k, loop, force_undirected

    def __call__(self, data):
        data.edge_attr = None
        edge_index = knn_graph(data.pos, self.k, self.loop)
        if self.force_undirected:
            edge_index = coalesce_undirected(edge_index, data.num_nodes)
        data.edge_index = edge_index
        return data

    def __repr__(self):
        return '{}(k={})'.format(self.__class__.__name__, self.k)
