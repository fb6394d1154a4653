"""Synthetic random-graph pair datasets.

* :class:`RandomGraphDataset` - the PascalPF training generator of the
  reference (``/root/reference/examples/pascal_pf.py:23-65``): 30-60 inlier
  keypoints in ``[-1, 1]^2`` with a jittered copy as target (Gaussian noise
  0.05), 0-20 outliers in ``(2, 3]^2`` added to both, each graph transformed
  independently (``Constant -> KNNGraph(8) -> Cartesian``), stored as ONE
  ``Data`` with ``_s``/``_t`` suffixed keys and ``num_nodes = N_s`` so that
  default collation offsets every ``*index*`` key by ``N_s`` (the
  reference's behaviour; ``y_index_s`` becomes a global source row, ``y_t``
  stays local).  ``min_scale``/``max_scale`` are stored but unused, like the
  reference.
* :func:`make_er_pair` - BASELINE config 1: an Erdos-Renyi source graph and a
  node-permuted, edge-perturbed target with noisy shared node features.
"""
import random

import torch

from ..graph.data import Data
from ..graph import transforms as T


def pascal_pf_transform():
    """``Constant -> KNNGraph(k=8) -> Cartesian`` (``pascal_pf.py:68-72``)."""
    return T.Compose([T.Constant(), T.KNNGraph(k=8), T.Cartesian()])


class RandomGraphDataset(torch.utils.data.Dataset):
    def __init__(self, min_inliers, max_inliers, min_outliers, max_outliers,
                 min_scale=0.9, max_scale=1.2, noise=0.05, transform=None,
                 length=1024):
        self.min_inliers, self.max_inliers = min_inliers, max_inliers
        self.min_outliers, self.max_outliers = min_outliers, max_outliers
        self.min_scale, self.max_scale = min_scale, max_scale
        self.noise = noise
        self.transform = transform
        self.length = length

    def __len__(self):
        return self.length

    def _side(self, pos, outliers, **extra):
        pos = torch.cat([pos, 3 - torch.rand((outliers, 2))], dim=0)
        data = Data(pos=pos, **extra)
        return self.transform(data) if self.transform is not None else data

    def __getitem__(self, idx):
        n_in = random.randint(self.min_inliers, self.max_inliers)
        n_out = random.randint(self.min_outliers, self.max_outliers)
        pos_s = 2 * torch.rand((n_in, 2)) - 1
        pos_t = pos_s + self.noise * torch.randn_like(pos_s)
        data_s = self._side(pos_s, n_out, y_index=torch.arange(n_in))
        data_t = self._side(pos_t, n_out, y=torch.arange(n_in))
        data = Data(num_nodes=data_s.pos.size(0))
        for key, item in data_s:
            data['{}_s'.format(key)] = item
        for key, item in data_t:
            data['{}_t'.format(key)] = item
        return data


def _er_edges(n, p, g):
    mask = torch.rand((n, n), generator=g) < p
    mask = torch.triu(mask, diagonal=1)
    mask = mask | mask.t()
    return mask.nonzero().t().contiguous()


def make_er_pair(num_nodes=20, p=0.2, feature_dim=32, feature_noise=1.0,
                 edge_noise=0.05, seed=0):
    r"""Erdos-Renyi pair ``(data_s, data_t, y)``: ``G_t`` is a node-permuted
    copy of ``G_s`` with ``edge_noise`` of its edges rewired; node features
    are shared up to Gaussian noise.  ``y [2, N]`` maps source -> target."""
    g = torch.Generator().manual_seed(seed)
    ei_s = _er_edges(num_nodes, p, g)
    perm = torch.randperm(num_nodes, generator=g)
    ei_t = perm[ei_s]
    E = ei_t.size(1)
    rewire = torch.rand(E, generator=g) < edge_noise
    ei_t[1, rewire] = torch.randint(num_nodes, (int(rewire.sum()), ),
                                    generator=g)
    keep = ei_t[0] != ei_t[1]
    ei_t = ei_t[:, keep]
    x_s = torch.randn((num_nodes, feature_dim), generator=g)
    x_t = torch.empty_like(x_s)
    x_t[perm] = x_s + feature_noise * torch.randn(x_s.shape, generator=g)
    y = torch.stack([torch.arange(num_nodes), perm], dim=0)
    return Data(x=x_s, edge_index=ei_s), Data(x=x_t, edge_index=ei_t), y
