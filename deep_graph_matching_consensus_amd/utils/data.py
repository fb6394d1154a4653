"""Graph-pair datasets (API of ``/root/reference/dgmc/utils/data.py``).

* :class:`PairData` - a :class:`~..graph.Data` holding a source and a target
  graph; ``*index_s*`` keys are offset by ``x_s`` rows and ``*index_t*`` keys
  by ``x_t`` rows during collation, every other key (including ``y``) by 0 so
  ``y`` stays a *local* target column (``data.py:9-16``).
* :class:`PairDataset` - Cartesian product of two datasets, or one random
  partner per source when ``sample=True`` (``data.py:19-60``).
* :class:`ValidPairDataset` - only pairs whose source keypoint classes are a
  subset of the target's, with the ground-truth map
  ``y[i] = position in the target of source node i's class``
  (``data.py:63-133``).  Pair validity is evaluated with one boolean
  matrix product over class-incidence matrices.
"""
import random
import re

import torch

from ..graph.data import Data


class PairData(Data):  # pragma: no cover
    def __inc__(self, key, value):
        if re.search('index_s', key):
            return self.x_s.size(0)
        if re.search('index_t', key):
            return self.x_t.size(0)
        return 0


def _pair(data_s, data_t, **extra):
    return PairData(x_s=data_s.x, edge_index_s=data_s.edge_index,
                    edge_attr_s=data_s.edge_attr, x_t=data_t.x,
                    edge_index_t=data_t.edge_index,
                    edge_attr_t=data_t.edge_attr, num_nodes=None, **extra)


class PairDataset(torch.utils.data.Dataset):
    r"""All (source, target) combinations, or one random target per source.

    Args:
        dataset_s, dataset_t: source / target datasets of :class:`Data`.
        sample (bool): draw one random target per source example.
    """

    def __init__(self, dataset_s, dataset_t, sample=False):
        self.dataset_s = dataset_s
        self.dataset_t = dataset_t
        self.sample = sample

    def __len__(self):
        n_s, n_t = len(self.dataset_s), len(self.dataset_t)
        return n_s if self.sample else n_s * n_t

    def __getitem__(self, idx):
        n_t = len(self.dataset_t)
        if self.sample:
            i, j = idx, random.randint(0, n_t - 1)
        else:
            i, j = divmod(idx, n_t)
        return _pair(self.dataset_s[i], self.dataset_t[j])

    def __repr__(self):
        return '{}({}, {}, sample={})'.format(type(self).__name__,
                                              self.dataset_s, self.dataset_t,
                                              self.sample)


class ValidPairDataset(torch.utils.data.Dataset):
    r"""Pairs in which every source node class also occurs in the target.

    Args:
        dataset_s, dataset_t: datasets of :class:`Data` with per-node class
            labels ``y``.
        sample (bool): draw one random valid target per source example.
    """

    def __init__(self, dataset_s, dataset_t, sample=False):
        self.dataset_s = dataset_s
        self.dataset_t = dataset_t
        self.sample = sample
        self.pairs, self.cumdeg = self.__compute_pairs__()

    @staticmethod
    def _incidence(dataset, num_classes):
        inc = torch.zeros((len(dataset), num_classes), dtype=torch.bool)
        for i, data in enumerate(dataset):
            inc[i, data.y] = True
        return inc

    def __compute_pairs__(self):
        labels = [d.y for d in self.dataset_s] + [d.y for d in self.dataset_t]
        num_classes = max(int(y.max()) + 1 for y in labels)
        inc_s = self._incidence(self.dataset_s, num_classes).float()
        inc_t = self._incidence(self.dataset_t, num_classes).float()
        # |classes(s) & classes(t)| == |classes(s)|  <=>  classes(s) <= t
        overlap = inc_s @ inc_t.t()
        valid = overlap == inc_s.sum(dim=1, keepdim=True)
        pairs = valid.nonzero()
        per_source = torch.bincount(pairs[:, 0], minlength=len(inc_s))
        cumdeg = torch.cat([torch.zeros(1, dtype=torch.long),
                            per_source.cumsum(0)])
        return pairs.tolist(), cumdeg.tolist()

    def __len__(self):
        return len(self.dataset_s) if self.sample else len(self.pairs)

    def __getitem__(self, idx):
        if self.sample:
            data_s = self.dataset_s[idx]
            lo, hi = self.cumdeg[idx], self.cumdeg[idx + 1]
            data_t = self.dataset_t[self.pairs[random.randint(lo, hi - 1)][1]]
        else:
            i, j = self.pairs[idx]
            data_s, data_t = self.dataset_s[i], self.dataset_t[j]

        position = torch.full((int(data_t.y.max()) + 1, ), -1,
                              dtype=data_s.y.dtype)
        position[data_t.y] = torch.arange(data_t.num_nodes,
                                          dtype=data_s.y.dtype)
        return _pair(data_s, data_t, y=position[data_s.y])

    def __repr__(self):
        return '{}({}, {}, sample={})'.format(type(self).__name__,
                                              self.dataset_s, self.dataset_t,
                                              self.sample)
