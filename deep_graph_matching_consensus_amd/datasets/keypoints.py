"""Synthetic keypoint-graph datasets shaped like PascalVOC-Keypoints / WILLOW.

The reference trains on PyG's ``PascalVOCKeypoints`` and ``WILLOWObjectClass``
(``/root/reference/examples/pascal.py:31-41``, ``willow.py:37-49``): per
image, the visible annotated keypoints of one object category become nodes
with 1024-d VGG16 features, connected by a Delaunay triangulation with
Cartesian pseudo-coordinates.  Those datasets (and torchvision/VGG) are not
available offline, so this module generates graphs with the same structure:

* every category has a fixed set of keypoint classes (``num_keypoints``,
  approximating the Berkeley annotation counts, 6-19 per category) with a
  canonical 2-D layout and a latent 1024-d appearance vector per class;
* an instance shows a random subset of the keypoints (``visible_prob``,
  at least ``min_nodes``), placed by a random similarity transform of the
  layout plus jitter, with features = class appearance + instance noise;
* node labels ``y`` are the keypoint-class ids, so ``ValidPairDataset``
  builds exactly the reference's pairs (target classes superset of source
  classes) and ground truths.

Matching is learnable (features and geometry are informative but noisy), so
training curves and Hits@1 behave like the real task; absolute accuracies are
of course not comparable with the paper's PascalVOC numbers.
"""
import math

import torch

from ..graph.data import Data
from ..graph import transforms as T

# (category, number of keypoint classes).  Approximate Berkeley annotations
# of PascalVOC (pyg PascalVOCKeypoints.categories order).
PASCAL_VOC_CATEGORIES = [
    ('aeroplane', 16), ('bicycle', 11), ('bird', 12), ('boat', 11),
    ('bottle', 8), ('bus', 8), ('car', 13), ('cat', 16), ('chair', 10),
    ('cow', 16), ('diningtable', 8), ('dog', 16), ('horse', 16),
    ('motorbike', 10), ('person', 19), ('pottedplant', 6), ('sheep', 16),
    ('sofa', 12), ('train', 7), ('tvmonitor', 8),
]

# WILLOW-ObjectClass: 5 categories, always exactly 10 visible keypoints.
WILLOW_CATEGORIES = [('face', 10), ('motorbike', 10), ('car', 10),
                     ('duck', 10), ('winebottle', 10)]


def keypoint_transform(isotropic=False):
    """``Delaunay -> FaceToEdge -> Cartesian`` (or ``Distance``), as in
    ``/root/reference/examples/pascal.py:24-29``."""
    return T.Compose([
        T.Delaunay(),
        T.FaceToEdge(),
        T.Distance() if isotropic else T.Cartesian(),
    ])


class KeypointCategory(object):
    """Latent description of one object category."""

    def __init__(self, name, num_keypoints, feature_dim, generator):
        self.name = name
        self.num_keypoints = num_keypoints
        g = generator
        self.layout = torch.rand((num_keypoints, 2), generator=g) * 2 - 1
        self.appearance = torch.randn((num_keypoints, feature_dim),
                                      generator=g)


class KeypointGraphDataset(torch.utils.data.Dataset):
    r"""In-memory dataset of keypoint graphs of ONE category.

    Args:
        category (KeypointCategory): latent category description.
        num_graphs (int): number of instances.
        visible_prob (float): per-keypoint visibility probability.
        min_nodes (int): minimum number of visible keypoints.
        feature_noise (float): std of the per-instance feature noise.
        pos_noise (float): std of the keypoint jitter.
        transform (callable): applied once at construction (pre_transform).
        seed (int): generator seed.
    """

    def __init__(self, category, num_graphs, visible_prob=0.75, min_nodes=3,
                 feature_noise=6.0, pos_noise=0.05, transform=None, seed=0):
        self.category = category
        g = torch.Generator().manual_seed(seed)
        self.graphs = [
            self._instance(g, visible_prob, min_nodes, feature_noise,
                           pos_noise, transform) for _ in range(num_graphs)
        ]

    def _instance(self, g, visible_prob, min_nodes, feature_noise,
                  pos_noise, transform):
        cat = self.category
        K = cat.num_keypoints
        vis = torch.rand(K, generator=g) < visible_prob
        if int(vis.sum()) < min(min_nodes, K):
            order = torch.randperm(K, generator=g)[:min(min_nodes, K)]
            vis[order] = True
        y = vis.nonzero().view(-1)
        # Random similarity transform of the canonical layout + jitter.
        angle = (torch.rand(1, generator=g).item() - 0.5) * math.pi / 3
        scale = 0.8 + 0.4 * torch.rand(1, generator=g).item()
        rot = torch.tensor([[math.cos(angle), -math.sin(angle)],
                            [math.sin(angle), math.cos(angle)]])
        shift = torch.rand((1, 2), generator=g) - 0.5
        pos = scale * cat.layout[y] @ rot.t() + shift
        pos = pos + pos_noise * torch.randn(pos.shape, generator=g)
        x = cat.appearance[y] + feature_noise * torch.randn(
            (y.numel(), cat.appearance.size(1)), generator=g)
        data = Data(x=x, pos=pos, y=y)
        if transform is not None:
            data = transform(data)
        return data

    def __len__(self):
        return len(self.graphs)

    def __getitem__(self, idx):
        return self.graphs[idx]

    @property
    def num_node_features(self):
        return self.graphs[0].num_node_features

    @property
    def num_edge_features(self):
        return self.graphs[0].num_edge_features

    def __repr__(self):
        return '{}({}, {})'.format(type(self).__name__, self.category.name,
                                   len(self))


def make_keypoint_datasets(categories=PASCAL_VOC_CATEGORIES, graphs=64,
                           feature_dim=1024, visible_prob=0.75, min_nodes=3,
                           feature_noise=6.0, transform=None, seed=0,
                           split='train'):
    """One :class:`KeypointGraphDataset` per category.  Calls with the same
    ``seed`` share the latent categories; ``split`` selects independent
    instances (``'train'`` / ``'test'``)."""
    if transform is None:
        transform = keypoint_transform()
    g = torch.Generator().manual_seed(seed)
    out = []
    for i, (name, K) in enumerate(categories):
        cat = KeypointCategory(name, K, feature_dim, g)
        out.append(KeypointGraphDataset(
            cat, graphs, visible_prob, min_nodes, feature_noise,
            transform=transform,
            seed=seed * 1000 + i + 1 + (0 if split == 'train' else 500)))
    return out
