"""Packed ``[sum N, C]`` <-> padded ``[B, N_max, C]`` conversions.

Replaces PyG's ``to_dense_batch`` (``/root/reference/dgmc/models/dgmc.py:4,
154-155``) and the boolean-mask ``to_sparse``/``to_dense`` helpers
(``dgmc.py:22-29``).  The reference versions index with boolean masks, which
forces a device->host sync (``nonzero``) on *every* call - ten times per
consensus step.  Here the flat dense index of every node is computed once on
the host from :class:`~.meta.BatchInfo` and cached on the device, so packing
and unpacking are single gather/scatter kernels with no synchronisation.
"""
import torch

from .meta import batch_info


class DenseLayout(object):
    """Mapping between packed node rows and a padded ``[B, N_max]`` grid."""

    def __init__(self, info, device, max_nodes=None):
        self.info = info
        self.B = info.num_graphs
        self.N = info.max_nodes if max_nodes is None else max_nodes
        self.device = device
        self.index = info.dense_index(device, self.N)        # [sum N] int64
        self.counts = info.device_tensor('counts', device, torch.int32)
        self.ptr = info.device_tensor('ptr', device, torch.int32)
        self.num_nodes = info.num_nodes
        # Static (padded) batches route padding rows to a trash slot B*N.
        self.trash = bool(getattr(info, 'has_trash', False))
        # No padding at all (e.g. batch=None, the full-graph KG path: B = 1):
        # the packed and dense layouts coincide, so both directions are
        # views - no fill / index_copy / index_select kernels (and none in
        # their backward).
        self.identity = not self.trash and self.B * self.N == self.num_nodes
        self._mask = None

    @property
    def mask(self):
        """``[B, N_max]`` bool validity mask."""
        if self._mask is None:
            m = torch.zeros(self.B * self.N + int(self.trash),
                            dtype=torch.bool, device=self.device)
            m[self.index] = True
            self._mask = m[:self.B * self.N].view(self.B, self.N)
        return self._mask

    def to_dense(self, x, fill_value=0.):
        """``[sum N, *]`` -> ``[B, N_max, *]`` (padding = ``fill_value``)."""
        feat = tuple(x.shape[1:])
        if self.identity:
            return x.reshape((self.B, self.N) + feat)
        rows = self.B * self.N
        out = x.new_full((rows + int(self.trash), ) + feat, fill_value)
        out = out.index_copy(0, self.index, x)
        if self.trash:
            out = out[:rows]
        return out.view((self.B, self.N) + feat)

    def to_sparse(self, x):
        """``[B, N_max, *]`` -> ``[sum N, *]``."""
        feat = tuple(x.shape[2:])
        flat = x.reshape((self.B * self.N, ) + feat)
        if self.identity:
            return flat
        if self.trash:
            flat = torch.cat([flat, flat.new_zeros((1, ) + feat)], dim=0)
        return flat.index_select(0, self.index)


class MaskLayout(object):
    """Reference-mode layout: sizes recovered from the device batch vector
    (two host syncs, like PyG's ``to_dense_batch``) and boolean-mask packing
    (``x[mask]``, one ``nonzero`` sync per call, like ``dgmc.py:22-29``)."""

    def __init__(self, batch, num_nodes, device):
        if batch is None:
            batch = torch.zeros(num_nodes, dtype=torch.long, device=device)
        self.B = int(batch[-1].item()) + 1 if num_nodes > 0 else 0
        counts = torch.zeros(self.B, dtype=torch.long, device=device)
        counts.scatter_add_(0, batch, torch.ones_like(batch))
        self.N = int(counts.max().item()) if self.B > 0 else 0
        self.counts = counts.to(torch.int32)
        self.num_nodes = num_nodes
        self.device = device
        ar = torch.arange(self.N, device=device).view(1, -1)
        self.mask = ar < counts.view(-1, 1)

    @property
    def index(self):
        return self.mask.view(-1).nonzero().view(-1)

    def to_dense(self, x, fill_value=0.):
        out = x.new_full((self.B, self.N) + tuple(x.shape[1:]), fill_value)
        out[self.mask] = x
        return out

    def to_sparse(self, x):
        return x[self.mask]


def dense_layout(batch, num_nodes, device, max_nodes=None):
    from ..runtime.mode import is_reference_mode
    if is_reference_mode():
        return MaskLayout(batch, num_nodes, device)
    return DenseLayout(batch_info(batch, num_nodes), device, max_nodes)


def to_dense_batch(x, batch=None, fill_value=0.):
    r"""Drop-in for PyG's ``to_dense_batch``: returns ``(dense, mask)``."""
    layout = dense_layout(batch, x.size(0), x.device)
    out = layout.to_dense(x, fill_value)
    if getattr(layout, 'identity', False):
        out = out.clone()    # PyG returns a new tensor, never a view of x
    return out, layout.mask
