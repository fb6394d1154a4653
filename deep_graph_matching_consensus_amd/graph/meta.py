"""Host-side metadata for batch-assignment vectors (sync-free dense packing).

``to_dense_batch`` in the reference (PyG, called at
``/root/reference/dgmc/models/dgmc.py:154-155``) derives the number of graphs
``B`` and the largest graph ``N_max`` from the device ``batch`` vector, which
costs two device->host synchronisations per call.  Our collation already
knows the per-graph node counts on the host, so it *registers* them against
the batch tensor here.  Lookups are identity based (weak references), and the
record is forwarded when a batch moves between devices (``Batch.to``).

When no record exists (a user-built batch vector) :func:`batch_info` falls
back to computing it, paying one synchronisation.
"""
import weakref

import torch

_REGISTRY = {}


def _upload(t, device):
    """Async H2D copy from pinned memory (never stalls the GPU queue)."""
    device = torch.device(device)
    if device.type == 'cuda':
        return t.pin_memory().to(device, non_blocking=True)
    return t.to(device)


class BatchInfo(object):
    """Per-graph node counts of a sorted, contiguous batch vector."""

    __slots__ = ('counts', 'ptr', 'num_graphs', 'max_nodes', 'num_nodes',
                 '_device_cache', '__weakref__')

    has_trash = False

    def __init__(self, counts):
        counts = torch.as_tensor(counts, dtype=torch.long).cpu()
        self.counts = counts
        self.ptr = torch.zeros(counts.numel() + 1, dtype=torch.long)
        if counts.numel() > 0:
            torch.cumsum(counts, 0, out=self.ptr[1:])
        self.num_graphs = int(counts.numel())
        self.max_nodes = int(counts.max()) if counts.numel() > 0 else 0
        self.num_nodes = int(self.ptr[-1])
        self._device_cache = {}

    def dense_index(self, device, max_nodes=None):
        """``[num_nodes]`` flat index of every node in a ``[B * N_max]``
        grid."""
        n_max = self.max_nodes if max_nodes is None else max_nodes
        key = ('dense_index', str(device), n_max)
        out = self._device_cache.get(key)
        if out is None:
            batch = torch.repeat_interleave(
                torch.arange(self.num_graphs), self.counts)
            local = torch.arange(self.num_nodes) - self.ptr[:-1][batch]
            out = _upload(batch * n_max + local, device)
            self._device_cache[key] = out
        return out

    def device_tensor(self, name, device, dtype=torch.int32):
        key = (name, str(device), dtype)
        out = self._device_cache.get(key)
        if out is None:
            src = getattr(self, name)
            out = _upload(src.to(dtype), device)
            self._device_cache[key] = out
        return out


class StaticBatchInfo(object):
    """Batch metadata living in *static device buffers* (hipGraph replay).

    Shapes are fixed by capacities: ``num_nodes`` is the padded row count,
    ``max_nodes`` the fixed per-graph bound; padded rows map to a trash slot
    ``B * max_nodes`` of the dense grid (``has_trash``).  The buffers are
    refreshed in place before every replay.
    """

    has_trash = True

    def __init__(self, num_graphs, max_nodes, num_nodes, counts, ptr,
                 dense_index):
        self.num_graphs = int(num_graphs)
        self.max_nodes = int(max_nodes)
        self.num_nodes = int(num_nodes)
        self._dev = {'counts': counts, 'ptr': ptr}
        self._dense_index = dense_index

    def dense_index(self, device, max_nodes=None):
        assert max_nodes in (None, self.max_nodes)
        return self._dense_index

    def device_tensor(self, name, device, dtype=torch.int32):
        t = self._dev[name]
        assert t.dtype == dtype
        return t


def _drop(key):
    _REGISTRY.pop(key, None)


def register_batch_info(batch, counts):
    """Associate host-side per-graph node ``counts`` with ``batch``."""
    info = counts if isinstance(counts, (BatchInfo, StaticBatchInfo)) \
        else BatchInfo(counts)
    key = id(batch)
    _REGISTRY[key] = (weakref.ref(batch, lambda _, k=key: _drop(k)), info)
    return info


def lookup_batch_info(batch):
    entry = _REGISTRY.get(id(batch))
    if entry is None:
        return None
    ref, info = entry
    if ref() is not batch:
        return None
    return info


def transfer_batch_info(src, dst):
    info = lookup_batch_info(src)
    if info is not None and dst is not None:
        register_batch_info(dst, info)


_SINGLE = {}


def batch_info(batch, num_nodes):
    """Return :class:`BatchInfo` for ``batch`` (``None`` = single graph)."""
    if batch is None:
        # Cached per size so device index maps upload once (graph-safe).
        info = _SINGLE.get(int(num_nodes))
        if info is None:
            info = _SINGLE[int(num_nodes)] = BatchInfo([num_nodes])
        return info
    info = lookup_batch_info(batch)
    if info is not None and info.num_nodes == num_nodes:
        return info
    # Fallback: one device sync (like the reference's to_dense_batch).
    if batch.numel() == 0:
        counts = torch.zeros(0, dtype=torch.long)
    else:
        num_graphs = int(batch[-1].item()) + 1
        counts = torch.zeros(num_graphs, dtype=torch.long,
                             device=batch.device)
        counts.scatter_add_(0, batch, torch.ones_like(batch))
        counts = counts.cpu()
    return register_batch_info(batch, counts)
