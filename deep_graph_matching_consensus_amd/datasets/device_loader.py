"""HBM-resident pair loader: the whole graph collection lives on the GPU.

The reference iterates a ``DataLoader(ValidPairDataset(..., sample=True))``
and collates every batch in Python on the host, then copies the 40 MB of
1024-d features of a 512-pair batch over PCIe
(``examples/pascal.py:42,64-66``).
On MI355X the synthetic (or pre-processed) dataset is small next to 288 GB of
HBM, so :class:`DevicePairLoader` keeps node features and edge attributes
resident on the device.  Per step the host:

1. draws source graphs (epoch permutation, like ``shuffle=True``) and one
   random *valid* partner per source (classes(s) subset of classes(t), the
   ``ValidPairDataset`` rule, ``/root/reference/dgmc/utils/data.py:82-101``);
2. builds int64 gather/offset arrays with the native C++ collator
   (``torch.ops.dgmc_host.collate_pairs``; numpy fallback otherwise);
3. ships ~1 MB of indices H2D (pinned, async) and the device gathers features
   with ``index_select``.

The produced batch has the reference's attribute names (``x_s``,
``edge_index_s``, ``edge_attr_s``, ``x_s_batch``, ..., ``y``) and registers
host-side per-graph counts so the forward needs no synchronisation.
"""
import numpy as np
import torch

from ..graph.data import Batch
from ..graph.meta import register_batch_info
from ..ops import _backend


class GraphStore(object):
    r"""Flattened, device-resident collection of graphs with class labels.

    Args:
        groups (list of list of Data): graphs grouped by category; pairs are
            only formed within a group.
        device: target device.
        x_dtype: storage dtype of node features (e.g. ``torch.bfloat16``).
    """

    def __init__(self, groups, device, x_dtype=torch.float32,
                 valid_pairs=True):
        graphs, group_of = [], []
        for gi, group in enumerate(groups):
            for data in group:
                graphs.append(data)
                group_of.append(gi)
        self.num_graphs = len(graphs)
        self.group_of = np.asarray(group_of, dtype=np.int64)
        n = np.asarray([d.num_nodes for d in graphs], dtype=np.int64)
        e = np.asarray([d.num_edges for d in graphs], dtype=np.int64)
        self.node_ptr = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
        self.edge_ptr = np.concatenate([[0], np.cumsum(e)]).astype(np.int64)
        self.device = torch.device(device)

        self.x = torch.cat([d.x for d in graphs]).to(self.device, x_dtype)
        has_attr = graphs[0].edge_attr is not None
        self.edge_attr = torch.cat([d.edge_attr for d in graphs]).to(
            self.device) if has_attr else None
        self.edge_local = torch.cat([d.edge_index for d in graphs],
                                    dim=1).long().contiguous()
        ys = [d.y if d.y is not None else torch.arange(d.num_nodes)
              for d in graphs]
        self.node_class = torch.cat(ys).long().contiguous()
        num_classes = int(self.node_class.max()) + 1
        poc = torch.full((self.num_graphs, num_classes), -1, dtype=torch.long)
        for gi, y in enumerate(ys):
            poc[gi, y] = torch.arange(y.numel())
        self.pos_of_class = poc.contiguous()
        self._node_ptr_t = torch.from_numpy(self.node_ptr)
        self._edge_ptr_t = torch.from_numpy(self.edge_ptr)
        self._build_partner_table(groups, ys, num_classes, valid_pairs)

    def _build_partner_table(self, groups, ys, num_classes, valid_pairs):
        """CSR of valid partners per source graph (within its group)."""
        partners, ptr = [], [0]
        offset = 0
        for group in groups:
            m = len(group)
            inc = torch.zeros((m, num_classes))
            for i in range(m):
                inc[i, ys[offset + i]] = 1
            if valid_pairs:
                ok = (inc @ inc.t()) == inc.sum(1, keepdim=True)
            else:
                ok = torch.ones((m, m), dtype=torch.bool)
            for i in range(m):
                cand = ok[i].nonzero().view(-1) + offset
                partners.append(cand.numpy())
                ptr.append(ptr[-1] + cand.numel())
            offset += m
        self.partner = np.concatenate(partners).astype(np.int64)
        self.partner_ptr = np.asarray(ptr, dtype=np.int64)

    def sample_partners(self, s_ids, rng):
        lo = self.partner_ptr[s_ids]
        cnt = self.partner_ptr[s_ids + 1] - lo
        pick = lo + (rng.random(len(s_ids)) * cnt).astype(np.int64)
        return self.partner[pick]

    # ------------------------------------------------------------------
    def _collate_host(self, s_ids, t_ids):
        s = torch.from_numpy(np.ascontiguousarray(s_ids, dtype=np.int64))
        t = torch.from_numpy(np.ascontiguousarray(t_ids, dtype=np.int64))
        if _backend.host_available():
            return torch.ops.dgmc_host.collate_pairs(
                self._node_ptr_t, self._edge_ptr_t, self.edge_local,
                self.node_class, self.pos_of_class, s, t)
        return _collate_numpy(self, s.numpy(), t.numpy())

    def collate(self, s_ids, t_ids):
        """Build a device :class:`Batch` of pairs ``(s_ids[b], t_ids[b])``."""
        (nis, nit, eis, eit, ei_s, ei_t, b_s, b_t, c_s, c_t,
         y) = self._collate_host(s_ids, t_ids)
        dev = self.device
        pin = dev.type == 'cuda'

        def up(t):
            if pin:
                t = t.pin_memory()
            return t.to(dev, non_blocking=True)

        batch = Batch()
        batch.x_s = self.x.index_select(0, up(nis))
        batch.x_t = self.x.index_select(0, up(nit))
        batch.edge_index_s, batch.edge_index_t = up(ei_s), up(ei_t)
        if self.edge_attr is not None:
            batch.edge_attr_s = self.edge_attr.index_select(0, up(eis))
            batch.edge_attr_t = self.edge_attr.index_select(0, up(eit))
        batch.x_s_batch, batch.x_t_batch = up(b_s), up(b_t)
        batch.y = up(y)
        batch.__num_graphs__ = len(s_ids)
        register_batch_info(batch.x_s_batch, c_s)
        register_batch_info(batch.x_t_batch, c_t)
        return batch


def _collate_numpy(store, s_ids, t_ids):
    """Reference implementation of ``dgmc_host::collate_pairs``."""
    np_, ep_ = store.node_ptr, store.edge_ptr
    c_s, c_t = np_[s_ids + 1] - np_[s_ids], np_[t_ids + 1] - np_[t_ids]
    e_s, e_t = ep_[s_ids + 1] - ep_[s_ids], ep_[t_ids + 1] - ep_[t_ids]

    def ranges(starts, counts):
        idx = np.repeat(starts - np.concatenate([[0], np.cumsum(counts)[:-1]]),
                        counts)
        return idx + np.arange(counts.sum())

    nis, nit = ranges(np_[s_ids], c_s), ranges(np_[t_ids], c_t)
    eis, eit = ranges(ep_[s_ids], e_s), ranges(ep_[t_ids], e_t)
    off_s = np.repeat(np.concatenate([[0], np.cumsum(c_s)[:-1]]), e_s)
    off_t = np.repeat(np.concatenate([[0], np.cumsum(c_t)[:-1]]), e_t)
    el = store.edge_local.numpy()
    ei_s = el[:, eis] + off_s
    ei_t = el[:, eit] + off_t
    b_s = np.repeat(np.arange(len(s_ids)), c_s)
    b_t = np.repeat(np.arange(len(t_ids)), c_t)
    cls = store.node_class.numpy()[nis]
    poc = store.pos_of_class.numpy()
    y = poc[np.repeat(t_ids, c_s), cls]
    out = [nis, nit, eis, eit, ei_s, ei_t, b_s, b_t, c_s, c_t, y]
    return [torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64))
            for a in out]


class DevicePairLoader(object):
    r"""Infinite/epoch iterator of device pair batches from a
    :class:`GraphStore` (``ValidPairDataset(sample=True)`` semantics).

    Args:
        store (GraphStore): resident graphs.
        batch_size (int): pairs per batch.
        shuffle (bool): epoch permutation of the source graphs.
        drop_last (bool): drop the final incomplete batch of an epoch.
        sources (array, optional): restrict sources (e.g. a rank's shard).
        seed (int): host RNG seed.
    """

    def __init__(self, store, batch_size, shuffle=True, drop_last=True,
                 sources=None, seed=0):
        self.store = store
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.sources = np.arange(store.num_graphs) if sources is None \
            else np.asarray(sources, dtype=np.int64)
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        n = len(self.sources)
        return n // self.batch_size if self.drop_last else \
            (n + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        order = self.rng.permutation(self.sources) if self.shuffle \
            else self.sources
        bs = self.batch_size
        for i in range(len(self)):
            s_ids = order[i * bs:(i + 1) * bs]
            t_ids = self.store.sample_partners(s_ids, self.rng)
            yield self.store.collate(s_ids, t_ids)

    def forever(self):
        """Endless full batches: epoch permutations are concatenated, so a
        batch may straddle an epoch boundary and a shard with fewer sources
        than ``batch_size`` (e.g. 2560 graphs over 8 ranks at batch 512)
        still yields ``batch_size`` pairs per step (some sources twice).
        The pending order lives on the loader, so :meth:`state_dict` /
        :meth:`load_state_dict` resume the exact stream."""
        bs = self.batch_size
        if getattr(self, '_order', None) is None:
            self._order = np.empty(0, dtype=np.int64)
        while True:
            while len(self._order) < bs:
                nxt = self.rng.permutation(self.sources) if self.shuffle \
                    else self.sources
                self._order = np.concatenate([self._order, nxt])
            s_ids, self._order = self._order[:bs], self._order[bs:]
            t_ids = self.store.sample_partners(s_ids, self.rng)
            yield self.store.collate(s_ids, t_ids)

    def state_dict(self):
        """Sampler state (``weights_only``-loadable leaves)."""
        order = getattr(self, '_order', None)
        return {'rng': sampler_rng_state(self.rng),
                'order': None if order is None else
                torch.from_numpy(np.asarray(order, dtype=np.int64).copy())}

    def load_state_dict(self, state):
        set_sampler_rng_state(self.rng, state['rng'])
        order = state.get('order')
        self._order = None if order is None else order.cpu().numpy()


def sampler_rng_state(rng):
    """``np.random.Generator`` state as tensors / primitives (PCG64)."""
    st = rng.bit_generator.state
    # 128-bit PCG64 words as bytes (torch.load(weights_only=True) safe).
    return {'bit_generator': st['bit_generator'],
            'state': [int(st['state']['state']).to_bytes(16, 'little'),
                      int(st['state']['inc']).to_bytes(16, 'little')],
            'has_uint32': int(st['has_uint32']),
            'uinteger': int(st['uinteger'])}


def set_sampler_rng_state(rng, state):
    s, inc = state['state']
    rng.bit_generator.state = {
        'bit_generator': state['bit_generator'],
        'state': {'state': int.from_bytes(bytes(s), 'little'),
                  'inc': int.from_bytes(bytes(inc), 'little')},
        'has_uint32': int(state['has_uint32']),
        'uinteger': int(state['uinteger'])}
