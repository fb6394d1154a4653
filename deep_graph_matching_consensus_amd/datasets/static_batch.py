"""Static-shape pair batches for hipGraph-captured training steps.

A captured graph replays fixed kernels on fixed addresses, but every pair
batch has a different number of nodes/edges.  :class:`StaticPairBatcher`
pads each batch to capacities estimated once from the dataset (node/edge
totals per side, plus the per-graph bound ``n_max``) and keeps ALL per-step
inputs in one static int64 device buffer:

* host: the native collator (``dgmc_host::collate_pairs_padded``) writes the
  padded index arrays into a pinned staging buffer (double-buffered, guarded
  by events so the host never overwrites a buffer an H2D copy still reads);
* one ``non_blocking`` H2D copy refreshes the device buffer;
* :meth:`materialize` (captured inside the graph) gathers node features and
  edge attributes from the HBM-resident :class:`GraphStore` and exposes the
  batch with the reference attribute names plus ``y_mask``.

Padding is inert: padded nodes have zero features, belong to no pair (the
per-pair kernels address rows through ``ptr``), are routed to a trash slot of
the dense grid, carry only self-loop padded edges, and are masked out of the
loss/metrics.  Batches that exceed a capacity (vanishingly rare with the 6
sigma headroom) are reported so the caller can run that step eagerly.
"""

import numpy as np
import torch

from ..graph.data import Batch
from ..graph.meta import StaticBatchInfo, register_batch_info
from ..ops import _backend
from ..ops import plans as _plans
from ..ops.sparse import SparseOperator


# Largest graph (nodes) for which batches use the fused slot conv's tiling
# (tile window 65 - n_max >= 17 rows).
SLOT_TILE_MAX_GRAPH = 48


def _round_up(x, m):
    return int((int(x) + m - 1) // m * m)


class StaticPairBatcher(object):
    r"""Fixed-capacity pair batches drawn from a :class:`GraphStore`.

    Args:
        store (GraphStore): HBM-resident graphs.
        batch_size (int): pairs per step.
        sources (array, optional): source graph ids (e.g. a rank shard).
        seed (int): host RNG seed.
        probe_batches (int): batches sampled to size the capacities.
        headroom (float): multiplicative slack on the probed maxima.
    """

    def __init__(self, store, batch_size, sources=None, seed=0,
                 probe_batches=256, headroom=1.04, n_max=None, caps=None):
        if not _backend.host_available():
            raise RuntimeError('StaticPairBatcher needs the native host '
                               'library (_C_host.so); build it first')
        self.store = store
        self.B = int(batch_size)
        self.rng = np.random.default_rng(seed)
        self.sources = np.arange(store.num_graphs) if sources is None \
            else np.asarray(sources, dtype=np.int64)
        counts = store.node_ptr[1:] - store.node_ptr[:-1]
        self.n_max = int(counts.max()) if n_max is None else int(n_max)
        if caps is None:
            self._size_capacities(probe_batches, headroom)
        else:
            self.cap_s, self.cap_t, self.ecap_s, self.ecap_t = \
                (int(c) for c in caps)
        self.device = store.device

        # Zero feature row / zero edge-attr row appended once for padding.
        self.zero_node = int(store.node_ptr[-1])
        self.zero_edge = int(store.edge_ptr[-1])
        self.x = torch.cat([store.x, store.x.new_zeros(1, store.x.size(1))])
        self.edge_attr = None if store.edge_attr is None else torch.cat(
            [store.edge_attr,
             store.edge_attr.new_zeros(1, store.edge_attr.size(1))])

        # Host copy of the fp32 edge-attribute table: the collator writes the
        # batch's attributes into the staged buffer (no device gather).
        self._ea_host = None
        if self.edge_attr is not None and \
                self.edge_attr.dtype == torch.float32:
            self._ea_host = self.edge_attr.cpu().contiguous()
        self.ea_dim = 0 if self._ea_host is None else self._ea_host.size(1)
        cs, ct, es, et, B = self.cap_s, self.cap_t, self.ecap_s, self.ecap_t, \
            self.B
        self.words = cs * 4 + ct * 2 + es * 3 + et * 3 + 2 * (B + 1) + \
            2 * B + 2 * et + (cs + 7) // 8 + (B + 1) + B + \
            ((es + et) * self.ea_dim + 1) // 2
        pin = self.device.type == 'cuda'
        self._host = [torch.zeros(self.words, dtype=torch.long,
                                  pin_memory=pin) for _ in range(2)]
        self._events = [None, None]
        self._slot = 0
        self.buf = torch.zeros(self.words, dtype=torch.long,
                               device=self.device)
        self._views()
        self.batch_s = torch.zeros(cs, dtype=torch.long, device=self.device)
        self.batch_t = torch.zeros(ct, dtype=torch.long, device=self.device)
        self._order = None
        self._pos = 0
        self.overflows = 0
        self._assembler = SlotPlanAssembler(self)

    # ------------------------------------------------------------------
    def _size_capacities(self, probes, headroom):
        st = self.store
        n = st.node_ptr[1:] - st.node_ptr[:-1]
        e = st.edge_ptr[1:] - st.edge_ptr[:-1]
        rng = np.random.default_rng(12345)
        mx = np.zeros(4)
        for _ in range(probes):
            s = rng.choice(self.sources, size=self.B,
                           replace=len(self.sources) < self.B)
            t = st.sample_partners(s, rng)
            mx = np.maximum(mx, [n[s].sum(), n[t].sum(), e[s].sum(),
                                 e[t].sum()])
        self.cap_s = _round_up(mx[0] * headroom + 1, 64)
        self.cap_t = _round_up(mx[1] * headroom + 1, 64)
        self.ecap_s = _round_up(mx[2] * headroom, 256)
        self.ecap_t = _round_up(mx[3] * headroom, 256)

    @property
    def caps(self):
        return (self.cap_s, self.cap_t, self.ecap_s, self.ecap_t)

    def fits(self, s_ids, t_ids):
        """Whether the pair batch ``(s_ids, t_ids)`` fits the capacities
        (host-side sizes; the collator applies the same bounds)."""
        st = self.store
        n = st.node_ptr[1:] - st.node_ptr[:-1]
        e = st.edge_ptr[1:] - st.edge_ptr[:-1]
        return (n[s_ids].sum() < self.cap_s and n[t_ids].sum() < self.cap_t
                and e[s_ids].sum() <= self.ecap_s and
                e[t_ids].sum() <= self.ecap_t)

    def _views(self):
        cs, ct, es, et, B = self.cap_s, self.cap_t, self.ecap_s, self.ecap_t, \
            self.B
        # Layout written by dgmc_host::collate_pairs_padded: source/target
        # regions are adjacent, so the disjoint union [s; t] of nodes, edge
        # attributes and edges (target endpoints stored offset by cap_s) is a
        # view - no concatenation kernels in the step.
        o = 0
        v = {}
        for name, n in [('node', cs + ct), ('ea', es + et),
                        ('ei', 2 * (es + et)), ('y', cs), ('ymask', cs),
                        ('dense_s', cs), ('dense_t', ct), ('ptr_s', B + 1),
                        ('ptr_t', B + 1), ('gid', 2 * B),
                        # typed tail (final dtypes, no device casts)
                        ('ei_tl', 2 * et), ('ymask_b', (cs + 7) // 8),
                        ('ptr32', B + 1), ('cnt32', B),
                        ('ea_val', ((es + et) * self.ea_dim + 1) // 2)]:
            v[name] = self.buf[o:o + n]
            o += n
        v['ei'] = v['ei'].view(2, es + et)
        v['ei_tl'] = v['ei_tl'].view(2, et)
        v['ymask_b'] = v['ymask_b'].view(torch.uint8)[:cs].view(torch.bool)
        p32 = v['ptr32'].view(torch.int32)
        v['ptr32_s'], v['ptr32_t'] = p32[:B + 1], p32[B + 1:]
        c32 = v['cnt32'].view(torch.int32)
        v['cnt32_s'], v['cnt32_t'] = c32[:B], c32[B:]
        if self.ea_dim:
            v['ea_val'] = v['ea_val'].view(torch.float32)[
                :(es + et) * self.ea_dim].view(es + et, self.ea_dim)
        self.v = v

    # ------------------------------------------------------------------
    def next_ids(self):
        """Next ``B`` sources (concatenated epoch permutations: a batch may
        straddle an epoch boundary, and a rank shard smaller than ``B`` -
        2560 graphs over 8 ranks at batch 512 - repeats sources) and random
        valid partners."""
        while self._order is None or self._pos + self.B > len(self._order):
            rest = self._order[self._pos:] if self._order is not None \
                else self.sources[:0]
            self._order = np.concatenate(
                [rest, self.rng.permutation(self.sources)])
            self._pos = 0
        s = self._order[self._pos:self._pos + self.B]
        self._pos += self.B
        return s, self.store.sample_partners(s, self.rng)

    def state_dict(self):
        """Sampler state: RNG, pending epoch order and position."""
        from .device_loader import sampler_rng_state
        return {'rng': sampler_rng_state(self.rng),
                'order': None if self._order is None else
                torch.from_numpy(np.asarray(self._order,
                                            dtype=np.int64).copy()),
                'pos': int(self._pos), 'overflows': int(self.overflows)}

    def load_state_dict(self, state):
        from .device_loader import set_sampler_rng_state
        set_sampler_rng_state(self.rng, state['rng'])
        order = state.get('order')
        self._order = None if order is None else order.cpu().numpy()
        self._pos = int(state.get('pos', 0))
        self.overflows = int(state.get('overflows', 0))

    def load(self, s_ids=None, t_ids=None):
        """Stage the next batch into the static device buffer.

        Returns False (buffer unchanged) if the batch exceeds a capacity.
        """
        if s_ids is None:
            s_ids, t_ids = self.next_ids()
        if len(s_ids) != self.B or len(t_ids) != self.B:
            # The static buffer layout is sized for exactly B pairs.
            raise ValueError('static batch of {} pairs needs exactly {} '
                             'source / target ids, got {} / {}'.format(
                                 self.B, self.B, len(s_ids), len(t_ids)))
        slot = self._slot
        self._slot ^= 1
        # The host stages at most one batch ahead of the device: wait for
        # the previous batch's copy (i.e. the step before it) before
        # collating this one (measured faster than two ahead, which lets
        # the host queue deeper: 179.5k vs 178.7k pairs/s same-box).
        wait = self._events[slot ^ 1]
        if wait is not None:
            wait.synchronize()
        host = self._host[slot]
        st = self.store
        ok = torch.ops.dgmc_host.collate_pairs_padded(
            st._node_ptr_t, st._edge_ptr_t, st.edge_local, st.node_class,
            st.pos_of_class,
            torch.from_numpy(np.ascontiguousarray(s_ids, dtype=np.int64)),
            torch.from_numpy(np.ascontiguousarray(t_ids, dtype=np.int64)),
            host, self.cap_s, self.cap_t, self.ecap_s, self.ecap_t,
            self.n_max, self.zero_node, self.zero_edge, self._ea_host)
        if not ok:
            self.overflows += 1
            return False
        self.buf.copy_(host, non_blocking=True)
        if self.device.type == 'cuda':
            ev = torch.cuda.Event()
            ev.record()
            self._events[slot] = ev    # guards the pinned host slot
        return True

    def materialize(self):
        """Device-side batch from the static buffer (graph-capturable)."""
        from ..models.dgmc import register_pair_graph
        v = self.v
        # Every materialisation is a new batch for the identity caches keyed
        # on (tensor, version) (ops/plans.py): the buffer views are the same
        # objects each step, so bump their shared version counter (no
        # kernel).  Otherwise a hipGraph capture following an eager warm-up
        # on the same staged batch would reuse the warm-up's plans instead of
        # recording their assembly.
        torch.autograd.graph.increment_version(self.buf)
        cs, es = self.cap_s, self.ecap_s
        batch = Batch()
        x_u = self.x.index_select(0, v['node'])
        batch.x_s, batch.x_t = x_u[:cs], x_u[cs:]
        ei_u = v['ei']
        batch.edge_index_s = ei_u[:, :es]
        batch.edge_index_t = v['ei_tl']           # local target ids
        ea_u = None
        if self.ea_dim:
            ea_u = v['ea_val']                    # written by the collator
        elif self.edge_attr is not None:
            ea_u = self.edge_attr.index_select(0, v['ea'])
        if ea_u is not None:
            batch.edge_attr_s, batch.edge_attr_t = ea_u[:es], ea_u[es:]
        else:
            batch.edge_attr_s = batch.edge_attr_t = None
        # DGMC encodes source and target as one disjoint union: hand it the
        # union graph directly, and route its sparse-operator requests to the
        # per-graph plan assembler (no per-step plan construction).
        register_pair_graph(batch.edge_index_s, batch.edge_attr_s,
                            batch.edge_index_t, batch.edge_attr_t, cs, ei_u,
                            ea_u)
        _plans.register_plan_provider(ei_u, ea_u, self._assembler)
        batch.y = v['y']
        batch.y_mask = v['ymask_b']
        info_s = StaticBatchInfo(self.B, self.n_max, self.cap_s,
                                 v['cnt32_s'], v['ptr32_s'], v['dense_s'])
        info_t = StaticBatchInfo(self.B, self.n_max, self.cap_t,
                                 v['cnt32_t'], v['ptr32_t'], v['dense_t'])
        batch.x_s_batch, batch.x_t_batch = self.batch_s, self.batch_t
        register_batch_info(self.batch_s, info_s)
        register_batch_info(self.batch_t, info_t)
        batch.__num_graphs__ = self.B
        return batch

    def __repr__(self):
        return ('{}(B={}, n_max={}, cap_s={}, cap_t={}, ecap_s={}, '
                'ecap_t={})').format(type(self).__name__, self.B, self.n_max,
                                     self.cap_s, self.cap_t, self.ecap_s,
                                     self.ecap_t)


def bucket_capacities(store, batch_size, sources=None, z=(-0.5, 0.5, 1.5),
                      probe_batches=512, seed=12345):
    r"""Capacity tuples ``(cap_s, cap_t, ecap_s, ecap_t)`` of smaller
    static-batch size buckets at ``mean + z * std`` of every size (probed on
    random pair batches), ascending.

    One fixed capacity must cover the largest batch, so a single bucket pads
    the average PascalVOC-shaped batch by ~8 % (11008 rows for 10171 real);
    with buckets at z = -0.5, 0.5, 1.5 plus the max-sized one the average
    capacity drops to ~10330 rows - every node-proportional kernel of the
    step (encoder GEMMs, SpMMs, dY stacks) shrinks by ~6 %.
    """
    n = store.node_ptr[1:] - store.node_ptr[:-1]
    e = store.edge_ptr[1:] - store.edge_ptr[:-1]
    src = np.arange(store.num_graphs) if sources is None \
        else np.asarray(sources, dtype=np.int64)
    rng = np.random.default_rng(seed)
    sizes = []
    for _ in range(probe_batches):
        s = rng.choice(src, size=batch_size, replace=len(src) < batch_size)
        t = store.sample_partners(s, rng)
        sizes.append((n[s].sum(), n[t].sum(), e[s].sum(), e[t].sum()))
    sizes = np.asarray(sizes, dtype=np.float64)
    mu, sd = sizes.mean(0), sizes.std(0)
    out = []
    for zz in sorted(z):
        c = mu + zz * sd
        caps = (_round_up(c[0] + 1, 64), _round_up(c[1] + 1, 64),
                _round_up(c[2], 256), _round_up(c[3], 256))
        if not out or caps != out[-1]:
            out.append(caps)
    return out


class _StaticSlotOperator(SparseOperator):
    """Fixed-capacity operator filled by ``assemble_slot_plan``: entries past
    ``rowptr[-1]`` are inert (col 0, val 0)."""

    @property
    def row(self):
        if self._row is None:
            pos = torch.arange(self.nnz, device=self.device, dtype=torch.int32)
            r = torch.searchsorted(self.rowptr[1:], pos, right=True)
            self._row = r.clamp_(max=max(self.num_rows - 1, 0)).long()
        return self._row


class SlotPlanAssembler(object):
    r"""Spline operators (``A`` and ``A^T``) of a static batch's union graph,
    assembled per step by ONE kernel (``csrc/hip/plan_assembly.hip``) from
    the store-level operator built once per conv configuration - instead of
    basis + degree + two stable sorts + scans every step.

    Valid rows are identical to :func:`~..ops.plans.spline_plan` on the batch
    (same per-graph entries, same order); padding rows carry only their root
    entry.  Returns None (generic build) off-GPU or during a first capture.
    """

    def __init__(self, batcher):
        self.b = batcher
        self._store = {}
        self._out = {}
        self._store_ei = None
        self._node_ptr = None

    def _store_graph(self):
        st = self.b.store
        if self._store_ei is None:
            e = st.edge_ptr[1:] - st.edge_ptr[:-1]
            off = torch.from_numpy(np.repeat(st.node_ptr[:-1], e))
            self._store_ei = (st.edge_local + off.view(1, -1)).to(st.device)
            self._node_ptr = torch.from_numpy(st.node_ptr).to(st.device)
        return self._store_ei

    def spline_plan(self, num_nodes, kernel_size, is_open_spline, degree,
                    root):
        b = self.b
        st = b.store
        if (b.device.type != 'cuda' or st.edge_attr is None or
                not _backend.hip_available() or
                num_nodes != b.cap_s + b.cap_t):
            return None
        key = (tuple(kernel_size), tuple(is_open_spline), degree, root)
        pieces = self._store.get(key)
        if pieces is None:
            if torch.cuda.is_current_stream_capturing():
                return None            # built eagerly (warm-up steps) first
            A = _plans.spline_plan(self._store_graph(), st.edge_attr,
                                   int(st.node_ptr[-1]), kernel_size,
                                   is_open_spline, degree, root)
            # The fused slot conv scatters entries into dense tiles without
            # accumulation: it needs every (row, column) entry to be unique.
            rc = A.row * A.num_cols + A.col.long()
            unique = int(torch.unique(rc).numel()) == A.nnz
            pieces = self._store[key] = (A, A.t(), unique,
                                         A.row.long().contiguous())
        A, At, unique, st_row = pieces
        K = 1
        for k in kernel_size:
            K *= int(k)
        S = K + (1 if root else 0)
        N = b.cap_s + b.cap_t
        out = self._out.get(key)
        if out is None:
            per_edge = (degree + 1) ** len(kernel_size)
            cap = per_edge * (b.ecap_s + b.ecap_t) + (N if root else 0)
            dev = b.device
            i32 = dict(dtype=torch.int32, device=dev)
            f32 = dict(dtype=torch.float32, device=dev)
            out = self._out[key] = (
                torch.zeros(N + 1, **i32), torch.zeros(cap, **i32),
                torch.zeros(cap, **f32), torch.zeros(N * S + 1, **i32),
                torch.zeros(cap, **i32), torch.zeros(cap, **f32),
                torch.zeros(N, dtype=torch.uint8, device=dev),
                torch.zeros(cap, dtype=torch.long, device=dev))
        rowptr, col, val, trowptr, tcol, tval, gflag, row = out
        v = b.v
        _backend.ops().assemble_slot_plan(
            A.rowptr, A.col, A.val, At.rowptr, At.col, At.val,
            self._node_ptr, v['gid'], v['ptr_s'], v['ptr_t'], b.cap_s,
            b.cap_t, S, K if root else -1, rowptr, col, val, trowptr, tcol,
            tval, gflag, st_row, row)
        op = _StaticSlotOperator(rowptr, col, val, N, N * S)
        # Entry rows written by the same kernel (tail entries past the
        # total are stale, like col/val there: consumers stop at rowptr[N]).
        op._row = row
        op._t = _StaticSlotOperator(trowptr, tcol, tval, N * S, N)
        op._t._t = op
        # Graph-closed row tiles for the fused slot conv: windows of
        # 65 - n_max rows never cut a graph into a tile of more than 64 rows.
        if unique and b.n_max <= SLOT_TILE_MAX_GRAPH:
            op.tile_flag = gflag
            op.tile_window = 65 - b.n_max
        return op
