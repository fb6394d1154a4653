"""Per-batch "plans": sparse operators derived from ``edge_index``.

The reference recomputes the B-spline basis and scatters for every one of the
``2 + 2 * num_steps`` encoder invocations per forward
(``/root/reference/dgmc/models/dgmc.py:149-150,174-175``).  Here the plan for
a graph (spline operator, adjacency, two-flow relational operator) is built
once - on the device, with no host synchronisation - and memoised against the
*identity* of the ``edge_index``/``edge_attr`` tensors, so every layer and
every consensus step of a forward (and its backward) reuses it.
"""
import weakref
from collections import OrderedDict

import torch

from . import _backend
from . import reference as ref
from .sparse import SparseOperator

_MAX_ENTRIES = 64


class _IdentityCache(object):
    def __init__(self, max_entries=_MAX_ENTRIES):
        self.max_entries = max_entries
        self.entries = OrderedDict()

    def _key(self, tensors, params):
        ids = tuple((id(t), t._version) if t is not None else None
                    for t in tensors)
        return ids + tuple(params)

    def get(self, tensors, params):
        key = self._key(tensors, params)
        entry = self.entries.get(key)
        if entry is None:
            return None
        refs, value = entry
        for r, t in zip(refs, tensors):
            if (r is None) != (t is None) or (r is not None and r() is not t):
                del self.entries[key]
                return None
        self.entries.move_to_end(key)
        return value

    def put(self, tensors, params, value):
        key = self._key(tensors, params)
        refs = tuple(
            weakref.ref(t, lambda _, k=key: self.entries.pop(k, None))
            if t is not None else None for t in tensors)
        self.entries[key] = (refs, value)
        while len(self.entries) > self.max_entries:
            self.entries.popitem(last=False)
        return value

    def clear(self):
        self.entries.clear()


_CACHE = _IdentityCache()
# Plan providers: objects that can produce the operators of a specific graph
# without the generic device build (e.g. a static batcher assembling them
# from per-graph pieces precomputed once, datasets/static_batch.py).
_PROVIDERS = _IdentityCache()


def clear_plan_cache():
    _CACHE.clear()
    _PROVIDERS.clear()


def register_plan_provider(edge_index, pseudo, provider):
    """Route plan requests for ``(edge_index, pseudo)`` (tensor identity) to
    ``provider.spline_plan(num_nodes, kernel_size, is_open_spline, degree,
    root)``; a provider may return None to fall back to the generic build."""
    _PROVIDERS.put((edge_index, pseudo), ('provider', ), provider)


def _degree(index, num_nodes):
    deg = torch.zeros(num_nodes, dtype=torch.float32, device=index.device)
    deg.index_add_(0, index, torch.ones(index.numel(), dtype=torch.float32,
                                        device=index.device))
    return deg


def compute_spline_basis(pseudo, kernel_size, is_open_spline, degree,
                         device_params=None):
    """``(basis [E,S] fp32, weight_index [E,S] int64)`` on pseudo's device.

    ``device_params`` = ``(kernel_size, is_open_spline)`` tensors already on
    the device (module buffers) - avoids host->device copies, which are not
    allowed while a hipGraph is being captured.
    """
    if pseudo.dim() == 1:
        pseudo = pseudo.view(-1, 1)
    if _backend.use_hip(pseudo) and pseudo.numel() > 0:
        if device_params is not None:
            ks, op = device_params
        else:
            ks = torch.tensor(list(kernel_size), dtype=torch.int32).to(
                pseudo.device)
            op = torch.tensor([int(v) for v in is_open_spline],
                              dtype=torch.int32).to(pseudo.device)
        basis, wi = _backend.ops().spline_basis(
            pseudo.float().contiguous(), ks, op, int(degree))
        return basis, wi
    return ref.spline_basis(pseudo.float(), kernel_size, is_open_spline,
                            degree)


def spline_plan(edge_index, pseudo, num_nodes, kernel_size, is_open_spline,
                degree=1, root=True, device_params=None):
    r"""Operator ``A [N, N * (K + root)]`` so that
    ``SplineConv(x) = A @ (x @ [W_0 | ... | W_{K-1} | root]).view(-1, C)``.
    Entry ``(i, src * (K+1) + wi)`` holds ``basis / deg_in(i)`` (mean
    aggregation, source_to_target flow); the root entry ``(i, i*(K+1)+K)``
    holds 1.
    """
    kernel_size = tuple(int(k) for k in kernel_size)
    is_open_spline = tuple(int(v) for v in is_open_spline)
    params = ('spline', int(num_nodes), kernel_size, is_open_spline,
              int(degree), bool(root))
    plan = _CACHE.get((edge_index, pseudo), params)
    if plan is not None:
        return plan
    provider = _PROVIDERS.get((edge_index, pseudo), ('provider', ))
    if provider is not None:
        plan = provider.spline_plan(int(num_nodes), kernel_size,
                                    is_open_spline, int(degree), bool(root))
        if plan is not None:
            return _CACHE.put((edge_index, pseudo), params, plan)

    device = edge_index.device
    K = 1
    for k in kernel_size:
        K *= k
    slots = K + (1 if root else 0)
    src, dst = edge_index[0], edge_index[1]
    N = int(num_nodes)
    if edge_index.numel() > 0:
        basis, wi = compute_spline_basis(pseudo, kernel_size, is_open_spline,
                                         degree, device_params)
        S = basis.size(1)
        inv_deg = 1.0 / _degree(dst, N).clamp_(min=1)
        row = dst.view(-1, 1).expand(-1, S).reshape(-1)
        col = (src.view(-1, 1) * slots + wi).reshape(-1)
        val = (basis * inv_deg[dst].view(-1, 1)).reshape(-1)
    else:
        row = torch.empty(0, dtype=torch.long, device=device)
        col = row.clone()
        val = torch.empty(0, dtype=torch.float32, device=device)
    if root:
        ar = torch.arange(N, device=device)
        row = torch.cat([row, ar])
        col = torch.cat([col, ar * slots + K])
        val = torch.cat([val, torch.ones(N, device=device)])
    plan = SparseOperator.from_coo(row, col, val, N, N * slots)
    return _CACHE.put((edge_index, pseudo), params, plan)


def adjacency_plan(edge_index, num_nodes, remove_self_loops=True):
    r"""``A [N, N]`` with ``A[i, j] = #edges j->i`` (sum aggregation)."""
    params = ('adj', int(num_nodes), bool(remove_self_loops))
    plan = _CACHE.get((edge_index, ), params)
    if plan is not None:
        return plan
    src, dst = edge_index[0], edge_index[1]
    val = torch.ones(src.numel(), dtype=torch.float32, device=src.device)
    if remove_self_loops:
        # Zero-weight instead of compaction: keeps shapes static (no sync).
        val = val * (src != dst).float()
    plan = SparseOperator.from_coo(dst, src, val, num_nodes, num_nodes)
    return _CACHE.put((edge_index, ), params, plan)


def relational_plan(edge_index, num_nodes):
    r"""``A [N, 3N]`` for RelConv on ``Y = x @ [lin1 | lin2 | root]``:
    ``out_i = Y[i,root] + mean_{j->i} Y[j,lin1] + mean_{i->j} Y[j,lin2]``
    (``/root/reference/dgmc/models/rel.py:26-31``).
    """
    params = ('rel', int(num_nodes))
    plan = _CACHE.get((edge_index, ), params)
    if plan is not None:
        return plan
    N = int(num_nodes)
    device = edge_index.device
    src, dst = edge_index[0], edge_index[1]
    inv_in = 1.0 / _degree(dst, N).clamp_(min=1)
    inv_out = 1.0 / _degree(src, N).clamp_(min=1)
    ar = torch.arange(N, device=device)
    row = torch.cat([dst, src, ar])
    col = torch.cat([src * 3 + 0, dst * 3 + 1, ar * 3 + 2])
    val = torch.cat([inv_in[dst], inv_out[src], torch.ones(N, device=device)])
    plan = SparseOperator.from_coo(row, col, val, N, 3 * N)
    # Knowledge graphs have hub entities (hundreds of neighbours per flow):
    # walk rows in pieces so one hub does not serialise the SpMM.
    plan.balanced = True
    plan.static = True
    return _CACHE.put((edge_index, ), params, plan)
