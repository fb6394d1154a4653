"""Loop-shared parameter gradients.

The consensus loop (``/root/reference/dgmc/models/dgmc.py:167-179``) applies
``psi_2`` and the consensus MLP ``num_steps`` times with the same weights.
Plain autograd computes one weight gradient per use and sums them with an
``add`` per reuse: for PascalVOC that is ~20 small split-K GEMMs (52 output
tiles each for 256 CUs), ~20 combine kernels and ~100 accumulation adds per
training step.

Inside :func:`loop_scope` every op that owns a reused weight registers a
:class:`LoopGrad` collector (one per op instance and forward) and its backward
deposits *contributions* instead of returning gradients:

* **stacked** - operands ``(x_l, dy_l)`` of ``dW = sum_l x_l^T dy_l`` are
  written into slot ``l`` of ``[uses, ...]`` buffers (``dy`` directly by the
  producing kernel); the last arriving use computes ONE GEMM with a
  ``uses``-times longer reduction dimension (fills the chip, one split-K
  combine);
* **accumulated** - small reductions (bias/vector gradients, small GEMMs)
  are folded into a persistent fp32 buffer by the producing kernel itself
  (``accumulate`` flags of ``col_sum``/``relu_bias_bwd``/``reduce_add_rows``)
  - no separate add kernels;
* **kept** - operands that already exist as separate tensors (a GEMM input
  saved by autograd, an incoming gradient) are only referenced per use and
  concatenated once at the end: one ``cat`` + one GEMM / column sum replace
  a split-K GEMM, combine and reduction per use.

Only the use whose backward completes the set returns the gradients; the
others return ``None``.  This is order-independent (the count, not the order,
decides) and deterministic (fixed fold order per buffer).  Requirement: all
registered uses take part in the same backward pass - true for the consensus
loop, whose every step feeds ``S_L``.
"""
import contextlib
import threading

import torch

_TLS = threading.local()
# Global switch (tests compare against plain per-use autograd).
ENABLED = True


def _rows16(t):
    """2-D tensor whose rows are 16-byte aligned with unit column stride."""
    es = t.element_size()
    return (t.dim() == 2 and t.stride(1) == 1 and
            (t.size(1) * es) % 16 == 0 and (t.stride(0) * es) % 16 == 0 and
            t.data_ptr() % 16 == 0)


class LoopGrad(object):
    """Collects the gradient contributions of one op reused in a loop."""

    def __init__(self):
        self.uses = 0
        self.arrived = 0
        self._stacks = {}
        self._accs = {}
        self._kept = {}

    def register(self):
        """Called by every forward use; returns the use index."""
        idx = self.uses
        self.uses += 1
        return idx

    def slot(self, name, idx, shape, dtype, device):
        """Slot ``idx`` of the ``[uses, *shape]`` stack ``name``."""
        buf = self._stacks.get(name)
        shape = tuple(shape)
        if buf is None:
            buf = torch.empty((self.uses, ) + shape, dtype=dtype,
                              device=device)
            self._stacks[name] = buf
        assert buf.shape[1:] == shape and buf.dtype == dtype, \
            'loop uses must have identical shapes ({} vs {})'.format(
                tuple(buf.shape[1:]), shape)
        return buf[idx]

    def slot_total(self, name, idx, shape, dtype, device, total):
        """Slot ``idx`` of the ``[total, *shape]`` stack ``name`` - for
        producers that write their contribution during the FORWARD, when
        ``uses`` is still growing (the caller knows the final count)."""
        buf = self._stacks.get(name)
        shape = tuple(shape)
        if buf is None:
            buf = torch.empty((total, ) + shape, dtype=dtype, device=device)
            self._stacks[name] = buf
        assert buf.shape[1:] == shape and buf.dtype == dtype and \
            idx < buf.size(0), 'loop stack {} mismatch'.format(name)
        return buf[idx]

    def stack(self, name):
        return self._stacks[name]

    def acc(self, name, shape, device):
        """``(buffer, accumulate)``: fp32 accumulator ``name``; ``accumulate``
        is False for the first contribution (the producer overwrites)."""
        buf = self._accs.get(name)
        if buf is None:
            buf = torch.empty(tuple(shape), dtype=torch.float32,
                              device=device)
            self._accs[name] = buf
            return buf, False
        return buf, True

    def add_to(self, name, value):
        """Accumulate a tensor computed elsewhere (fallback paths)."""
        buf, accumulate = self.acc(name, value.shape, value.device)
        if accumulate:
            buf.add_(value)
        else:
            buf.copy_(value)

    def get_acc(self, name):
        return self._accs.get(name)

    def keep(self, name, idx, tensor):
        """Reference ``tensor`` as use ``idx``'s contribution ``name``."""
        lst = self._kept.get(name)
        if lst is None:
            lst = self._kept[name] = [None] * self.uses
        lst[idx] = tensor

    def kept_list(self, name):
        """The kept contributions of all uses, in use order (for kernels
        that read them in place)."""
        lst = self._kept[name]
        assert all(t is not None for t in lst), name
        return list(lst)

    def kept(self, name):
        """Concatenation (dim 0, use order) of the kept contributions (one
        ``cat_rows`` HIP launch on the GPU: torch.cat splits a 10-way list
        over several slower batched launches)."""
        lst = self._kept[name]
        assert all(t is not None for t in lst), name
        if len(lst) == 1:
            return lst[0]
        from ..ops import _backend
        if len(lst) <= 32 and _backend.use_hip(lst[0]) and \
                all(_rows16(t) for t in lst):
            return _backend.ops().cat_rows(lst)
        return torch.cat(lst, dim=0)

    def arrive(self):
        """Called once per backward use; True for the use completing the set
        (which then computes/returns the gradients and calls
        :meth:`release`)."""
        self.arrived += 1
        return self.arrived == self.uses

    def release(self):
        self._stacks = {}
        self._accs = {}
        self._kept = {}
        self.arrived = 0


@contextlib.contextmanager
def loop_scope(enabled=True):
    """Ops called inside share one :class:`LoopGrad` per op instance."""
    outer = getattr(_TLS, 'groups', None)
    if outer is not None or not (enabled and ENABLED):
        yield
        return
    _TLS.groups = {}
    try:
        yield
    finally:
        _TLS.groups = None


def group(key):
    """The collector for ``key`` in the active loop scope, or None (no scope
    or no autograd recording)."""
    groups = getattr(_TLS, 'groups', None)
    if groups is None or not torch.is_grad_enabled():
        return None
    g = groups.get(key)
    if g is None:
        g = groups[key] = LoopGrad()
    return g
