"""Forward-scoped memoisation of derived weight tensors.

Inside one DGMC forward the consensus encoder ``psi_2`` runs ``num_steps``
times with identical weights; every SplineConv call would otherwise rebuild
(permute + concat + bf16 cast) its stacked ``[in, 26 * out]`` GEMM operand,
i.e. ~60 extra copy kernels per training step.  ``forward_cache()`` opens a
scope in which such derived tensors are computed once and shared (autograd
accumulates their gradient across uses); the scope closes with the forward,
so parameter updates between steps are always picked up.
"""
import contextlib
import threading

_TLS = threading.local()


@contextlib.contextmanager
def forward_cache():
    outer = getattr(_TLS, 'store', None)
    if outer is not None:      # nested: share the outer scope
        yield outer
        return
    _TLS.store = {}
    try:
        yield _TLS.store
    finally:
        _TLS.store = None


def in_forward_scope():
    return getattr(_TLS, 'store', None) is not None


def cached(key, fn):
    """``fn()`` memoised under ``key`` in the active scope (if any)."""
    import torch
    store = getattr(_TLS, 'store', None)
    if store is None:
        return fn()
    key = key + (torch.is_grad_enabled(), )
    value = store.get(key)
    if value is None:
        value = fn()
        store[key] = value
    return value


def prime(key, value, any_grad_mode=False):
    """Store ``value`` under ``key`` in the active scope (if any), for a
    producer that computes several cached tensors in one kernel.
    ``any_grad_mode``: also serve lookups made with the other grad mode
    (e.g. from inside an autograd ``Function.forward``, where grad mode is
    off) - for values that carry no autograd history."""
    import torch
    store = getattr(_TLS, 'store', None)
    if store is not None:
        modes = (True, False) if any_grad_mode else \
            (torch.is_grad_enabled(), )
        for m in modes:
            store[key + (m, )] = value
