"""Execution-mode switches.

``reference_mode()`` runs the framework as a plain eager PyTorch expression
of the reference algorithm - the denominator BASELINE.md asks us to measure
("an eager PyTorch-ROCm expression of the reference algorithm ... on 1x
MI355X"):

* every native op uses its pure-PyTorch oracle (``ops/reference.py``) - no
  HIP kernels, unfactored consensus MLP with the ``[B, N_s, N_t, R]`` tensor
  (``/root/reference/dgmc/models/dgmc.py:178-179``);
* source and target graphs are encoded by separate encoder calls
  (``dgmc.py:149-150,174-175``);
* batch sizes are recovered from the device batch vector and packing uses
  boolean masks, i.e. the reference's host synchronisations
  (``to_dense_batch`` + ``x[mask]``, ``dgmc.py:22-29,154-155``).
"""
import contextlib

_STATE = {'reference': False}


def is_reference_mode():
    return _STATE['reference']


def set_reference_mode(enabled):
    _STATE['reference'] = bool(enabled)


@contextlib.contextmanager
def reference_mode(enabled=True):
    prev = _STATE['reference']
    _STATE['reference'] = bool(enabled)
    try:
        yield
    finally:
        _STATE['reference'] = prev
