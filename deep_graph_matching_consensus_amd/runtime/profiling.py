"""Tracing hooks: roctx ranges + torch.profiler labels.

The reference has no tracing at all.  Here every phase of a training step is
wrapped in :func:`trace_range`:

* ``DGMC_AMD_PROFILE=1`` (or :func:`enable`) turns the ranges on: each one
  is pushed to roctx (``libroctx64.so`` / rocprofiler-sdk, visible in
  ``rocprofv3 --marker-trace`` timelines) and recorded as a
  ``torch.profiler`` ``record_function`` label;
* disabled (default) the context manager is a no-op costing one attribute
  read - safe on the hot path.

Ranges are host-side: inside a captured hipGraph they mark capture, not
replay (profile ``mode='static'`` to see per-phase GPU time).  Kernel-level
timing comes from ``rocprofv3 --kernel-trace --stats`` (``tools/kstats.py``
summarises it per training step; ``tools/gpu_session.sh prof``).
"""
import contextlib
import ctypes
import os

import torch

_ENABLED = os.environ.get('DGMC_AMD_PROFILE', '0') not in ('', '0')
_ROCTX = None
_ROCTX_TRIED = False


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if not _ROCTX_TRIED:
        _ROCTX_TRIED = True
        for name in ('libroctx64.so', 'libroctx64.so.4',
                     'librocprofiler-sdk-roctx.so'):
            for base in ('', '/opt/rocm/lib/'):
                try:
                    lib = ctypes.CDLL(base + name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    _ROCTX = lib
                    return _ROCTX
                except (OSError, AttributeError):
                    continue
    return _ROCTX


def enable(flag=True):
    """Turn tracing ranges on/off at runtime."""
    global _ENABLED
    _ENABLED = bool(flag)


def enabled():
    return _ENABLED


def roctx_available():
    return _roctx() is not None


@contextlib.contextmanager
def _active_range(name):
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


_NULL = contextlib.nullcontext()


def trace_range(name):
    """Context manager marking one phase (no-op unless enabled)."""
    if not _ENABLED:
        return _NULL
    return _active_range(name)


def mark(name):
    """Instantaneous roctx marker (no-op unless enabled)."""
    if _ENABLED:
        lib = _roctx()
        if lib is not None:
            lib.roctxMarkA(name.encode())
