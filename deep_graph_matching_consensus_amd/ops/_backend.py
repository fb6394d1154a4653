"""Loader for the in-tree native libraries.

Two shared objects live next to this package (built by ``setup.py
build_ext --inplace`` / :func:`__graft_entry__.build`):

* ``_C_hip``  - gfx950 HIP kernels, registered as ``torch.ops.dgmc_amd.*``
  for the CUDA (=HIP) dispatch key;
* ``_C_host`` - host-side C++ runtime (pair collation index builder, plan
  construction), registered for the CPU dispatch key.

Device tensors are *always* routed to the HIP kernels.  If the HIP library is
missing while a GPU tensor arrives we raise instead of silently degrading to
the pure-PyTorch oracle (set ``DGMC_AMD_ALLOW_FALLBACK=1`` to opt into the
oracle for debugging).  CPU tensors use the oracle in :mod:`.reference`.
"""
import glob
import os
import os.path as osp

import torch

_PKG_DIR = osp.dirname(osp.dirname(osp.abspath(__file__)))
_STATE = {'hip': None, 'host': None}


def _find(name):
    hits = sorted(glob.glob(osp.join(_PKG_DIR, name + '.so')) +
                  glob.glob(osp.join(_PKG_DIR, name + '.*.so')))
    return hits[0] if hits else None


def diag_requested():
    """``DGMC_AMD_DIAG=1``: load the diagnostic HIP library
    (``tools/build_native.py --diag``), whose kernel ablation knobs read the
    environment.  Never for measurements of record."""
    return os.environ.get('DGMC_AMD_DIAG', '0') == '1'


def _load(kind):
    if _STATE[kind] is not None:
        return _STATE[kind]
    name = '_C_' + kind
    if kind == 'hip' and diag_requested():
        name += '_diag'
    path = _find(name)
    ok = False
    if path is not None:
        try:
            torch.ops.load_library(path)
            ok = True
        except OSError as e:  # pragma: no cover - depends on build
            _STATE[kind + '_error'] = str(e)
    _STATE[kind] = ok
    _STATE[kind + '_path'] = path
    return ok


def set_cu_reserve(n):
    """CUs the persistent / CU-sized HIP grids leave free (e.g. for RCCL
    channel kernels running concurrently under data parallelism); returns
    the previous value (default 0; the data-parallel reducer sets it only
    while its all-reduces are in flight, parallel/ddp.py)."""
    _load('hip')
    return int(torch.ops.dgmc_amd.set_cu_reserve(int(n)))


def hip_available():
    return _load('hip')


def host_available():
    return _load('host')


def library_path(kind):
    _load(kind)
    return _STATE.get(kind + '_path')


def allow_fallback():
    return os.environ.get('DGMC_AMD_ALLOW_FALLBACK', '0') == '1'


def use_hip(*tensors):
    """True if the op should run the HIP kernel for these tensors."""
    t = next((t for t in tensors if torch.is_tensor(t)), None)
    if t is None or not t.is_cuda:
        return False
    from ..runtime.mode import is_reference_mode
    if is_reference_mode():
        return False
    if hip_available():
        return True
    if allow_fallback():
        return False
    raise RuntimeError(
        'deep_graph_matching_consensus_amd: GPU tensor received but the HIP '
        'extension (_C_hip*.so) is not built/loadable: {}. Run `python '
        'setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950).'.format(
            _STATE.get('hip_error', library_path('hip'))))


def ops():
    # (Loads the libraries on first use: an op looked up before any
    # use_hip() / hip_available() call still resolves.)
    if _STATE['hip'] is None or _STATE['host'] is None:
        _load('hip')
        _load('host')
    return torch.ops.dgmc_amd
