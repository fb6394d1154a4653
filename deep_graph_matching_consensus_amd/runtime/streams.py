"""Side-stream branches of the training step (opt-in:
``DGMC_AMD_SIDE_STREAMS=1``; see train.py for the measured status).

The weight gradients that the consensus loop folds at its last backward
arrival (psi_2's slot weight gradients and bias sums) are not on the path
to psi_1's backward - nothing downstream of them runs before the optimizer.
Inside :func:`side_streams` (the trainer's static / captured step) such work
runs on a second HIP stream forked from the main one, so it overlaps the
psi_1 backward; :func:`join` (end of backward, before the gradients are
packed) makes the main stream wait for it.  Under hipGraph capture the fork /
join become graph edges (two parallel branches in the replayed step).

Memory: every input the branch reads is kept referenced until the join, so
the caching allocator cannot hand its blocks to main-stream work that could
overwrite them while the branch still reads; outputs are allocated on the
side stream and only consumed after the join (or handed to AccumulateGrad,
which steals them without a kernel - see parallel/ddp.py::release_grads).
"""
import contextlib

import torch

_ACTIVE = [False]
_STREAMS = {}
_KEEP = []
_FORKED = set()


def enabled():
    return _ACTIVE[0]


def _side(device):
    s = _STREAMS.get(device)
    if s is None:
        s = _STREAMS[device] = torch.cuda.Stream(device=device)
    return s


@contextlib.contextmanager
def side_streams(active=True):
    """Scope in which :func:`side` forks work to the side stream; joins on
    exit."""
    prev = _ACTIVE[0]
    _ACTIVE[0] = bool(active)
    try:
        yield
    finally:
        join()
        _ACTIVE[0] = prev


@contextlib.contextmanager
def side(device, keep=()):
    """Run the body on ``device``'s side stream (forked from the current
    stream) when side streams are active; yields whether it did.  ``keep``:
    tensors (or nested lists of tensors) the body reads, held until
    :func:`join`."""
    device = torch.device(device)
    if not _ACTIVE[0] or device.type != 'cuda':
        yield False
        return
    main = torch.cuda.current_stream(device)
    s = _side(device)
    s.wait_stream(main)
    _KEEP.append(keep)
    _FORKED.add(device)
    with torch.cuda.stream(s):
        yield True


def join():
    """Make every forked device's current stream wait for its side stream
    and release the kept inputs."""
    for dev in list(_FORKED):
        torch.cuda.current_stream(dev).wait_stream(_side(dev))
    _FORKED.clear()
    del _KEEP[:]
