"""Process-group setup for one-process-per-GPU training.

The reference is single-process/single-device (``examples/pascal.py:45``);
the north-star adds data parallelism across the 8 MI355X of a node.  We use
``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm, over xGMI) for
GPU ranks and ``gloo`` for CPU ranks (tests).  Rendezvous uses the standard
``RANK``/``WORLD_SIZE``/``LOCAL_RANK``/``MASTER_ADDR``/``MASTER_PORT``
environment (``torch.distributed.run``).
"""
import datetime
import os

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get('RANK', '0'))


def env_world_size():
    return int(os.environ.get('WORLD_SIZE', '1'))


def env_local_rank():
    return int(os.environ.get('LOCAL_RANK', '0'))


def is_distributed():
    return dist.is_available() and dist.is_initialized()


def rank():
    return dist.get_rank() if is_distributed() else 0


def world_size():
    return dist.get_world_size() if is_distributed() else 1


def init_distributed(backend=None, timeout_s=None):
    """Initialise the default process group from the environment.

    Returns the device this rank should use.  No-op for a single process.

    Failure detection: collectives time out after ``timeout_s`` seconds
    (default ``DGMC_AMD_DIST_TIMEOUT`` or 600) and RCCL's asynchronous error
    handling is enabled, so a crashed or hung rank makes its peers raise
    instead of blocking forever (gloo peers fail at once on a closed
    connection, see tests/test_failures.py).
    """
    if timeout_s is None:
        timeout_s = float(os.environ.get('DGMC_AMD_DIST_TIMEOUT', '600'))
    os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '1')
    use_cuda = torch.cuda.is_available()
    if use_cuda:
        device = torch.device('cuda', env_local_rank() %
                              max(torch.cuda.device_count(), 1))
        torch.cuda.set_device(device)
    else:
        device = torch.device('cpu')
    if env_world_size() > 1 and not is_distributed():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        # DGMC_AMD_DIST_BACKEND=gloo runs GPU ranks over gloo (rehearsing
        # the multi-rank path with several ranks on one device).
        backend = backend or os.environ.get('DGMC_AMD_DIST_BACKEND') or \
            ('nccl' if use_cuda else 'gloo')
        kwargs = dict(backend=backend,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if backend == 'nccl':
            kwargs['device_id'] = device
        dist.init_process_group(**kwargs)
    return device


def barrier():
    if is_distributed():
        if dist.get_backend() == 'nccl':
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(value, device):
    """Max of a Python float over ranks."""
    if not is_distributed():
        return value
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(tensor):
    if is_distributed():
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM)
    return tensor


def all_gather_state(state, device):
    """Every rank's ``state`` (tensors + Python primitives), gathered on
    every rank.  Serialised with ``torch.save`` and decoded with
    ``torch.load(weights_only=True)``, so nothing is unpickled; moved as a
    padded uint8 tensor (device tensor for RCCL)."""
    import io
    if not is_distributed():
        return [state]
    buf = io.BytesIO()
    torch.save(state, buf)
    raw = torch.frombuffer(bytearray(buf.getvalue()), dtype=torch.uint8)
    dev = device if dist.get_backend() == 'nccl' else torch.device('cpu')
    n = torch.tensor([raw.numel()], dtype=torch.long, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    pad = torch.zeros(max(sizes), dtype=torch.uint8, device=dev)
    pad[:raw.numel()] = raw.to(dev)
    outs = [torch.empty_like(pad) for _ in sizes]
    dist.all_gather(outs, pad)
    return [torch.load(io.BytesIO(o[:s].cpu().numpy().tobytes()),
                       map_location='cpu', weights_only=True)
            for o, s in zip(outs, sizes)]


def shutdown():
    if is_distributed():
        dist.destroy_process_group()
