"""hipGraph capture of whole training/inference steps.

The DGMC step is launch-bound in eager mode: ~1,000 kernels per step (ten
consensus iterations, forward and backward), ~9.5 ms of GPU work inside a
~20 ms wall-clock step on MI355X (rocprofv3 trace, profiles/).  Capturing the
step once and replaying it removes the per-kernel host cost (Python
dispatch, autograd bookkeeping, HIP launch) so the GPU runs the kernels back
to back.

Requirements honoured by the library so that a step is capturable:
static shapes (:class:`~..datasets.static_batch.StaticPairBatcher`), no host
synchronisation and no host->device copies inside the step (plans are built
on the device, spline parameters are module buffers, batch metadata lives in
static device buffers), graph-safe RNG (Philox offsets for dropout and the
random indicators), ``torch.autocast(cache_enabled=False)``, and an optimizer
with ``capturable=True``.
"""
import torch


class GraphedStep(object):
    r"""Capture ``fn()`` (a closure over static tensors) into a hipGraph.

    Args:
        fn (callable): the step body; must only touch static tensors.
        warmup (int): eager iterations on a side stream before capture
            (initialises lazy state such as optimizer moments and library
            workspaces).
    """

    def __init__(self, fn, warmup=3):
        self.fn = fn
        self.warmup = warmup
        self.graph = None

    def capture(self):
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            for _ in range(self.warmup):
                self.fn()
        torch.cuda.current_stream().wait_stream(stream)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: with data parallelism the process group's watchdog
        # thread polls collective events while the step is captured; a
        # global-mode capture would be invalidated by those calls.
        mode = 'thread_local' if (torch.distributed.is_available() and
                                  torch.distributed.is_initialized()) \
            else 'global'
        with torch.cuda.graph(self.graph, capture_error_mode=mode):
            self.fn()
        torch.cuda.synchronize()
        return self

    def __call__(self):
        if self.graph is None:
            self.capture()
        self.graph.replay()


def graph_capture_supported(device):
    return torch.device(device).type == 'cuda' and torch.cuda.is_available()
