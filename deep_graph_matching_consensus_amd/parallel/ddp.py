"""Data parallelism over graph-pair batches: flat-bucket gradient all-reduce.

Design for MI355X / RCCL over xGMI (each GPU has 7 point-to-point links):

* every trainable parameter's ``.grad`` is a *view* into one flat fp32
  buffer, partitioned into contiguous buckets (default 8 MiB).  Gradients
  accumulate in place, so a bucket is all-reduced without any packing copy;
* buckets are ordered by (reverse) registration order, which matches the
  order autograd finalises gradients, and each bucket's all-reduce is
  launched asynchronously from a post-accumulate-grad hook the moment its
  last gradient lands - communication overlaps the rest of the backward.
  For DGMC the 25 MiB ``psi_1.convs.0.weight`` gradient is produced last, so
  it forms its own bucket and the smaller ones are already in flight;
* :meth:`finish` waits for outstanding work and averages (``ReduceOp.AVG``
  is used on RCCL, SUM+scale on gloo);
* parameters and buffers are broadcast from rank 0 at construction.

Static / hipGraph steps (``in_step=True``) let AccumulateGrad *steal* each
fresh gradient instead of accumulating into the flat views: the hook of the
parameter that completes a bucket packs that bucket into its flat range (one
multi-tensor kernel) and launches its all-reduce right away, so on RCCL the
whole data-parallel step - backward, bucketed all-reduces overlapping the
rest of the backward, the non-finite check and Adam - is ONE captured
hipGraph (exercised on hardware by ``tests/test_rccl_step.py`` with a
one-rank RCCL group).  Uncaptured static steps use the same in-step
buckets on any backend.  A gloo graph step (the multi-rank rehearsal on one
GPU) cannot capture its collectives: there the step packs all gradients and
the trainer runs one flat all-reduce after the replay.

With a single process every call is a no-op, so the same training loop runs
on 1..8 GPUs.
"""
import weakref

import torch
import torch.distributed as dist
from torch.utils.weak import WeakIdKeyDictionary

from .dist import is_distributed

# Gradient sinks: parameter -> the in-step reducer that owns its flat
# gradient view.  A backward op that produces a large weight gradient in
# pieces (ops/slot_gemm.py: psi_1 layer 0) writes each piece into the view
# and starts its all-reduce at once, so the last - largest - gradient of the
# backward does not leave its whole bucket exposed.
_SINKS = WeakIdKeyDictionary()          # (tensor keys: by identity)


def grad_sink(param):
    """The in-step reducer collecting ``param``'s gradient, or None."""
    r = _SINKS.get(param)
    return r() if r is not None else None


def _pad4(n):
    return (n + 3) // 4 * 4


class GradBucketAllReducer(object):
    r"""Attach to ``module``; call :meth:`finish` after ``backward()``.

    Args:
        module (torch.nn.Module): model whose gradients are synchronised.
        bucket_bytes (int): target bucket size in bytes.
        overlap (bool): launch bucket all-reduces from backward hooks.
        process_group: optional process group.
    """

    def __init__(self, module, bucket_bytes=8 << 20, overlap=True,
                 process_group=None, in_step=False, reserve_cus=0):
        self.module = module
        # CUs the persistent HIP grids leave to RCCL's kernels - only while
        # this step's all-reduces are in flight (from the first launch to
        # finish(); in a captured step the grids of the kernels captured in
        # that window are sized so).  Forward and Adam get every CU.
        self.reserve_cus = int(reserve_cus)
        self._reserve_prev = None
        self.group = process_group
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.distributed = is_distributed()
        self.world = dist.get_world_size(process_group) \
            if self.distributed else 1
        # in_step: stolen gradients, buckets packed + all-reduced from the
        # backward hooks inside the (captured) step.
        self.in_step = bool(in_step) and self.distributed
        self.overlap = (overlap or self.in_step) and self.distributed
        dev = self.params[0].device if self.params else torch.device('cpu')
        # Every gradient view starts on a 16-byte boundary (vectorised
        # optimizer / finiteness kernels); the padding stays zero.
        total = sum(_pad4(p.numel()) for p in self.params)
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)

        # Layout: reverse registration order (≈ backward completion order).
        order = list(reversed(self.params))
        self.buckets, cur, cur_bytes, offset = [], [], 0, 0
        self._slot = {}
        for p in order:
            n = p.numel()
            if cur and cur_bytes + 4 * n > bucket_bytes:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
            self._slot[p] = (offset, n)
            cur.append(p)
            cur_bytes += 4 * n
            offset += _pad4(n)
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {}
        self._bucket_range = []
        for bi, bucket in enumerate(self.buckets):
            lo = self._slot[bucket[0]][0]
            hi = self._slot[bucket[-1]][0] + self._slot[bucket[-1]][1]
            self._bucket_range.append((lo, hi))
            for p in bucket:
                self._bucket_of[p] = bi
        self.attach_grads()
        self._pending = [0] * len(self.buckets)
        self._works = []
        if self.distributed:
            self.broadcast_state()
        if self.overlap:
            self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad)
                           for p in self.params]
        self._pre = set()          # params whose gradient was pre-reduced
        # Optional record of the collectives each step issues: a list with
        # one [(lo, hi), ...] list per step (started by release_grads /
        # zero_grad) - checked across captured size-bucket graphs and ranks
        # (train.py::PairTrainer._check_collective_sequence).
        self.seq_log = None
        if self.in_step:
            me = weakref.ref(self)
            for p in self.params:
                _SINKS[p] = me
        self._reset_counts()

    # ------------------------------------------------------------------
    def attach_grads(self):
        """(Re)bind every ``p.grad`` to its view of the flat buffer."""
        for p in self.params:
            off, n = self._slot[p]
            p.grad = self.flat[off:off + n].view_as(p)

    def zero_grad(self):
        if self.seq_log is not None:
            self.seq_log.append([])
        self.flat.zero_()
        self.attach_grads()

    # ------------------------------------------------------------------
    # Static / captured steps: let AccumulateGrad *steal* the gradients.
    def release_grads(self):
        """Drop every ``p.grad`` before backward: AccumulateGrad then stores
        the freshly computed gradient tensor as ``p.grad`` (no copy) instead
        of adding it into a zeroed view of the flat buffer - which costs a
        zero-fill of the whole buffer plus one add kernel per parameter."""
        if self.seq_log is not None:
            self.seq_log.append([])
        for p in self.params:
            p.grad = None

    def pack_grads(self, with_flags=False):
        """After backward: copy the stolen gradients into the flat buffer in
        ONE multi-tensor kernel (zeros for parameters without a gradient)
        and re-bind every ``p.grad`` to its flat view.  ``with_flags``: also
        return the kernel's per-block non-finite flags (HIP path; None
        otherwise) - the optimizer's step kernel folds them, so no separate
        finiteness pass is needed."""
        from ..ops import _backend
        views = [self.flat[o:o + n].view_as(p)
                 for p, (o, n) in ((p, self._slot[p]) for p in self.params)]
        grads = [p.grad for p in self.params]
        if _backend.use_hip(self.flat):
            fast, slow = [], []
            for g, v in zip(grads, views):
                ok = g is None or (g.dtype == torch.float32 and g.is_cuda and
                                   g.is_contiguous() and
                                   g.data_ptr() % 16 == 0 and
                                   g.numel() == v.numel())
                fast.append(g if ok else None)
                if not ok:
                    slow.append((g, v))
            flags = _backend.ops().pack_grads(fast, views,
                                              with_flags and not slow)
            for g, v in slow:
                v.copy_(g)
            for p, v in zip(self.params, views):
                p.grad = v
            return flags
        else:
            for g, v in zip(grads, views):
                if g is None:
                    v.zero_()
                else:
                    v.copy_(g)
        for p, v in zip(self.params, views):
            p.grad = v
        return None

    def broadcast_state(self):
        with torch.no_grad():
            for t in list(self.module.parameters()) + \
                    list(self.module.buffers()):
                dist.broadcast(t.data, src=0, group=self.group)

    def _reset_counts(self):
        self._pending = [len(b) for b in self.buckets]
        self._works = []
        self._pre = set()

    # ------------------------------------------------------------------
    # Pieces of one parameter's gradient reduced as they are produced.
    def grad_view(self, p):
        """``p``'s view of the flat gradient buffer (write pieces here)."""
        off, n = self._slot[p]
        return self.flat[off:off + n].view_as(p)

    def reduce_piece(self, p, lo, hi):
        """All-reduce elements ``[lo, hi)`` of ``p``'s flat gradient view
        now (asynchronously); call :meth:`mark_reduced` once every piece of
        ``p`` has been launched, before ``p``'s gradient is accumulated."""
        off, n = self._slot[p]
        assert 0 <= lo <= hi <= n
        if hi > lo:
            self._launch_range(off + lo, off + hi)

    def is_pre_reduced(self, p):
        return p in self._pre

    def mark_reduced(self, p):
        """``p``'s whole gradient is in its flat view and being reduced:
        its bucket skips it."""
        self._pre.add(p)

    def _launch(self, bi):
        if not self._pre:
            self._launch_range(*self._bucket_range[bi])
            return
        # Contiguous runs of the bucket's parameters not already reduced.
        run = None
        for p in self.buckets[bi]:
            off, n = self._slot[p]
            if p in self._pre:
                if run is not None:
                    self._launch_range(*run)
                    run = None
                continue
            run = (off, off + n) if run is None else (run[0], off + n)
        if run is not None:
            self._launch_range(*run)

    def _launch_range(self, lo, hi):
        if self.seq_log is not None and self.seq_log:
            self.seq_log[-1].append((int(lo), int(hi)))
        if self.reserve_cus and self._reserve_prev is None and \
                self.flat.is_cuda:
            from ..ops import _backend
            self._reserve_prev = _backend.set_cu_reserve(self.reserve_cus)
        buf = self.flat[lo:hi]
        if dist.get_backend(self.group) == 'nccl':
            work = dist.all_reduce(buf, op=dist.ReduceOp.AVG,
                                   group=self.group, async_op=True)
            self._works.append((work, None))
        else:
            work = dist.all_reduce(buf, op=dist.ReduceOp.SUM,
                                   group=self.group, async_op=True)
            self._works.append((work, buf))

    def _pack_bucket(self, bi):
        """Copy bucket ``bi``'s stolen gradients into its flat range (one
        kernel; zeros for parameters without a gradient) and re-bind their
        ``p.grad`` to the flat views."""
        from ..ops import _backend
        # (pre-reduced parameters already hold their flat view)
        bucket = [p for p in self.buckets[bi] if p not in self._pre]
        if not bucket:
            return
        views = [self.flat[o:o + n].view_as(p)
                 for p, (o, n) in ((p, self._slot[p]) for p in bucket)]
        grads = [p.grad for p in bucket]
        if _backend.use_hip(self.flat) and all(
                g is None or (g.dtype == torch.float32 and g.is_cuda and
                              g.is_contiguous() and g.data_ptr() % 16 == 0)
                for g in grads):
            _backend.ops().pack_grads(grads, views, False)
        else:
            for g, v in zip(grads, views):
                if g is None:
                    v.zero_()
                elif g.data_ptr() != v.data_ptr():
                    v.copy_(g)
        for p, v in zip(bucket, views):
            p.grad = v

    def _on_grad(self, p):
        if p in self._pre:
            # Accumulation may have copied the view: the update must read
            # the (reduced in place) flat view itself.
            p.grad = self.grad_view(p)
        bi = self._bucket_of[p]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            if self.in_step:
                self._pack_bucket(bi)
            self._launch(bi)

    def finish(self):
        """Complete gradient synchronisation (call after ``backward``)."""
        if not self.distributed:
            return
        if not self.overlap:
            # Nothing in flight (e.g. backward replayed from a hipGraph):
            # ONE collective over the whole flat buffer - the fewest RCCL
            # launches and the largest messages for the xGMI rings.
            self._launch_range(0, self.flat.numel())
        else:
            launched = {i for i, c in enumerate(self._pending) if c == 0}
            for bi in range(len(self.buckets)):
                if bi not in launched:
                    if self.in_step:
                        self._pack_bucket(bi)
                    self._launch(bi)
        for work, buf in self._works:
            work.wait()
            if buf is not None:
                buf.div_(self.world)
        if self._reserve_prev is not None:
            from ..ops import _backend
            _backend.set_cu_reserve(self._reserve_prev)
            self._reserve_prev = None
        # Parameters that did not receive a gradient this step keep a
        # consistent (averaged) zero; reset counters for the next step.
        self._reset_counts()


def captured_allreduce_preflight(device, sizes, group=None, reps=2):
    """Capture ONE ``all_reduce(AVG)`` of each size in ``sizes`` (elements)
    into a hipGraph on the real communicator, replay it ``reps`` times and
    compare with the uncaptured result - before the training step, whose
    gradient buckets are captured the same way, is.  Ranks agree on the
    outcome through an uncaptured ``all_reduce(MIN)``; returns ``(ok,
    reason)`` (``ok`` identical on every rank).  RCCL only."""
    ok, reason = True, 'ok'
    try:
        gen = torch.Generator().manual_seed(1234 + dist.get_rank(group))
        for n in sizes:
            x = torch.randn(int(n), generator=gen).to(device)
            ref = x.clone()
            dist.all_reduce(ref, op=dist.ReduceOp.AVG, group=group)
            buf = x.clone()
            torch.cuda.synchronize(device)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, capture_error_mode='thread_local'):
                work = dist.all_reduce(buf, op=dist.ReduceOp.AVG,
                                       group=group, async_op=True)
                work.wait()
            for _ in range(reps):
                buf.copy_(x)
                graph.replay()
                torch.cuda.synchronize(device)
                if not torch.allclose(buf, ref, rtol=1e-5, atol=1e-6):
                    ok, reason = False, 'captured all_reduce of {} elements ' \
                        'differs from the uncaptured one'.format(n)
                    break
            del graph
            if not ok:
                break
    except Exception as e:       # capture refused / RCCL error
        ok, reason = False, '{}: {}'.format(type(e).__name__, e)[:300]
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    agreed = bool(flag.item())
    if ok and not agreed:
        reason = 'failed on another rank'
    return agreed, reason


def sequence_digest(seq):
    """Stable 63-bit digest of a collective sequence ``[(lo, hi), ...]``."""
    import hashlib
    h = hashlib.sha256(repr([tuple(map(int, r)) for r in seq]).encode())
    return int.from_bytes(h.digest()[:8], 'little') & ((1 << 63) - 1)
