"""Training/evaluation driver shared by ``bench.py`` and ``examples/``.

The reference drivers (``/root/reference/examples/pascal.py:60-99``,
``willow.py:60-140``) loop over a host DataLoader, call ``.item()`` twice per
step and keep the model in a single process.  :class:`PairTrainer` runs the
same objective (``NLL(S_0) + NLL(S_L)``, ``pascal.py:70-72``) in one of three
execution modes:

* ``'eager'``  - dynamic batches from :class:`DevicePairLoader`, gradient
  all-reduce overlapped with backward;
* ``'static'`` - fixed-capacity padded batches (:class:`StaticPairBatcher`),
  eager execution (useful on CPU and for debugging the graph path);
* ``'graph'``  - static batches + the whole step (gather, forward, backward,
  optimizer) captured once into a hipGraph and replayed.

Metrics are accumulated on the device and synchronised only when read.
Checkpoints store the model in the reference state-dict schema plus
optimizer state, step counter and RNG states (resume support).
"""
import gc
import json
import os
import random
import time
import warnings

import numpy as np
import torch

from . import parallel
from .datasets.device_loader import DevicePairLoader
from .datasets.static_batch import StaticPairBatcher, bucket_capacities
from .runtime.graphs import GraphedStep
from .runtime.profiling import trace_range
from .runtime.tuning import tuned_gemms, use_tuned_gemms

# Data-parallel gradient all-reduce inside the (captured) step, overlapped
# with the backward (DGMC_AMD_IN_STEP_ALLREDUCE=0: one flat all-reduce after
# the step).
IN_STEP_ALLREDUCE = os.environ.get('DGMC_AMD_IN_STEP_ALLREDUCE', '1') == '1'
# CUs the persistent GEMM grids leave to RCCL's channel kernels under data
# parallelism, applied only while the step's all-reduces are in flight
# (parallel/ddp.py; DGMC_AMD_RESERVE_CUS overrides; single-GPU runs reserve
# none).  tools/bench_cu_reserve.py (profiles/cu_reserve_r6.json, psi_1's
# 1024 -> 256 bf16x6 forward / input gradient, persistent grids): a
# concurrent kernel holding h CUs stretches them 400 -> 611-623 / 419 ->
# 602-635 us whenever the reserve r < h, and costs nothing beyond the lost
# CUs once r >= h (dX 440 / 455 us at r = 8 / 32); the weight gradient's
# item grid is insensitive (469-540 us either way).  8 covers an RCCL
# all-reduce on up to 8 channel workgroups at ~5 % on the backward's
# persistent kernels; DGMC_AMD_RESERVE_CUS raises it where RCCL runs more
# channels (untested on multi-GPU hardware by us).
DP_RESERVE_CUS = 8
# Captured all-reduce pre-flight before the first step capture
# (DGMC_AMD_DP_PREFLIGHT=0 skips it).
PREFLIGHT = os.environ.get('DGMC_AMD_DP_PREFLIGHT', '1') == '1'


class PairTrainer(object):
    r"""DGMC trainer over an HBM-resident :class:`GraphStore`.

    Args:
        model (DGMC): the matching model (already on ``device``).
        store (GraphStore): training graphs.
        batch_size (int): pairs per step and rank.
        lr (float): Adam learning rate.
        mode (str): ``'eager'``, ``'static'`` or ``'graph'``.
        bf16 (bool): bf16 autocast for the encoder GEMMs (opt-in; the
            default is fp32, the reference's training precision).
        seed (int): data-order seed (offset by rank).
        overlap (bool): overlap gradient all-reduce with backward (eager).
        bucket_bytes (int): data-parallel all-reduce bucket size.
        guard_nonfinite (bool): skip the optimizer update of any step whose
            (all-reduced) gradients contain NaN/Inf - on the device, inside
            the captured graph, via the fused Adam ``found_inf`` input; the
            skipped-step count is reported by :meth:`read_stats`.
        dp_mode (str): ``'captured'`` (default; ``DGMC_AMD_IN_STEP_ALLREDUCE``
            =1): bucketed all-reduces launched from the backward hooks inside
            the step - captured in its hipGraph on RCCL; ``'flat'``: one flat
            all-reduce of the whole gradient buffer after the step (replay).
    """

    def __init__(self, model, store, batch_size, lr=1e-3, mode='graph',
                 bf16=False, seed=0, overlap=True, sources=None,
                 guard_nonfinite=True, buckets=True, bucket_bytes=8 << 20,
                 dp_mode=None):
        self.model = model
        self.store = store
        self.device = store.device
        self.rank, self.world = parallel.rank(), parallel.world_size()
        if mode == 'graph' and self.device.type != 'cuda':
            mode = 'static'
        self.mode = mode
        self.bf16 = bf16 and self.device.type == 'cuda'
        if sources is None:
            sources = np.arange(store.num_graphs)[self.rank::self.world]
        # Data parallel: bucketed all-reduces launched from the backward
        # hooks INSIDE the step body.
        # * static mode: always (any backend - nothing is captured);
        # * graph mode: only on RCCL, whose collectives are captured into the
        #   step's hipGraph; gloo cannot be captured, so a gloo graph step
        #   packs every gradient and one flat all-reduce runs after the
        #   replay (parallel/ddp.py).
        graph_rccl = (mode == 'graph' and parallel.is_distributed() and
                      torch.distributed.get_backend() == 'nccl')
        if dp_mode is None:
            dp_mode = 'captured' if IN_STEP_ALLREDUCE else 'flat'
        assert dp_mode in ('captured', 'flat'), dp_mode
        in_step = dp_mode == 'captured' and (mode == 'static' or graph_rccl)
        # First-run insurance for captured collectives: one bucket-sized and
        # one piece-sized all-reduce captured + replayed on the real
        # communicator before anything else is; every rank falls back to
        # the flat after-replay all-reduce together if any rank fails.
        self.dp_checks = {}
        if in_step and graph_rccl and PREFLIGHT:
            from .ops.slot_gemm import PIECES
            piece = max(p.numel() for p in model.parameters()) // \
                max(PIECES, 1)
            ok, why = parallel.captured_allreduce_preflight(
                self.device, [bucket_bytes // 4, piece])
            self.dp_checks['preflight'] = why
            if not ok:
                warnings.warn('captured all-reduce pre-flight failed ({}): '
                              'using one flat all-reduce after each '
                              'replay'.format(why))
                in_step = False
        cuda = self.device.type == 'cuda'
        self.reserved_cus = 0
        if self.world > 1:
            # (recorded on any device; only HIP grids are resized)
            env = os.environ.get('DGMC_AMD_RESERVE_CUS')
            self.reserved_cus = int(env) if env else DP_RESERVE_CUS
        self.reducer = parallel.GradBucketAllReducer(
            model, bucket_bytes=bucket_bytes,
            overlap=overlap and mode == 'eager', in_step=in_step,
            reserve_cus=self.reserved_cus)
        if cuda:
            use_tuned_gemms()     # measured GEMM solutions (runtime/tuning.py)
        self.optimizer = torch.optim.Adam(model.parameters(), lr=lr,
                                          fused=cuda,
                                          capturable=mode == 'graph')
        # loss sum, correct, ground truths, skipped (non-finite) steps
        self.stats = torch.zeros(4, dtype=torch.float64, device=self.device)
        self.guard = guard_nonfinite
        # 0-dim: fused Adam subtracts it from the (0-dim) step counters.
        self._found_inf = torch.zeros((), dtype=torch.float32,
                                      device=self.device)
        if self.guard and cuda:
            # Read by the fused Adam kernel: a nonzero value skips the update
            # (and the step counter) on the device - no host sync, capturable.
            self.optimizer.found_inf = self._found_inf
        self.step_count = 0
        self._one = None
        # Optional CUDA-event timing of the exposed (after-step) all-reduce
        # (bench diagnostics): (start, end) event pairs of the timed steps.
        self.time_allreduce = False
        self.allreduce_events = []
        data_seed = seed + 1000 * self.rank
        if mode == 'eager':
            self.loader = DevicePairLoader(store, batch_size, sources=sources,
                                           seed=data_seed)
            self._batches = self.loader.forever()
        else:
            # The largest bucket covers every batch (and owns the sampler);
            # in graph mode smaller size buckets, each with its own static
            # buffers and captured graph, cut the padding (see
            # datasets/static_batch.py::bucket_capacities).
            self.batcher = StaticPairBatcher(store, batch_size,
                                             sources=sources, seed=data_seed)
            if self.world > 1:
                # Every rank must capture the same graphs in the same order
                # (their in-step collectives pair up across ranks): agree on
                # the largest capacities (max over the rank shards) and size
                # the smaller buckets from the whole store, not the shard.
                agreed = tuple(int(parallel.all_reduce_max(c, self.device))
                               for c in self.batcher.caps)
                if agreed != self.batcher.caps:
                    self.batcher = StaticPairBatcher(
                        store, batch_size, sources=sources, seed=data_seed,
                        caps=agreed)
            self.batchers = [self.batcher]
            if mode == 'graph' and buckets:
                probe = sources if self.world == 1 else None
                caps = [c for c in bucket_capacities(store, batch_size, probe)
                        if all(a < b for a, b in zip(c, self.batcher.caps))]
                self.batchers = [
                    StaticPairBatcher(store, batch_size, sources=sources,
                                      seed=data_seed, caps=c)
                    for c in caps] + [self.batcher]
            self._rows = [torch.arange(b.cap_s, device=self.device)
                          for b in self.batchers]
            self._graphs = [GraphedStep(self._bucket_body(i), warmup=2)
                            for i in range(len(self.batchers))] \
                if mode == 'graph' else None
            self._captured = False

    # ------------------------------------------------------------------
    def _autocast(self):
        return torch.autocast(device_type=self.device.type,
                              dtype=torch.bfloat16, enabled=self.bf16,
                              cache_enabled=False)

    def _forward_backward(self, batch, rows, mask):
        model = self.model
        fused_stats = False
        if hasattr(model, 'objective') and rows.numel() == batch.y.numel():
            # NLL(S_0) + NLL(S_L) on the raw scores (fused softmax + NLL; the
            # loss kernel also accumulates the running stats).
            with self._autocast():
                loss, count, correct = model.objective(
                    batch.x_s, batch.edge_index_s, batch.edge_attr_s,
                    batch.x_s_batch, batch.x_t, batch.edge_index_t,
                    batch.edge_attr_t, batch.x_t_batch, batch.y, mask,
                    stats=self.stats)
            fused_stats = getattr(model, 'last_stats_fused', False)
        else:
            with self._autocast():
                S_0, S_L = model(batch.x_s, batch.edge_index_s,
                                 batch.edge_attr_s, batch.x_s_batch,
                                 batch.x_t, batch.edge_index_t,
                                 batch.edge_attr_t, batch.x_t_batch)
            y = torch.stack([rows, batch.y], dim=0)
            if model.num_steps:
                loss_L, count, correct = model.loss_stats(S_L, y, mask)
                loss = loss_L + model.loss(S_0, y, mask=mask)
            else:
                loss, count, correct = model.loss_stats(S_0, y, mask)
        # A persistent seed gradient: no fill kernel in the captured step.
        if self._one is None or self._one.device != loss.device:
            self._one = torch.ones((), dtype=loss.dtype, device=loss.device)
        loss.backward(self._one)
        if not fused_stats:
            self.stats[:3] += torch.stack(
                [loss.detach().float(), correct.float(),
                 count.float()]).double()

    def _check_finite(self):
        """Flag non-finite gradients in ``_found_inf`` (device-side)."""
        if not self.guard:
            return
        from .ops import _backend
        flat = self.reducer.flat
        if _backend.use_hip(flat) and flat.dtype == torch.float32:
            # One pass + one fold kernel: found_inf and the skip counter.
            _backend.ops().nonfinite_flag(flat, self._found_inf,
                                          self.stats[3:4])
            return
        bad = torch.logical_not(torch.isfinite(flat).all())
        self._found_inf.copy_(bad.float())
        self.stats[3] += self._found_inf.double()

    def _optimizer_step(self):
        if self.guard and self.device.type != 'cuda':
            # Unfused CPU Adam has no found_inf input: skip on the host.
            if self._found_inf.item() != 0:
                return
        from .runtime import optim as hip_optim
        if hip_optim.supported(self.optimizer):
            hip_optim.hip_adam_step(
                self.optimizer, self._found_inf if self.guard else None)
            return
        self.optimizer.step()

    def _static_body(self, bucket=-1):
        # Gradients are stolen by AccumulateGrad (no zero-fill, no add per
        # parameter) and packed into the flat buffer by one kernel
        # (parallel/ddp.py::pack_grads).
        self.reducer.release_grads()
        batch = self.batchers[bucket].materialize()
        self._forward_backward(batch, self._rows[bucket], batch.y_mask)
        if self.reducer.in_step:
            # DP: the buckets were packed and all-reduced from the backward
            # hooks; wait for the last ones, then check and update - all
            # inside the step (and its hipGraph).
            self.reducer.finish()
            self._check_finite()
            self._optimizer_step()
            return
        # Single process: the pack kernel also flags non-finite gradients
        # and the optimizer's step kernel folds the flags.
        flags = self.reducer.pack_grads(
            with_flags=self.world == 1 and self.guard)
        if self.world == 1:
            from .runtime import optim as hip_optim
            if flags is not None and hip_optim.supported(self.optimizer):
                hip_optim.hip_adam_step(self.optimizer, self._found_inf,
                                        flags, self.stats[3:4])
            else:
                self._check_finite()
                self._optimizer_step()

    def _bucket_body(self, i):
        return lambda: self._static_body(i)

    @property
    def dp_mode_used(self):
        """How gradients are synchronised: ``'none'`` (one rank),
        ``'captured-in-step'`` (bucketed all-reduces inside the captured
        hipGraph), ``'in-step'`` (same, uncaptured static step),
        ``'overlapped-eager'`` (eager step, bucket all-reduces from the
        backward hooks) or ``'flat-after-step'`` (one all-reduce after the
        step / replay)."""
        if self.world == 1:
            return 'none'
        if self.reducer.in_step:
            return 'captured-in-step' if self.mode == 'graph' else 'in-step'
        if self.mode == 'eager' and self.reducer.overlap:
            return 'overlapped-eager'
        return 'flat-after-step'

    @property
    def overflows(self):
        """Batches that fitted no static capacity (resampled)."""
        return sum(b.overflows for b in getattr(self, 'batchers', []))

    def _load_next(self):
        """Stage the next batch into the smallest bucket it fits; returns
        the bucket index."""
        while True:
            s, t = self.batcher.next_ids()
            for i, b in enumerate(self.batchers):
                if b is self.batcher or b.fits(s, t):
                    if b.load(s, t):
                        return i
                    break
            else:
                self.batcher.overflows += 1

    def _snapshot(self):
        """Everything the capture warm-ups advance (model parameters and
        buffers, optimizer moments and step counters, running stats, RNG and
        sampler states), restored IN PLACE by :meth:`_restore` after the
        capture - the captured graphs keep their tensor addresses, and the
        training trajectory is the same as without capturing (a resumed
        graph-mode run continues exactly)."""
        with torch.no_grad():
            snap = {
                'model': {k: t.detach().clone()
                          for k, t in self.model.state_dict().items()},
                'opt': {id(p): {k: v.detach().clone()
                                for k, v in st.items() if torch.is_tensor(v)}
                        for p, st in self.optimizer.state.items()},
                'stats': self.stats.clone(),
                'found_inf': self._found_inf.clone(),
                'cpu_rng': torch.get_rng_state(),
                'sampler': self.batcher.state_dict(),
            }
        if self.device.type == 'cuda':
            snap['cuda_rng'] = torch.cuda.get_rng_state(self.device)
        return snap

    def _restore(self, snap):
        with torch.no_grad():
            for k, t in self.model.state_dict().items():
                t.copy_(snap['model'][k])
            for p, st in self.optimizer.state.items():
                old = snap['opt'].get(id(p), {})
                for k, v in st.items():
                    if not torch.is_tensor(v):
                        continue
                    if k in old:
                        v.copy_(old[k])
                    else:
                        v.zero_()     # created by a warm-up: "never stepped"
            self.stats.copy_(snap['stats'])
            self._found_inf.copy_(snap['found_inf'])
        torch.set_rng_state(snap['cpu_rng'])
        if 'cuda_rng' in snap:
            torch.cuda.set_rng_state(snap['cuda_rng'], self.device)
        self.batcher.load_state_dict(snap['sampler'])

    def _capture_all(self):
        """Capture every bucket's graph up front (so no capture ever lands
        in a timed step): each is staged with a batch that fits it.  The
        warm-up iterations before each capture run real steps; their effect
        on the model, optimizer, RNG and sampler is undone afterwards."""
        snap = self._snapshot()
        check = self.reducer.in_step and self.reducer.distributed
        seqs = []
        for i, b in enumerate(self.batchers):
            for _ in range(10000):
                s, t = self.batcher.next_ids()
                if b.fits(s, t) and b.load(s, t):
                    break
            else:
                raise RuntimeError('no batch fits bucket {}'.format(b))
            if check:
                self.reducer.seq_log = []
            try:
                self._graphs[i].capture()
            finally:
                if check:
                    seqs.append(self.reducer.seq_log)
                    self.reducer.seq_log = None
        self._captured = True
        self._restore(snap)
        if check:
            self._check_collective_sequence(seqs)
        # The capture phase leaves large autograd graphs behind: collect them
        # now, not in the middle of a replayed step (steps pause the cyclic
        # collector themselves, see step()).
        gc.collect()

    def _check_collective_sequence(self, runs_per_bucket):
        """Ranks replay DIFFERENT size-bucket graphs in the same step, so
        every captured graph must issue the same ordered (offset, length)
        all-reduces, on every rank.  ``runs_per_bucket``: per bucket, the
        collective lists of its warm-up runs and its captured run.  Checked
        here (bucket vs bucket) and across ranks (digest all-gather); every
        rank raises together on a mismatch (the bench supervisor then
        retries with the flat after-replay all-reduce)."""
        import torch.distributed as dist
        from .parallel.ddp import sequence_digest
        problems = []
        ref = None
        for i, runs in enumerate(runs_per_bucket):
            if not runs or not runs[-1]:
                problems.append('bucket {}: no collective captured'.format(i))
                continue
            if any(r != runs[-1] for r in runs):
                problems.append('bucket {}: warm-up and captured runs '
                                'differ'.format(i))
            if ref is None:
                ref = runs[-1]
            elif runs[-1] != ref:
                problems.append('bucket {}: sequence differs from bucket '
                                '0'.format(i))
        digest = sequence_digest(ref or [])
        mine = torch.tensor([digest, len(problems)], dtype=torch.int64,
                            device=self.device)
        every = [torch.zeros_like(mine) for _ in range(self.world)]
        dist.all_gather(every, mine)
        every = [tuple(int(v) for v in t.tolist()) for t in every]
        if len({d for d, _ in every}) != 1:
            problems.append('sequence digests differ across ranks')
        bad = any(n for _, n in every) or problems
        self.dp_checks.update({
            'collective_sequence': 'identical' if not bad else 'MISMATCH',
            'collectives_per_step': len(ref or []),
            'bucket_graphs': len(runs_per_bucket),
            'sequence_digest': '{:016x}'.format(digest)})
        if bad:
            raise RuntimeError('captured collective sequence check failed: '
                               '{}'.format('; '.join(problems) or
                                           'on another rank'))

    def step(self):
        """One training step (data, forward, backward, all-reduce, Adam).

        Process-wide settings are only changed for the duration of the
        step: the tuned GEMM solutions are active inside it, and the cyclic
        garbage collector is paused (no collection lands between a step's
        launches); both are restored on return."""
        with tuned_gemms(self.device.type == 'cuda'), _gc_paused():
            self._step()

    def _step(self):
        self.model.train()
        if self.mode == 'eager':
            with trace_range('train.load'):
                batch = next(self._batches)
            self.reducer.zero_grad()
            rows = torch.arange(batch.y.numel(), device=self.device)
            with trace_range('train.forward_backward'):
                self._forward_backward(batch, rows, None)
            with trace_range('train.allreduce'):
                self.reducer.finish()
            with trace_range('train.optimizer'):
                self._check_finite()
                self._optimizer_step()
        else:
            if self._graphs is not None and not self._captured:
                self._capture_all()
            with trace_range('train.load'):
                bucket = self._load_next()
            with trace_range('train.graph_replay' if self._graphs is not None
                             else 'train.forward_backward'):
                if self._graphs is not None:
                    self._graphs[bucket]()
                else:
                    self._static_body(bucket)
            if self.world > 1 and not self.reducer.in_step:
                with trace_range('train.allreduce'):
                    if self.time_allreduce:
                        ev = (torch.cuda.Event(enable_timing=True),
                              torch.cuda.Event(enable_timing=True))
                        ev[0].record()
                    self.reducer.finish()
                    if self.time_allreduce:
                        ev[1].record()
                        self.allreduce_events.append(ev)
                with trace_range('train.optimizer'):
                    self._check_finite()
                    self._optimizer_step()
        self.step_count += 1

    def read_stats(self, reset=True):
        """``(mean loss, Hits@1)`` over the steps since the last reset,
        reduced over ranks (one host synchronisation)."""
        s = self.stats.clone()
        parallel.all_reduce_sum(s)
        out = {'loss_sum': float(s[0]), 'correct': float(s[1]),
               'count': float(s[2]),
               'hits@1': float(s[1] / s[2]) if s[2] > 0 else None,
               'skipped_steps': int(s[3] / max(self.world, 1))}
        if reset:
            self.stats.zero_()
        return out

    # ------------------------------------------------------------------
    @torch.no_grad()
    def evaluate(self, store, num_pairs=1024, batch_size=None, seed=123,
                 k=(1, 10)):
        """Hits@k of ``S_L`` (fraction of ground-truth nodes) on
        ``num_pairs`` random valid pairs of ``store`` (the reference's test
        loop, ``/root/reference/examples/pascal.py:80-99``).  Counts stay on
        the device; one host synchronisation per evaluation."""
        with tuned_gemms(self.device.type == 'cuda'):
            return self._evaluate(store, num_pairs, batch_size, seed, k)

    def _evaluate(self, store, num_pairs, batch_size, seed, k):
        model = self.model
        was_training = model.training
        model.eval()
        bs = batch_size or min(num_pairs, 512)
        loader = DevicePairLoader(store, bs, shuffle=True, drop_last=False,
                                  seed=seed)
        seen = 0
        gt = torch.zeros((), dtype=torch.long, device=self.device)
        hits = {kk: torch.zeros((), dtype=torch.long, device=self.device)
                for kk in k}
        while seen < num_pairs:
            for batch in loader:
                with self._autocast():
                    _, S_L = model(batch.x_s, batch.edge_index_s,
                                   batch.edge_attr_s, batch.x_s_batch,
                                   batch.x_t, batch.edge_index_t,
                                   batch.edge_attr_t, batch.x_t_batch)
                y = torch.stack([torch.arange(batch.y.numel(),
                                              device=self.device), batch.y])
                for kk in k:
                    hits[kk] += model.hits_count(kk, S_L, y)
                gt += y.size(1)
                seen += batch.num_graphs
                if seen >= num_pairs:
                    break
        model.train(was_training)
        tot = torch.stack([gt] + [hits[kk] for kk in k]).cpu()
        return {kk: float(tot[i + 1]) / max(float(tot[0]), 1.0)
                for i, kk in enumerate(k)}

    # ------------------------------------------------------------------
    def _rank_state(self):
        """This rank's private resume state: its sampler (shard order and
        generator), its share of the running stats and its RNG streams."""
        np_state = np.random.get_state()
        sampler = self.loader if self.mode == 'eager' else self.batcher
        rng = {
            'torch': torch.get_rng_state(),
            'python': random.getstate(),
            'numpy': (np_state[0], torch.from_numpy(np_state[1].copy()),
                      int(np_state[2]), int(np_state[3]),
                      float(np_state[4])),
        }
        if self.device.type == 'cuda':
            rng['cuda'] = torch.cuda.get_rng_state(self.device)
        return {'sampler': sampler.state_dict(),
                'stats': self.stats.detach().cpu(), 'rng': rng}

    def state_dict(self, ranks=None):
        """Checkpoint content; every leaf is a tensor or a Python primitive
        so it loads with ``torch.load(..., weights_only=True)``.

        ``ranks``: the per-rank states of every rank (gathered by
        :meth:`save`); defaults to this rank's alone."""
        if ranks is None:
            ranks = [self._rank_state()]
        return {
            'model': self.model.state_dict(),
            'optimizer': self.optimizer.state_dict(),
            'step': self.step_count,
            'world_size': len(ranks),
            'ranks': ranks,
        }

    def save(self, path):
        """Checkpoint written by rank 0: the model (reference key schema)
        and optimizer, which are identical on every rank, plus EVERY rank's
        sampler / stats / RNG state (gathered), so a data-parallel resume
        gives each rank back its own shard position."""
        ranks = parallel.all_gather_state(self._rank_state(), self.device)
        if self.rank == 0:
            tmp = path + '.tmp'
            torch.save(self.state_dict(ranks), tmp)
            os.replace(tmp, path)
        parallel.barrier()

    def _load_optimizer(self, sd):
        """Load optimizer state; tensors that already exist are updated IN
        PLACE (captured graphs and the HIP Adam pointer table hold their
        addresses), missing ones are created by the regular loader."""
        if not self.optimizer.state:
            self.optimizer.load_state_dict(sd)
            return
        params = [p for g in self.optimizer.param_groups for p in g['params']]
        ids = [i for g in sd['param_groups'] for i in g['params']]
        with torch.no_grad():
            for i, p in zip(ids, params):
                src = sd['state'].get(i)
                dst = self.optimizer.state.get(p)
                if src is None or dst is None:
                    continue
                for k, v in src.items():
                    if k in dst and torch.is_tensor(dst[k]) and \
                            torch.is_tensor(v):
                        dst[k].copy_(v.to(dst[k]).reshape(dst[k].shape))
                    else:
                        dst[k] = v
        for g, gs in zip(self.optimizer.param_groups, sd['param_groups']):
            for k, v in gs.items():
                if k != 'params':
                    g[k] = v

    def load(self, path):
        state = torch.load(path, map_location=self.device,
                           weights_only=True)
        self.model.load_state_dict(state['model'])
        self._load_optimizer(state['optimizer'])
        self.step_count = int(state.get('step', 0))
        # (Parameters and optimizer tensors were updated in place, so
        # captured graphs stay valid and are replayed as they are.)
        ranks = state.get('ranks')
        if ranks is None and 'sampler' in state:
            # Round-3 layout: one rank's sampler / stats / RNG streams at the
            # top level of the checkpoint.
            ranks = [{k: state[k] for k in ('sampler', 'stats', 'rng')
                      if k in state}]
        ranks = ranks or []
        if len(ranks) != self.world:
            # Different world size: the shards changed, so the saved sampler
            # positions mean nothing here - keep this rank's freshly seeded
            # sampler and start the running stats from zero.
            warnings.warn(
                'checkpoint {} holds {} rank state(s) for a world of {}: '
                'sampler positions, running stats and RNG streams are NOT '
                'restored (model and optimizer are)'.format(
                    path, len(ranks), self.world))
            self.stats.zero_()
            return state
        mine = ranks[self.rank]
        if self.mode == 'eager':
            self.loader.load_state_dict(mine['sampler'])
            self._batches = self.loader.forever()
        else:
            self.batcher.load_state_dict(mine['sampler'])
        if 'stats' in mine:
            self.stats.copy_(mine['stats'].to(self.stats))
        rng = mine.get('rng', {})
        if 'torch' in rng:
            torch.set_rng_state(rng['torch'].cpu())
        if 'python' in rng:
            random.setstate(rng['python'])
        if 'numpy' in rng:
            name, keys, pos, has_gauss, cached = rng['numpy']
            np.random.set_state((name, keys.cpu().numpy().astype(np.uint32),
                                 pos, has_gauss, cached))
        if 'cuda' in rng and self.device.type == 'cuda':
            torch.cuda.set_rng_state(_cuda_rng_of(rng['cuda'], self.device),
                                     self.device)
        return state


def _cuda_rng_of(saved, device):
    """The CUDA generator state for ``device`` from a checkpoint: a state
    tensor, or (older checkpoints) a list with one state per device."""
    if isinstance(saved, (list, tuple)):
        idx = device.index or 0
        saved = saved[idx] if idx < len(saved) else saved[0]
    return saved.cpu()


class _gc_paused(object):
    """Pause the cyclic garbage collector inside the block (restoring the
    caller's setting)."""

    def __enter__(self):
        self._was = gc.isenabled()
        gc.disable()

    def __exit__(self, *exc):
        if self._was:
            gc.enable()
        return False


class MetricsLogger(object):
    """Append-only JSONL metrics (rank 0)."""

    def __init__(self, path=None):
        self.path = path
        self.t0 = time.time()

    def log(self, **fields):
        if self.path is None or parallel.rank() != 0:
            return
        fields.setdefault('time', round(time.time() - self.t0, 3))
        with open(self.path, 'a') as f:
            f.write(json.dumps(fields) + '\n')


class KGTrainer(object):
    r"""Full-graph KG alignment trainer (DBP15K driver semantics,
    ``/root/reference/examples/dbp15k.py:37-69``).

    One step = forward on the whole pair with ``train_y`` (random negatives
    + ground-truth injection in the sparse top-k path), ``NLL(S_L)``,
    backward, Adam.  The graph is static, so with ``graph=True`` each phase
    (``num_steps``/``detach`` setting) is captured once into a hipGraph.
    """

    def __init__(self, model, data, lr=1e-3, graph=True, bf16=False,
                 guard_nonfinite=True):
        self.model = model
        self.data = data
        if data.x1.dim() == 2 and data.x1.shape[1:] == data.x2.shape[1:] \
                and data.x1.dtype == data.x2.dtype and \
                not (data.x1._base is not None and
                     data.x1._base is data.x2._base):
            # Both graphs' features in ONE buffer (x1 / x2 become row views
            # of it): the model's joint encoding reads it in place - no
            # concatenation per step (models/dgmc.py::_cat_rows); in-place
            # writes to data.x1 / x2 still reach a captured step.
            joint = torch.cat([data.x1, data.x2], 0)
            data.x1 = joint[:data.x1.size(0)]
            data.x2 = joint[data.x1.size(0):]
        self.device = data.x1.device
        cuda = self.device.type == 'cuda'
        self.graph = graph and cuda
        self.bf16 = bf16 and cuda
        if cuda:
            use_tuned_gemms()
        self.optimizer = torch.optim.Adam(model.parameters(), lr=lr,
                                          fused=cuda, capturable=self.graph)
        self.last_loss = torch.zeros((), device=self.device)
        # Non-finite guard as in PairTrainer: a step whose gradients hold a
        # NaN / Inf skips its update (and step counters) on the device;
        # ``skipped`` counts them (no host sync, capturable).
        self.guard = guard_nonfinite
        self._found_inf = torch.zeros((), dtype=torch.float32,
                                      device=self.device)
        self._unit = torch.ones((), dtype=torch.float32, device=self.device)
        self.skipped = torch.zeros((), dtype=torch.float64, device=self.device)
        if self.guard and cuda:
            self.optimizer.found_inf = self._found_inf
        self._graphs = {}
        self.step_count = 0

    def _autocast(self):
        return torch.autocast(device_type=self.device.type,
                              dtype=torch.bfloat16, enabled=self.bf16,
                              cache_enabled=False)

    def _body(self):
        d, model = self.data, self.model
        for p in model.parameters():
            p.grad = None
        with self._autocast():
            _, S_L = model(d.x1, d.edge_index1, None, None, d.x2,
                           d.edge_index2, None, None, d.train_y)
        loss = model.loss(S_L, d.train_y)
        loss.backward()
        self._update()
        self.last_loss.copy_(loss.detach())

    def _update(self):
        """Non-finite check over the gradients this phase produced (one
        multi-tensor kernel) + the HIP multi-tensor Adam reading the flag
        (runtime/optim.py); stock Adam where that is unsupported."""
        from .runtime import optim as hip_optim
        grads = [p.grad for p in self.model.parameters()
                 if p.grad is not None]
        if self.guard and grads:
            self._found_inf.zero_()
            torch._amp_foreach_non_finite_check_and_unscale_(
                grads, self._found_inf, self._unit)
            self.skipped += self._found_inf.double()
            if self.device.type != 'cuda' and self._found_inf.item() != 0:
                return                   # CPU Adam has no found_inf input
        if hip_optim.supported(self.optimizer):
            hip_optim.hip_adam_step(self.optimizer,
                                    self._found_inf if self.guard else None)
            return
        self.optimizer.step()

    def step(self):
        with tuned_gemms(self.device.type == 'cuda'), _gc_paused():
            self._step()

    def _step(self):
        self.model.train()
        if not self.graph:
            self._body()
            self.step_count += 1
            return
        key = (self.model.num_steps, self.model.detach, self.model.k)
        g = self._graphs.get(key)
        if g is None:
            # Capture this phase; its warm-up steps are undone afterwards
            # (same trajectory as without capturing).
            snap = self._snapshot()
            g = self._graphs[key] = GraphedStep(self._body_static,
                                                warmup=2).capture()
            self._restore(snap)
        g()
        self.step_count += 1

    def _snapshot(self):
        with torch.no_grad():
            snap = {'model': {k: t.detach().clone()
                              for k, t in self.model.state_dict().items()},
                    'opt': {id(p): {k: v.detach().clone()
                                    for k, v in st.items()
                                    if torch.is_tensor(v)}
                            for p, st in self.optimizer.state.items()},
                    'loss': self.last_loss.clone(),
                    'skipped': self.skipped.clone(),
                    'cpu_rng': torch.get_rng_state()}
        if self.device.type == 'cuda':
            snap['cuda_rng'] = torch.cuda.get_rng_state(self.device)
        return snap

    def _restore(self, snap):
        with torch.no_grad():
            for k, t in self.model.state_dict().items():
                t.copy_(snap['model'][k])
            for p, st in self.optimizer.state.items():
                old = snap['opt'].get(id(p), {})
                for k, v in st.items():
                    if torch.is_tensor(v):
                        if k in old:
                            v.copy_(old[k])
                        else:
                            v.zero_()
            self.last_loss.copy_(snap['loss'])
            self.skipped.copy_(snap['skipped'])
        torch.set_rng_state(snap['cpu_rng'])
        if 'cuda_rng' in snap:
            torch.cuda.set_rng_state(snap['cuda_rng'], self.device)

    def state_dict(self):
        """Checkpoint: model (reference key schema), optimizer, step count,
        schedule knobs (``num_steps`` / ``detach``, ``dbp15k.py:64-69``) and
        RNG states; loads with ``torch.load(..., weights_only=True)``."""
        state = {'model': self.model.state_dict(),
                 'optimizer': self.optimizer.state_dict(),
                 'step': self.step_count,
                 'schedule': {'num_steps': self.model.num_steps,
                              'detach': bool(self.model.detach),
                              'k': int(self.model.k)},
                 'rng': {'torch': torch.get_rng_state()},
                 # non-finite steps skipped so far (the device counter)
                 'skipped': float(self.skipped)}
        if self.device.type == 'cuda':
            state['rng']['cuda'] = torch.cuda.get_rng_state(self.device)
        return state

    def save(self, path):
        if parallel.rank() == 0:
            tmp = path + '.tmp'
            torch.save(self.state_dict(), tmp)
            os.replace(tmp, path)
        parallel.barrier()

    def load(self, path):
        state = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(state['model'])
        PairTrainer._load_optimizer(self, state['optimizer'])
        self.step_count = int(state.get('step', 0))
        sch = state.get('schedule', {})
        if sch:
            self.model.num_steps = sch['num_steps']
            self.model.detach = sch['detach']
            self.model.k = sch['k']
        if 'skipped' in state:
            self.skipped.fill_(float(state['skipped']))
        rng = state.get('rng', {})
        if 'torch' in rng:
            torch.set_rng_state(rng['torch'].cpu())
        if 'cuda' in rng and self.device.type == 'cuda':
            torch.cuda.set_rng_state(_cuda_rng_of(rng['cuda'], self.device),
                                     self.device)
        return state

    def _body_static(self):
        d, model = self.data, self.model
        # AccumulateGrad *steals* each freshly computed gradient (no zero
        # fill + add kernel per parameter); inside the captured graph the
        # stolen tensors keep their addresses, which the captured Adam
        # step reads.  Parameters without a gradient this phase (psi_1 under
        # detach=True) are skipped by Adam, as after torch's default
        # zero_grad(set_to_none=True) in the reference driver's loop.
        for p in model.parameters():
            p.grad = None
        with self._autocast():
            _, S_L = model(d.x1, d.edge_index1, None, None, d.x2,
                           d.edge_index2, None, None, d.train_y)
        loss = model.loss(S_L, d.train_y)
        loss.backward()
        self._update()
        self.last_loss.copy_(loss.detach())

    @torch.no_grad()
    def evaluate(self, k=10):
        with tuned_gemms(self.device.type == 'cuda'):
            return self._evaluate(k)

    def _evaluate(self, k):
        d, model = self.data, self.model
        model.eval()
        with self._autocast():
            _, S_L = model(d.x1, d.edge_index1, None, None, d.x2,
                           d.edge_index2, None, None)
        hits1 = model.acc(S_L, d.test_y)
        hitsk = model.hits_at_k(k, S_L, d.test_y)
        model.train()
        return hits1, hitsk
