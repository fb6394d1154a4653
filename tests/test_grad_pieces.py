"""Pieces of one parameter's gradient all-reduced as they are produced
(parallel/ddp.py: ``grad_sink`` / ``reduce_piece`` / ``mark_reduced``; the
producer is psi_1 layer 0's weight gradient in ops/slot_gemm.py).

* CPU / gloo, 2 ranks: a toy op writes its weight gradient in two pieces
  into the in-step reducer's flat view and reduces each at once; after
  ``finish`` every rank holds the rank average (equal to the plain bucket
  path), the parameter's gradient IS the flat view, and its bucket did not
  reduce it a second time.
* GPU, 2 ranks on one device over gloo, static mode: the PascalVOC-width
  model (psi_1 layer 0 >= 8 MiB, pieced, each piece reduced from inside the
  backward) trains bit-identically to the same run with one flat all-reduce
  after the step.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


class _PiecedMatmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        return x @ w

    @staticmethod
    def backward(ctx, g):
        from deep_graph_matching_consensus_amd.parallel.ddp import grad_sink
        x, = ctx.saved_tensors
        gw = x.t() @ g
        sink = _PiecedMatmul.sink_override
        if sink is None:
            return None, gw
        view = sink.grad_view(_PiecedMatmul.param)
        K, N = gw.shape
        half = K // 2
        view[:half] = gw[:half]
        sink.reduce_piece(_PiecedMatmul.param, 0, half * N)
        view[half:] = gw[half:]
        sink.reduce_piece(_PiecedMatmul.param, half * N, K * N)
        sink.mark_reduced(_PiecedMatmul.param)
        assert grad_sink(_PiecedMatmul.param) is sink
        return None, view


def _toy_worker(rank, world, port, pieced, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS='1')
    torch.set_num_threads(1)
    import torch.distributed as dist
    from deep_graph_matching_consensus_amd.parallel.ddp import \
        GradBucketAllReducer
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.manual_seed(0)
    lin = torch.nn.Linear(6, 5)
    w = torch.nn.Parameter(torch.randn(8, 5))
    mod = torch.nn.Module()
    mod.lin, mod.w = lin, w
    red = GradBucketAllReducer(mod, bucket_bytes=64, in_step=True)
    _PiecedMatmul.param = w
    _PiecedMatmul.sink_override = red if pieced else None
    g = torch.Generator().manual_seed(10 + rank)
    x = torch.randn(3, 8, generator=g)
    red.release_grads()
    y = _PiecedMatmul.apply(x, w)
    loss = (y * lin(torch.randn(3, 6, generator=g))).sum()
    launches = []
    orig = red._launch_range
    red._launch_range = lambda lo, hi: (launches.append((lo, hi)),
                                        orig(lo, hi))
    loss.backward()
    red.finish()
    off, n = red._slot[w]
    out[rank] = (w.grad.clone(), lin.weight.grad.clone(),
                 w.grad.data_ptr() == red.flat[off:].data_ptr(),
                 sum(1 for lo, hi in launches if lo <= off < hi))
    dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context('spawn')
    manager = ctx.Manager()
    out = manager.dict()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args +
                         (out, )) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    return [out[r] for r in range(world)]


def test_gradient_pieces_reduced_once_cpu():
    a = _spawn(_toy_worker, 2, True)
    b = _spawn(_toy_worker, 2, False)
    for r in range(2):
        assert torch.equal(a[r][0], a[0][0])          # averaged everywhere
        torch.testing.assert_close(a[r][0], b[r][0])  # == bucket path
        torch.testing.assert_close(a[r][1], b[r][1])
        assert a[r][2]                    # the gradient IS the flat view
        assert a[r][3] == 1               # piece 1 only (no second reduce)


def _pascal_worker(rank, world, port, env, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK='0',
                      OMP_NUM_THREADS='1', **env)
    import torch.distributed as dist
    from deep_graph_matching_consensus_amd import train as train_mod
    from deep_graph_matching_consensus_amd.datasets import (
        PASCAL_VOC_CATEGORIES, GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.ops import slot_gemm
    train_mod.IN_STEP_ALLREDUCE = env['IN_STEP'] == '1'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(1024, 256, 2, 2, cat=False, dropout=0.0),
                 SplineCNN(128, 128, 2, 2, cat=True), num_steps=2).cuda()
    assert model.psi_1.convs[0].weight.numel() * 4 >= slot_gemm.PIECE_BYTES
    groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES[:4], graphs=16,
                                    seed=3)
    store = GraphStore(groups, 'cuda', valid_pairs=True)
    trainer = train_mod.PairTrainer(model, store, 32, mode='static',
                                    seed=0)
    assert trainer.reducer.in_step == (env['IN_STEP'] == '1')
    for _ in range(3):
        trainer.step()
    torch.cuda.synchronize()
    out[rank] = torch.cat([p.detach().reshape(-1).cpu()
                           for p in model.parameters()])
    dist.destroy_process_group()


@pytest.mark.gpu
def test_pieced_weight_gradient_two_ranks_static_gpu():
    # (pieces in both runs: the flat after-step all-reduce has no sink)
    env = {'DGMC_AMD_DIST_BACKEND': 'gloo',
           'DGMC_AMD_WGRAD_PIECES_ALWAYS': '1'}
    a = _spawn(_pascal_worker, 2, dict(env, IN_STEP='1'))
    b = _spawn(_pascal_worker, 2, dict(env, IN_STEP='0'))
    assert torch.equal(a[0], a[1])
    assert torch.equal(a[0], b[0])


def _twice_worker(rank, world, port, env, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK='0',
                      OMP_NUM_THREADS='1', **env)
    import torch.distributed as dist
    from deep_graph_matching_consensus_amd.nn import SplineConv
    from deep_graph_matching_consensus_amd.ops import slot_gemm
    from deep_graph_matching_consensus_amd.parallel.ddp import \
        GradBucketAllReducer
    from deep_graph_matching_consensus_amd.runtime.cache import forward_cache
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    conv = SplineConv(1024, 256, dim=2, kernel_size=5).cuda()
    assert conv.weight.numel() * 4 >= slot_gemm.PIECE_BYTES
    g = torch.Generator().manual_seed(20 + rank)
    n, e = 96, 384
    ei = torch.randint(n, (2, e), generator=g).cuda()
    pseudo = torch.rand(e, 2, generator=g).cuda()
    x = torch.randn(n, 1024, generator=g).cuda()
    red = GradBucketAllReducer(conv, in_step=env['IN_STEP'] == '1')
    if env['IN_STEP'] == '1':
        red.release_grads()
    else:
        red.zero_grad()
    with forward_cache():
        # The same weight used twice in one step (the ADVICE r4 case): the
        # pieced path must not run (it would reduce the first use's view
        # while the second use still adds into it).
        y = conv(x, ei, pseudo) + conv(x.flip(0), ei, pseudo)
    (y * y).sum().backward()
    if env['IN_STEP'] == '1':
        assert not red._pre, 'pieced path taken for a twice-used weight'
    red.finish()
    torch.cuda.synchronize()
    out[rank] = torch.cat([p.grad.reshape(-1).cpu()
                           for p in conv.parameters()])
    dist.destroy_process_group()


@pytest.mark.gpu
def test_twice_used_weight_skips_pieces_gpu():
    """a SplineConv weight used twice in one step must take the
    ordinary weight-gradient path even with pieces forced; the averaged
    gradient equals the flat after-step all-reduce."""
    env = {'DGMC_AMD_DIST_BACKEND': 'gloo',
           'DGMC_AMD_WGRAD_PIECES_ALWAYS': '1'}
    a = _spawn(_twice_worker, 2, dict(env, IN_STEP='1'))
    b = _spawn(_twice_worker, 2, dict(env, IN_STEP='0'))
    assert torch.equal(a[0], a[1])
    torch.testing.assert_close(a[0], b[0], rtol=1e-5, atol=1e-5)
