"""Data-parallel training steps through :class:`PairTrainer` (static and
captured-graph modes) with two ranks.

* CPU / gloo: the in-step path (stolen gradients, each bucket packed and
  all-reduced from the backward hook that completes it, check + Adam inside
  the step) gives bit-identical parameters on both ranks and the same
  parameters as one flat all-reduce after the step.
* GPU: two ranks on ``cuda:0`` over gloo (``DGMC_AMD_DIST_BACKEND=gloo``) in
  ``mode='graph'`` - the captured step with the non-capturable backend's
  fallback (all-reduce after the replay) - stay bit-identical across ranks
  and match the uncaptured static step.  (RCCL refuses two ranks on one
  device; the captured RCCL all-reduce runs in the driver's 8-GPU bench.)
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


def _worker(rank, world, port, mode, device, env, steps, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0', OMP_NUM_THREADS='1', **env)
    torch.set_num_threads(1)
    import torch.distributed as dist
    from deep_graph_matching_consensus_amd import train as train_mod
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    train_mod.IN_STEP_ALLREDUCE = env.get('DGMC_AMD_IN_STEP_ALLREDUCE',
                                          '1') == '1'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    if device == 'cuda':
        torch.cuda.set_device(0)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(16, 16, 2, 2, cat=False, dropout=0.5),
                 SplineCNN(8, 8, 2, 2, cat=True), num_steps=2).to(device)
    groups = make_keypoint_datasets(graphs=8, feature_dim=16, seed=2)
    store = GraphStore(groups, device)
    trainer = train_mod.PairTrainer(model, store, 8, mode=mode, bf16=False,
                                    seed=0, buckets=env.get(
                                        'DGMC_TEST_BUCKETS') == '1',
                                    bucket_bytes=16 << 10)
    assert len(trainer.reducer.buckets) > 2      # several all-reduces
    assert trainer.reducer.in_step == (mode == 'static' and
                                       env.get('DGMC_AMD_IN_STEP_ALLREDUCE',
                                               '1') == '1')
    for _ in range(steps):
        trainer.step()
    if device == 'cuda':
        torch.cuda.synchronize()
    out[rank] = torch.cat([p.detach().reshape(-1).cpu()
                           for p in model.parameters()])
    out['caps%d' % rank] = [b.caps for b in getattr(trainer, 'batchers', [])]
    dist.destroy_process_group()


def _run(mode, device, env=None, steps=3, world=2):
    ctx = mp.get_context('spawn')
    manager = ctx.Manager()
    out = manager.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, mode, device, env or {}, steps,
                               out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    _run.caps = [out['caps%d' % r] for r in range(world)]
    return [out[r] for r in range(world)]


def test_in_step_allreduce_matches_post_step_cpu():
    a = _run('static', 'cpu')
    assert torch.equal(a[0], a[1])
    # Shards differ, static capacities agree (max over the ranks).
    assert _run.caps[0] == _run.caps[1]
    b = _run('static', 'cpu', {'DGMC_AMD_IN_STEP_ALLREDUCE': '0'})
    assert torch.equal(b[0], b[1])
    assert torch.equal(a[0], b[0])


@pytest.mark.gpu
def test_graph_mode_two_ranks_gloo_on_one_gpu():
    env = {'DGMC_AMD_DIST_BACKEND': 'gloo'}
    g = _run('graph', 'cuda', env)
    assert torch.equal(g[0], g[1])
    s = _run('static', 'cuda', env)
    assert torch.equal(s[0], s[1])
    torch.testing.assert_close(g[0], s[0], atol=1e-6, rtol=1e-5)


@pytest.mark.gpu
def test_graph_mode_size_buckets_agree_across_ranks():
    """Rank shards differ, yet every rank builds the same static capacities
    and size buckets (so the captured graphs - and their collectives - pair
    up across ranks); parameters stay bit-identical."""
    env = {'DGMC_AMD_DIST_BACKEND': 'gloo', 'DGMC_TEST_BUCKETS': '1'}
    g = _run('graph', 'cuda', env, steps=4)
    assert torch.equal(g[0], g[1])
    assert _run.caps[0] == _run.caps[1] and len(_run.caps[0]) >= 1
