"""Data-parallel correctness on CPU with the gloo backend (world_size 2).

Each rank computes gradients on its own shard; after
``GradBucketAllReducer.finish`` every rank must hold the exact average of
the per-rank gradients (checked against a single-process recomputation),
overlap hooks included, and parameters must stay bit-identical across ranks
through optimizer steps.  The bench's distributed path uses the same
reducer over RCCL.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deep_graph_matching_consensus_amd.datasets import (
    DevicePairLoader, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
from deep_graph_matching_consensus_amd.parallel import GradBucketAllReducer


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _model():
    torch.manual_seed(0)
    return DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                SplineCNN(8, 8, 2, 2, cat=True), num_steps=2)


def _batches():
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=2)
    store = GraphStore(groups, 'cpu')
    loader = DevicePairLoader(store, batch_size=8, shuffle=False, seed=0)
    return list(loader)[:2]


def _loss(model, batch, seed):
    torch.manual_seed(seed)
    S_0, S_L = model(batch.x_s, batch.edge_index_s, batch.edge_attr_s,
                     batch.x_s_batch, batch.x_t, batch.edge_index_t,
                     batch.edge_attr_t, batch.x_t_batch)
    y = torch.stack([torch.arange(batch.y.numel()), batch.y])
    return model.loss(S_0, y) + model.loss(S_L, y)


def _worker(rank, world, port, overlap, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    model = _model()
    if rank == 1:   # desynchronise: the reducer must broadcast rank 0 state
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    reducer = GradBucketAllReducer(model, bucket_bytes=64 << 10,
                                   overlap=overlap)
    batch = _batches()[rank]
    reducer.zero_grad()
    _loss(model, batch, seed=10 + rank).backward()
    reducer.finish()
    grads = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    opt.step()
    params = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    out[rank] = (grads.clone(), params.clone())
    dist.destroy_process_group()


@pytest.mark.parametrize('overlap', [True, False])
def test_grad_allreduce_matches_average(overlap):
    world = 2
    ctx = mp.get_context('spawn')
    manager = ctx.Manager()
    out = manager.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, overlap, out))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0

    # Single-process reference: average of the two shard gradients.
    batches = _batches()
    ref = []
    for rank in range(world):
        model = _model()
        _loss(model, batches[rank], seed=10 + rank).backward()
        ref.append(torch.cat([p.grad.reshape(-1)
                              for p in model.parameters()]))
    expected = (ref[0] + ref[1]) / 2
    g0, p0 = out[0]
    g1, p1 = out[1]
    assert torch.allclose(g0, expected, atol=1e-6, rtol=1e-5)
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)


def _bench_worker(rank, world, port, mode, out_path, batch=16,
                  dp_mode='captured'):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS='1')
    torch.set_num_threads(1)
    import bench
    bench.main(['--gpus', str(world), '--steps', '2', '--warmup', '1',
                '--batch-size', str(batch),
                '--graphs-per-category', '8', '--dtype', 'fp32', '--mode',
                mode, '--dp-mode', dp_mode, '--json-out', out_path])


@pytest.mark.parametrize('mode,world,batch,dp_mode', [
    ('eager', 2, 16, 'captured'), ('static', 2, 16, 'captured'),
    ('static', 2, 16, 'flat'), ('eager', 8, 32, 'captured'),
    ('static', 8, 32, 'captured')])
def test_bench_ranks_gloo(tmp_path, mode, world, batch, dp_mode):
    """The bench's distributed path (rank sharding, all-reduce, max-time
    reduction, rank-0 JSON) runs end to end with gloo ranks.  With 8 ranks
    each shard (160 graphs / 8 = 20 sources) is smaller than the batch, as
    in the 8-GPU PascalVOC run (2560 / 8 = 320 < 512)."""
    import json
    out_path = str(tmp_path / 'bench.json')
    ctx = mp.get_context('spawn')
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker,
                         args=(r, world, port, mode, out_path, batch,
                               dp_mode))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    with open(out_path) as f:
        result = json.loads(f.read())
    assert result['n_gpus'] == world
    assert result['config']['global_batch'] == batch * world
    assert result['config']['parallelism'] == 'dp{}'.format(world)
    assert result['value'] > 0
    # DP diagnostics
    expect = {'eager': 'overlapped-eager',
              'static': 'in-step' if dp_mode == 'captured'
              else 'flat-after-step'}[mode]
    assert result['dp_mode'] == expect
    assert result['ms_per_step_rank_min'] <= result['ms_per_step_rank_max']
    assert result['allreduce_standalone_ms'] > 0
    assert result['allreduce_bytes'] > 0
    assert 'gemm_arith' in result
    # every rank applied the same averaged update: bit-identical parameters
    assert result['params_in_sync'], result['params_max_rank_diff']
