"""Failure detection: non-finite steps are skipped; a failing rank does not
hang its peers."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from deep_graph_matching_consensus_amd.datasets import (
    GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
from deep_graph_matching_consensus_amd.train import PairTrainer


def _trainer(store, mode):
    torch.manual_seed(0)
    model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                 SplineCNN(8, 8, 2, 2, cat=True), num_steps=1)
    return PairTrainer(model, store, 8, mode=mode, bf16=False, seed=0)


@pytest.mark.parametrize('mode', ['eager', 'static'])
def test_nonfinite_step_is_skipped(mode):
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=5)
    store = GraphStore(groups, 'cpu')
    tr = _trainer(store, mode)
    tr.step()                                   # a normal step
    before = {k: v.clone() for k, v in tr.model.state_dict().items()}
    feats = [store.x] + ([tr.batcher.x] if hasattr(tr, 'batcher') else [])
    good = [f.clone() for f in feats]
    for f in feats:
        f.fill_(float('nan'))                   # poisoned batch
    tr.step()
    for k, v in tr.model.state_dict().items():
        assert torch.equal(v, before[k]), k     # update skipped
    stats = tr.read_stats()
    assert stats['skipped_steps'] == 1
    for f, g in zip(feats, good):
        f.copy_(g)
    tr.step()                                   # training resumes
    changed = any(not torch.equal(v, before[k])
                  for k, v in tr.model.state_dict().items())
    assert changed
    assert tr.read_stats()['skipped_steps'] == 0


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _fault_worker(rank, world, port, q):
    import datetime
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.distributed.init_process_group(
        'gloo', rank=rank, world_size=world,
        timeout=datetime.timedelta(seconds=20))
    t = torch.ones(4)
    torch.distributed.all_reduce(t)             # healthy collective
    def report(msg, code):
        q.put((rank, msg))
        q.close()
        q.join_thread()
        os._exit(code)      # skip process-group teardown of a broken group

    if rank == 1:
        report('raised', 3)                     # rank dies mid-training
    try:
        torch.distributed.all_reduce(t)
        report('no-error', 0)
    except Exception as e:                      # peers fail, not hang
        report('error:' + type(e).__name__, 0)


def test_dead_rank_fails_peers_instead_of_hanging():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fault_worker, args=(r, 2, port, q))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=90)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, 'a rank hung after its peer died'
    out = dict(q.get(timeout=5) for _ in range(2))
    assert out[1] == 'raised'
    assert out[0].startswith('error:'), out
