"""Checkpoint schema (reference state-dict keys) and trainer resume."""
import pytest
import torch

from deep_graph_matching_consensus_amd.datasets import (
    GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import (DGMC, GIN, RelCNN,
                                                      SplineCNN)
from deep_graph_matching_consensus_amd.train import PairTrainer


def test_reference_state_dict_keys_spline():
    model = DGMC(SplineCNN(1024, 256, 2, 2, cat=False, dropout=0.5),
                 SplineCNN(128, 128, 2, 2, cat=True), num_steps=10)
    sd = model.state_dict()
    expect = {
        'psi_1.convs.0.weight': (25, 1024, 256),
        'psi_1.convs.0.root': (1024, 256),
        'psi_1.convs.0.bias': (256, ),
        'psi_1.convs.0.kernel_size': (2, ),
        'psi_1.convs.0.is_open_spline': (2, ),
        'psi_1.convs.1.weight': (25, 256, 256),
        'psi_1.final.weight': (256, 256),
        'psi_2.convs.0.weight': (25, 128, 128),
        'psi_2.final.weight': (128, 128 + 2 * 128),
        'mlp.0.weight': (128, 128), 'mlp.0.bias': (128, ),
        'mlp.2.weight': (1, 128), 'mlp.2.bias': (1, ),
    }
    for key, shape in expect.items():
        assert tuple(sd[key].shape) == shape, key
    assert sd['psi_1.convs.0.kernel_size'].dtype == torch.long
    assert sd['psi_1.convs.0.is_open_spline'].dtype == torch.uint8
    # Parameter count from SURVEY.md section 2.2 (PascalVOC config).
    n = sum(p.numel() for p in model.parameters())
    assert n == 9504129


def test_reference_state_dict_keys_gin_rel():
    gin = DGMC(GIN(32, 16, 2), GIN(8, 8, 2), num_steps=1).state_dict()
    assert 'psi_1.convs.0.eps' in gin
    assert 'psi_1.convs.0.nn.lins.0.weight' in gin
    assert 'psi_1.convs.0.nn.batch_norms.1.running_var' in gin
    rel_model = DGMC(RelCNN(300, 256, 3, dropout=0.5), RelCNN(32, 32, 3),
                     num_steps=None, k=10)
    rel = rel_model.state_dict()
    for key in ['psi_1.convs.0.lin1.weight', 'psi_1.convs.0.lin2.weight',
                'psi_1.convs.0.root.weight', 'psi_1.convs.0.root.bias',
                'psi_1.batch_norms.2.num_batches_tracked',
                'psi_1.final.weight']:
        assert key in rel, key
    n = sum(p.numel() for p in rel_model.parameters())
    assert n == 914305  # DBP15K parameter total


def test_trainer_checkpoint_resume(tmp_path):
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=5)
    store = GraphStore(groups, 'cpu')

    def make():
        torch.manual_seed(0)
        model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                     SplineCNN(8, 8, 2, 2, cat=True), num_steps=1)
        return PairTrainer(model, store, 8, mode='eager', bf16=False,
                           seed=0)

    a = make()
    a.step()
    path = str(tmp_path / 'ckpt.pt')
    a.save(path)
    ref_state = {k: v.clone() for k, v in a.model.state_dict().items()}
    b = make()
    b.load(path)
    assert b.step_count == 1
    for k, v in b.model.state_dict().items():
        assert torch.equal(v, ref_state[k]), k
    sa = a.optimizer.state_dict()['state']
    sb = b.optimizer.state_dict()['state']
    for i in sa:
        assert torch.equal(sa[i]['exp_avg'], sb[i]['exp_avg'])


def _pair_trainer(store, mode, seed_model=0):
    # (graph mode: the store lives on the GPU)
    torch.manual_seed(seed_model)
    model = DGMC(SplineCNN(16, 16, 2, 2, cat=False, dropout=0.5),
                 SplineCNN(8, 8, 2, 2, cat=True), num_steps=2).to(store.device)
    return PairTrainer(model, store, 8, mode=mode, bf16=False, seed=3)


def _run_trajectory(trainer, steps):
    losses = []
    for _ in range(steps):
        trainer.step()
        losses.append(trainer.read_stats()['loss_sum'])
    return losses


@pytest.mark.parametrize('mode', [
    'eager', 'static', pytest.param('graph', marks=pytest.mark.gpu)])
def test_interrupted_run_continues_bit_for_bit(tmp_path, mode):
    """Save after 2 of 5 steps, resume in a fresh process-like trainer (other
    init): losses of steps 3-5 and the final weights / Adam moments equal the
    uninterrupted run bit for bit (model, optimizer, RNG AND sampler state
    are in the checkpoint).  Graph mode: the resumed trainer captures its
    graphs (warm-ups undone by _snapshot/_restore) after the load and then
    replays them; the trajectory still continues exactly."""
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=5)
    store = GraphStore(groups, 'cuda' if mode == 'graph' else 'cpu')
    torch.manual_seed(123)
    full = _pair_trainer(store, mode)
    ref_losses = _run_trajectory(full, 5)

    torch.manual_seed(123)
    first = _pair_trainer(store, mode)
    assert _run_trajectory(first, 2) == ref_losses[:2]
    path = str(tmp_path / 'ckpt.pt')
    first.save(path)
    torch.manual_seed(999)                  # a different process state
    resumed = _pair_trainer(store, mode, seed_model=7)
    resumed.load(path)
    assert resumed.step_count == 2
    assert _run_trajectory(resumed, 3) == ref_losses[2:]
    for (k, v), w in zip(full.model.state_dict().items(),
                         resumed.model.state_dict().values()):
        assert torch.equal(v, w), k
    sa = full.optimizer.state_dict()['state']
    sb = resumed.optimizer.state_dict()['state']
    for i in sa:
        assert torch.equal(sa[i]['exp_avg_sq'], sb[i]['exp_avg_sq'])


def test_kg_trainer_checkpoint_resume(tmp_path):
    from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair
    from deep_graph_matching_consensus_amd.train import KGTrainer
    data = make_kg_pair('zh_en', scale=0.01, seed=0)

    def make(seed):
        torch.manual_seed(seed)
        psi_1 = RelCNN(data.x1.size(-1), 16, 2, cat=True, lin=True,
                       dropout=0.5)
        psi_2 = RelCNN(8, 8, 2, cat=True, lin=True)
        model = DGMC(psi_1, psi_2, num_steps=None, k=4)
        return KGTrainer(model, data, lr=1e-3, graph=False)

    def run(tr, steps):
        out = []
        for _ in range(steps):
            tr.step()
            out.append(float(tr.last_loss))
        return out

    torch.manual_seed(1)
    full = make(0)
    full.model.num_steps, full.model.detach = 2, True
    ref = run(full, 4)
    torch.manual_seed(1)
    a = make(0)
    a.model.num_steps, a.model.detach = 2, True
    assert run(a, 2) == ref[:2]
    path = str(tmp_path / 'kg.pt')
    a.save(path)
    b = make(5)
    b.load(path)
    assert b.step_count == 2 and b.model.num_steps == 2 and b.model.detach
    assert run(b, 2) == ref[2:]
    for (k, v), w in zip(full.model.state_dict().items(),
                         b.model.state_dict().values()):
        assert torch.equal(v, w), k


def _dp_resume_worker(rank, world, port, path, out):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS='1')
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=5)
    store = GraphStore(groups, 'cpu')

    torch.manual_seed(123)
    full = _pair_trainer(store, 'eager')
    ref = _run_trajectory(full, 5)
    torch.manual_seed(123)
    first = _pair_trainer(store, 'eager')
    _run_trajectory(first, 2)
    first.save(path)
    torch.manual_seed(999)
    resumed = _pair_trainer(store, 'eager', seed_model=7)
    state = resumed.load(path)
    out[rank] = {'ref': ref, 'resumed': _run_trajectory(resumed, 3),
                 'world': state['world_size'],
                 'order': [r['sampler']['order'] for r in state['ranks']]}
    dist.destroy_process_group()


def test_data_parallel_resume_restores_each_rank_shard(tmp_path):
    """Two gloo ranks: the checkpoint holds BOTH ranks' sampler states (their
    shards differ), each rank resumes its own, and every rank's per-step
    losses (reduced over ranks by read_stats) continue the uninterrupted
    run exactly - no rank replays rank 0's batches, no stats inflation."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    out = ctx.Manager().dict()
    path = str(tmp_path / 'dp.pt')
    procs = [ctx.Process(target=_dp_resume_worker,
                         args=(r, 2, port, path, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    for r in range(2):
        res = out[r]
        assert res['world'] == 2
        assert res['resumed'] == res['ref'][2:], r
    o0, o1 = out[0]['order']
    assert o0 is not None and o1 is not None and not torch.equal(o0, o1)


def test_legacy_round3_checkpoint_layout_resumes(tmp_path):
    """a round-3 checkpoint (sampler / stats / rng at the top
    level, one rank, CUDA RNG as a per-device list) still restores the
    sampler position, running stats and RNG streams - the resumed run
    continues the uninterrupted trajectory."""
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=5)
    store = GraphStore(groups, 'cpu')
    torch.manual_seed(123)
    full = _pair_trainer(store, 'eager')
    ref = _run_trajectory(full, 5)
    torch.manual_seed(123)
    first = _pair_trainer(store, 'eager')
    _run_trajectory(first, 2)
    state = first.state_dict()
    mine = state.pop('ranks')[0]
    state.pop('world_size')
    state.update(mine)                     # the round-3 layout
    path = str(tmp_path / 'legacy.pt')
    torch.save(state, path)
    torch.manual_seed(999)
    resumed = _pair_trainer(store, 'eager', seed_model=7)
    resumed.load(path)
    assert torch.equal(resumed.stats, first.stats)
    assert _run_trajectory(resumed, 3) == ref[2:]


def test_world_size_change_warns(tmp_path):
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=5)
    store = GraphStore(groups, 'cpu')
    torch.manual_seed(123)
    a = _pair_trainer(store, 'eager')
    _run_trajectory(a, 1)
    state = a.state_dict()
    state['ranks'] = state['ranks'] * 2     # as written by 2 ranks
    state['world_size'] = 2
    path = str(tmp_path / 'w2.pt')
    torch.save(state, path)
    b = _pair_trainer(store, 'eager')
    with pytest.warns(UserWarning, match='NOT restored'):
        b.load(path)
    assert float(b.stats.abs().sum()) == 0.0


def test_kg_trainer_checkpoint_keeps_skipped_count(tmp_path):
    """KGTrainer's non-finite skipped-step counter survives a
    save / load."""
    from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair
    from deep_graph_matching_consensus_amd.train import KGTrainer
    data = make_kg_pair('zh_en', scale=0.01, feature_dim=16, seed=0)

    def make():
        torch.manual_seed(0)
        model = DGMC(RelCNN(16, 8, 2), RelCNN(4, 4, 2), num_steps=0, k=4)
        return KGTrainer(model, data, lr=1e-3, graph=False)

    a = make()
    a.step()
    data.x1[0, 0] = float('nan')
    a.step()
    data.x1[0, 0] = 0.0
    assert float(a.skipped) == 1.0
    path = str(tmp_path / 'kg.pt')
    a.save(path)
    b = make()
    b.load(path)
    assert float(b.skipped) == 1.0
