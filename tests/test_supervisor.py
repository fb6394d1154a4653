"""Multi-GPU first-run insurance (``bench.py`` supervisor), on CPU ranks.

Under ``torch.distributed.run`` every bench rank supervises a child that
does the GPU work; a failing, hanging or silent attempt makes every rank
move to the next data-parallel mode together (captured -> flat -> static),
and rank 0 prints ONE JSON line carrying ``dp_attempts``.  Failures are
injected with ``DGMC_AMD_BENCH_INJECT=<kind>:<attempt>:<rank>``.

Also here: the captured-collective sequence check
(``PairTrainer._check_collective_sequence``) over a gloo group, and the
recorded all-reduce sequence of real in-step steps (identical across steps
and ranks, as replaying different size-bucket graphs requires).
"""
import json
import os
import os.path as osp
import socket
import subprocess
import sys
import time
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
BENCH = osp.join(ROOT, 'bench.py')
SMALL = ['--steps', '1', '--warmup', '0', '--batch-size', '4',
         '--graphs-per-category', '2', '--eval-pairs', '0', '--mode', 'graph']

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env(**extra):
    env = dict(os.environ)
    env['CUDA_VISIBLE_DEVICES'] = ''
    env['HIP_VISIBLE_DEVICES'] = ''
    env['OMP_NUM_THREADS'] = '1'
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR',
              'MASTER_PORT', 'DGMC_AMD_BENCH_INJECT'):
        env.pop(k, None)
    env.update(extra)
    return env


def _run(env, timeout=600):
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, BENCH, '--gpus', '2'] + SMALL,
                       env=env, capture_output=True, text=True,
                       timeout=timeout)
    wall = time.monotonic() - t0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, (r.stdout, r.stderr[-3000:])
    return r, json.loads(lines[0]), wall


def test_ladder_and_budgets():
    assert [m for m, _ in bench.dp_ladder([])] == \
        ['graph-captured', 'graph-flat', 'static-flat']
    assert [m for m, _ in bench.dp_ladder(['--dp-mode', 'flat'])] == \
        ['graph-flat', 'static-flat']
    assert [m for m, _ in bench.dp_ladder(['--mode', 'static'])] == \
        ['static-flat']
    assert [m for m, _ in bench.dp_ladder(['--mode', 'eager'])] == ['eager']
    # three attempts fit inside the driver's 600 s run limit
    b0 = bench.attempt_budgets(560, 3, 0, 0)
    b1 = bench.attempt_budgets(560, 3, b0, 1)
    b2 = bench.attempt_budgets(560, 3, b0 + b1, 2)
    assert b0 + b1 + b2 <= 560 + 1e-9
    assert min(b0, b1, b2) >= 60


def test_clean_run_single_attempt():
    r, out, _ = _run(_env())
    assert r.returncode == 0, r.stderr[-3000:]
    assert [a['mode'] for a in out['dp_attempts']] == ['graph-captured']
    assert out['dp_attempts'][0]['rc'] == [0, 0]
    assert out['params_in_sync'] and out['value'] > 0


@pytest.mark.parametrize('kind', ['crash', 'nojson'])
def test_failed_first_attempt_falls_back(kind):
    rank = '1' if kind == 'crash' else '0'
    r, out, _ = _run(_env(DGMC_AMD_BENCH_INJECT='{}:0:{}'.format(kind,
                                                                  rank)))
    assert r.returncode == 0, r.stderr[-3000:]
    att = out['dp_attempts']
    assert [a['mode'] for a in att] == ['graph-captured', 'graph-flat']
    assert att[1]['rc'] == [0, 0] and att[1]['reason'] == ['ok']
    if kind == 'crash':
        assert 1 in att[0]['rc']
    else:
        assert 'no JSON line' in att[0]['reason']
    assert out['n_gpus'] == 2 and out['value'] > 0
    assert out['params_in_sync']
    assert out['dp_mode'] == 'flat-after-step'


def test_hung_attempt_is_killed_within_budget():
    env = _env(DGMC_AMD_BENCH_INJECT='hang:0:1',
               DGMC_AMD_BENCH_ATTEMPT_S='40', DGMC_AMD_DIST_TIMEOUT='20')
    r, out, wall = _run(env)
    assert r.returncode == 0, r.stderr[-3000:]
    att = out['dp_attempts']
    assert len(att) == 2
    assert any('timeout' in why for why in att[0]['reason'])
    assert att[0]['wall_s'] <= 40 + 45     # budget + kill grace
    assert att[1]['reason'] == ['ok']
    assert wall < 300
    assert out['value'] > 0 and out['params_in_sync']


def test_every_attempt_failing_still_prints_one_line():
    env = _env(DGMC_AMD_BENCH_INJECT='crash:0:0')
    # only one rung (static), and it fails
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, BENCH, '--gpus', '2'] + SMALL[:-2] +
                       ['--mode', 'static'], env=env, capture_output=True,
                       text=True, timeout=600)
    assert time.monotonic() - t0 < 300
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out['value'] is None and out['dp_attempts'][0]['mode'] == \
        'static-flat'


# ---------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _seq_worker(rank, world, port, case, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from deep_graph_matching_consensus_amd.train import PairTrainer
    fake = types.SimpleNamespace(device=torch.device('cpu'), world=world,
                                 dp_checks={})
    seq = [(0, 10), (10, 30), (30, 31)]
    runs = [[seq, seq, seq], [seq, seq, seq]]
    if case == 'bucket' and rank == 1:
        runs[1][-1] = [(0, 10), (10, 31)]
    if case == 'rank' and rank == 1:
        alt = [(0, 12), (12, 30), (30, 31)]
        runs = [[alt] * 3, [alt] * 3]
    try:
        PairTrainer._check_collective_sequence(fake, runs)
        out[rank] = ('ok', fake.dp_checks)
    except RuntimeError as e:
        out[rank] = ('raised', str(e))
    dist.destroy_process_group()


@pytest.mark.parametrize('case', ['same', 'bucket', 'rank'])
def test_collective_sequence_check(case):
    world = 2
    ctx = mp.get_context('spawn')
    out = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_seq_worker, args=(r, world, port, case, out))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    if case == 'same':
        for r in range(world):
            assert out[r][0] == 'ok'
            assert out[r][1]['collective_sequence'] == 'identical'
            assert out[r][1]['collectives_per_step'] == 3
    else:
        # every rank raises together (no rank replays alone)
        assert all(out[r][0] == 'raised' for r in range(world)), dict(out)


def _steps_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.train import PairTrainer
    torch.manual_seed(0)
    groups = make_keypoint_datasets(graphs=6, feature_dim=32, seed=3)
    store = GraphStore(groups, 'cpu')
    model = DGMC(SplineCNN(32, 32, 2, 2, cat=False),
                 SplineCNN(16, 16, 2, 2, cat=True), num_steps=2)
    trainer = PairTrainer(model, store, 8, mode='static',
                          bucket_bytes=16 << 10)
    assert trainer.reducer.in_step
    trainer.reducer.seq_log = []
    for _ in range(3):
        trainer.step()
    out[rank] = trainer.reducer.seq_log
    dist.destroy_process_group()


def test_in_step_sequence_is_identical_across_steps_and_ranks():
    """The real hook-driven bucket all-reduces of in-step DP steps: the
    (offset, length) list is the same at every step (different batches)
    and on every rank, and covers the whole flat gradient buffer."""
    world = 2
    ctx = mp.get_context('spawn')
    out = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_steps_worker, args=(r, world, port, out))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    runs0, runs1 = out[0], out[1]
    assert len(runs0) == 3 and runs0 == runs1
    assert runs0[0] == runs0[1] == runs0[2]
    assert len(runs0[0]) > 2
    covered = sorted(runs0[0])
    assert covered[0][0] == 0
    for (a, b), (c, d) in zip(covered, covered[1:]):
        assert b <= c
