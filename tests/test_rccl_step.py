"""Multi-GPU launch contract (CPU) and the captured RCCL step (GPU).

* ``bench.py --gpus 2`` started as a plain process launches two ranks
  itself (``torch.distributed.run`` child, gloo on CPU) and reports
  ``n_gpus: 2``; under a launcher whose ``WORLD_SIZE`` disagrees with
  ``--gpus`` it exits non-zero.
* GPU: an RCCL process group of ONE rank drives ``PairTrainer`` down the
  real in-step data-parallel path (hooks, ``_pack_bucket``, captured
  ``all_reduce`` + ``work.wait()``) in graph mode; 6 replayed steps are
  bit-identical to the single-process trainer
  (``tests/rccl_world1_worker.py``).
"""
import json
import os
import os.path as osp
import subprocess
import sys

import pytest

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
BENCH = osp.join(ROOT, 'bench.py')
SMALL = ['--steps', '1', '--warmup', '0', '--batch-size', '4',
         '--graphs-per-category', '2', '--eval-pairs', '0']


def _env():
    env = dict(os.environ)
    env['CUDA_VISIBLE_DEVICES'] = ''        # CPU ranks (gloo)
    env['HIP_VISIBLE_DEVICES'] = ''
    env['OMP_NUM_THREADS'] = '1'
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR',
              'MASTER_PORT'):
        env.pop(k, None)
    return env


def test_bench_gpus_2_launches_two_ranks():
    r = subprocess.run([sys.executable, BENCH, '--gpus', '2'] + SMALL,
                       env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout     # rank 0 prints ONE line
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2
    assert out['config']['parallelism'] == 'dp2'
    assert out['config']['global_batch'] == 2 * 4


def test_bench_rejects_world_size_mismatch():
    env = _env()
    env.update(WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, BENCH, '--gpus', '2'] + SMALL,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert 'WORLD_SIZE=1' in r.stderr


@pytest.mark.gpu
def test_rccl_world1_captured_step_bit_identical(tmp_path):
    out = tmp_path / 'rccl.json'
    # Both runs produce psi_1 layer 0's weight gradient in pieces (the RCCL
    # run all-reduces each piece from inside the captured backward).
    env = dict(os.environ, DGMC_AMD_WGRAD_PIECES_ALWAYS='1')
    r = subprocess.run([sys.executable, '-u',
                        osp.join(ROOT, 'tests', 'rccl_world1_worker.py'),
                        '--steps', '6', '--json', str(out)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert out.exists(), r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(out.read_text())
    assert res['rccl']['distributed'] and res['rccl']['in_step']
    assert res['rccl']['buckets'] > 4
    assert res['equal'], res
    assert r.returncode == 0, r.stderr[-4000:]
