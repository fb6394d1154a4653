"""Every remaining ``DGMC_AMD_*`` environment switch is exercised here (or
in the test named next to it in docs/architecture.md): the variable is set
in a fresh process (module-level switches are read at import) or through
``monkeypatch.setenv`` and its effect is checked.  Code-path alternatives
are module attributes, not environment variables (tested by
monkeypatching them, tests/test_hip_kernels.py::
test_dgmc_fp32_headline_widths_vs_reference_mode)."""
import json
import os
import os.path as osp
import socket
import subprocess
import sys

import pytest
import torch

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))


def _py(code, **env):
    e = dict(os.environ)
    e.update(env)
    e['CUDA_VISIBLE_DEVICES'] = ''
    e['HIP_VISIBLE_DEVICES'] = ''
    r = subprocess.run([sys.executable, '-c', code], cwd=ROOT, env=e,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout.strip().splitlines()[-1]


def test_x6_switch_selects_exact_f32():
    code = ('import bench; from deep_graph_matching_consensus_amd.ops '
            'import gemm, slot_gemm; print(gemm.NT_X6, slot_gemm.X6, '
            'bench.gemm_arith("fp32").split(" ")[0])')
    assert _py(code) == 'True True bf16x6'
    assert _py(code, DGMC_AMD_X6='0') == 'False False exact_f32'


def test_dp_preflight_and_in_step_switches():
    code = ('from deep_graph_matching_consensus_amd import train; '
            'print(train.PREFLIGHT, train.IN_STEP_ALLREDUCE)')
    assert _py(code) == 'True True'
    assert _py(code, DGMC_AMD_DP_PREFLIGHT='0',
               DGMC_AMD_IN_STEP_ALLREDUCE='0') == 'False False'


def test_profile_switch():
    code = ('from deep_graph_matching_consensus_amd.runtime import '
            'profiling; print(profiling.enabled())')
    assert _py(code) == 'False'
    assert _py(code, DGMC_AMD_PROFILE='1') == 'True'


def test_diag_switch(monkeypatch):
    from deep_graph_matching_consensus_amd.ops import _backend
    monkeypatch.delenv('DGMC_AMD_DIAG', raising=False)
    assert not _backend.diag_requested()
    monkeypatch.setenv('DGMC_AMD_DIAG', '1')
    assert _backend.diag_requested()


def test_tuned_gemms_switch(monkeypatch):
    from deep_graph_matching_consensus_amd.runtime import tuning
    monkeypatch.setattr(torch.cuda, 'is_available', lambda: True)
    monkeypatch.setattr(tuning, '_STATE', {'path': tuning.TUNED_FILE,
                                           'ok': True})
    monkeypatch.setenv('DGMC_AMD_TUNED_GEMMS', '0')
    assert tuning.use_tuned_gemms() is False
    if osp.exists(tuning.TUNED_FILE):
        monkeypatch.setenv('DGMC_AMD_TUNED_GEMMS', '1')
        assert tuning.use_tuned_gemms() is True    # (the cached load)


@pytest.mark.gpu
def test_allow_fallback_switch(monkeypatch):
    """A GPU tensor without the HIP library raises, unless
    DGMC_AMD_ALLOW_FALLBACK=1 (then the oracle runs)."""
    from deep_graph_matching_consensus_amd.ops import _backend
    monkeypatch.setitem(_backend._STATE, 'hip', False)
    x = torch.ones(4, device='cuda')
    monkeypatch.delenv('DGMC_AMD_ALLOW_FALLBACK', raising=False)
    with pytest.raises(RuntimeError):
        _backend.use_hip(x)
    monkeypatch.setenv('DGMC_AMD_ALLOW_FALLBACK', '1')
    assert _backend.use_hip(x) is False


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_bench_supervise_switch_and_reserve_cus(tmp_path):
    """DGMC_AMD_BENCH_SUPERVISE=0: the launcher's ranks run the benchmark
    themselves (no ``dp_attempts``); DGMC_AMD_RESERVE_CUS is the data-
    parallel CU reserve the JSON reports."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='',
               OMP_NUM_THREADS='1', DGMC_AMD_BENCH_SUPERVISE='0',
               DGMC_AMD_RESERVE_CUS='12')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR',
              'MASTER_PORT', 'DGMC_AMD_BENCH_INJECT'):
        env.pop(k, None)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), osp.join(ROOT, 'bench.py'),
           '--gpus', '2', '--steps', '1', '--warmup', '0', '--batch-size',
           '4', '--graphs-per-category', '2', '--eval-pairs', '0']
    r = subprocess.run(cmd, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert 'dp_attempts' not in out
    assert out['reserved_cus'] == 12 and out['n_gpus'] == 2
