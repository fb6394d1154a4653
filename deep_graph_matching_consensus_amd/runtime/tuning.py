"""Tuned hipBLASLt / rocBLAS solutions for the encoder GEMMs.

The plain library GEMMs of the step (psi_1's SplineConv projections
``[N, 1024] x [1024, 26 * 256]`` and ``[N, 256] x [256, 26 * 256]``, their
input gradients, psi_2's Linear layers) go through PyTorch's TunableOp, which
dispatches each GEMM shape to a solution measured fastest on MI355X instead
of hipBLASLt's heuristic pick.  Measured on the PascalVOC-shaped flagship
(``gpurun_out/tune``): the first-layer projection 185 -> 120 us, the
second-layer input gradient 86 -> 45 us per step.

The results file (``tuned/gemm_gfx950.csv``) is produced on a GPU box by
``tools/tune_gemms.py`` for every static-batch capacity the benchmark uses
at 1/2/4/8 ranks, and only READ at run time: tuning stays disabled, so no
GEMM is ever benchmarked inside a timed step or a hipGraph capture, and
shapes missing from the file fall back to the default heuristic.  TunableOp
validates the file against the PyTorch / HIP / hipBLASLt / rocBLAS versions
and the GPU architecture, so a file from another stack is ignored.
``DGMC_AMD_TUNED_GEMMS=0`` disables it.
"""
import contextlib
import os
import os.path as osp

import torch

TUNED_FILE = osp.join(osp.dirname(osp.abspath(__file__)), 'tuned',
                      'gemm_gfx950.csv')
_STATE = {}


def use_tuned_gemms(path=None):
    """Load the tuned solutions in ``path`` (default: the shipped file) into
    TunableOp's result table.  TunableOp itself is only switched on inside
    :func:`tuned_gemms` scopes (the trainers' steps), so the process-wide
    setting outside them is left as the caller had it.  Returns True if the
    file was loaded."""
    if os.environ.get('DGMC_AMD_TUNED_GEMMS', '1') != '1':
        return False
    if not torch.cuda.is_available():
        return False
    path = path or TUNED_FILE
    if not osp.exists(path):
        return False
    if _STATE.get('path') == path:
        return _STATE['ok']
    tunable = torch.cuda.tunable
    prev = (tunable.is_enabled(), tunable.tuning_is_enabled(),
            tunable.get_filename())
    tunable.enable(True)
    tunable.tuning_enable(False)
    ok = bool(tunable.read_file(path))
    tunable.enable(prev[0])
    tunable.tuning_enable(prev[1])
    tunable.set_filename(prev[2])
    _STATE.update(path=path, ok=ok)
    return ok


@contextlib.contextmanager
def tuned_gemms(active=True):
    """Dispatch the GEMMs issued inside the scope through the loaded tuned
    solutions (read-only: tuning stays off, nothing is written), restoring
    the previous TunableOp settings on exit."""
    if not (active and _STATE.get('ok')):
        yield
        return
    tunable = torch.cuda.tunable
    prev = (tunable.is_enabled(), tunable.tuning_is_enabled())
    tunable.enable(True)
    tunable.tuning_enable(False)
    try:
        yield
    finally:
        tunable.enable(prev[0])
        tunable.tuning_enable(prev[1])


def start_tuning(out_path, max_duration_ms=15):
    """Enable online tuning: every new GEMM shape is benchmarked once and
    its best solution recorded (``tools/tune_gemms.py``)."""
    tunable = torch.cuda.tunable
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_max_tuning_duration(max_duration_ms)
    tunable.set_filename(out_path)
    if osp.exists(out_path):
        tunable.read_file(out_path)


def write_results(out_path):
    """Write the validators and every result of this process to
    ``out_path`` in TunableOp's CSV format (rows sorted, so files from
    several runs merge with ``sort -u``)."""
    tunable = torch.cuda.tunable
    lines = ['Validator,{},{}'.format(k, v)
             for k, v in tunable.get_validators()]
    rows = sorted('{},{},{},{}'.format(op, params, sol, t)
                  for op, params, sol, t in tunable.get_results())
    with open(out_path, 'w') as f:
        f.write('\n'.join(lines + rows) + '\n')
    return len(rows)
