"""Multi-tensor Adam on the HIP path (``csrc/hip/optim.hip``).

``torch.optim.Adam`` stays the optimizer object - its ``state_dict`` /
``load_state_dict`` and the checkpoint schema are unchanged (``step``,
``exp_avg``, ``exp_avg_sq`` per parameter) - but the update itself is ONE
launch over a pointer table of all parameters instead of torch's fused
``multi_tensor_apply`` (122 us -> see docs/performance.md for the PascalVOC
flagship's 9.5 M parameters).  The step counter is a single fp32 device
tensor shared by every parameter's state (re-shared after a load), read by
the kernel after ``adam_step_inc`` bumps it unless ``found_inf`` is set, so
the update is capturable and skips itself on the device.
"""
import os

import torch

from ..ops import _backend

ENABLED = os.environ.get('DGMC_AMD_HIP_ADAM', '1') == '1'


def supported(optimizer):
    if not (ENABLED and isinstance(optimizer, torch.optim.Adam) and
            len(optimizer.param_groups) == 1):
        return False
    g = optimizer.param_groups[0]
    ps = g['params']
    return (not g['amsgrad'] and not g.get('maximize', False) and
            not g.get('decoupled_weight_decay', False) and
            len(ps) > 0 and all(p.is_cuda and p.dtype == torch.float32
                                for p in ps) and _backend.use_hip(ps[0]))


def hip_adam_step(optimizer, found_inf=None):
    """One Adam step of ``optimizer`` (see module docstring)."""
    group = optimizer.param_groups[0]
    params = [p for p in group['params'] if p.grad is not None]
    if not params:
        return
    state = optimizer.state
    first = state[params[0]]
    if 'step' not in first:
        first['step'] = torch.zeros((), dtype=torch.float32,
                                    device=params[0].device)
    step = first['step']
    if step.device != params[0].device or step.dtype != torch.float32:
        step = first['step'] = step.to(params[0].device, torch.float32)
    for p in params:
        st = state[p]
        if 'exp_avg' not in st:
            st['exp_avg'] = torch.zeros_like(
                p, memory_format=torch.preserve_format)
            st['exp_avg_sq'] = torch.zeros_like(
                p, memory_format=torch.preserve_format)
        st['step'] = step                      # one shared counter
    b1, b2 = group['betas']
    ops = _backend.ops()
    ops.adam_step_inc(step, found_inf)
    ops.adam_multi(params, [p.grad for p in params],
                   [state[p]['exp_avg'] for p in params],
                   [state[p]['exp_avg_sq'] for p in params], step, found_inf,
                   float(group['lr']), float(b1), float(b2),
                   float(group['eps']), float(group['weight_decay']))
