"""Multi-tensor Adam on the HIP path (``csrc/hip/optim.hip``).

``torch.optim.Adam`` stays the optimizer object - its ``state_dict`` /
``load_state_dict`` and the checkpoint schema are unchanged (``step``,
``exp_avg``, ``exp_avg_sq`` per parameter) - but the update itself is ONE
launch over a pointer table of all parameters instead of torch's fused
``multi_tensor_apply`` (122 us -> see docs/performance.md for the PascalVOC
flagship's 9.5 M parameters).

Every parameter keeps its OWN ``state['step']`` (an fp32 device scalar, as
torch's capturable Adam keeps it): ``adam_step_inc`` bumps each counter on
the device unless ``found_inf`` is set and the update kernel reads each
parameter's own counter for its bias correction, so the update is
capturable, skips itself on the device, and a parameter that gets its first
gradient late (or a checkpoint with per-parameter steps) follows torch's
per-parameter semantics exactly.  Counters are never shared between
parameters, so a state dict saved here resumes correctly under
``torch.optim.Adam`` and vice versa (``tests/test_checkpoint.py``).
"""

import torch

from ..ops import _backend

ENABLED = True                # (tests compare against torch's Adam)


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


def _device_step(st, p):
    """``st['step']`` as this parameter's own fp32 device scalar (a torch
    checkpoint loads it as a CPU tensor; converted once, then kept)."""
    step = st.get('step')
    if step is None:
        step = torch.zeros((), dtype=torch.float32, device=p.device)
    elif not (torch.is_tensor(step) and step.device == p.device and
              step.dtype == torch.float32 and step.dim() == 0):
        step = torch.as_tensor(step, dtype=torch.float32).reshape(()) \
            .to(p.device).clone()
    st['step'] = step
    return step


def hip_adam_step(optimizer, found_inf=None, flags=None, skips=None):
    """One Adam step of ``optimizer`` (see module docstring).  ``flags``:
    per-block non-finite flags of the gradients (``pack_grads``) folded into
    ``found_inf`` (and ``skips += 1`` on a skipped step) by the step-counter
    kernel."""
    group = optimizer.param_groups[0]
    params = [p for p in group['params'] if p.grad is not None]
    if not params:
        return
    state = optimizer.state
    steps = []
    for p in params:
        st = state[p]
        if 'exp_avg' not in st:
            st['exp_avg'] = torch.zeros_like(
                p, memory_format=torch.preserve_format)
            st['exp_avg_sq'] = torch.zeros_like(
                p, memory_format=torch.preserve_format)
        steps.append(_device_step(st, p))
    b1, b2 = group['betas']
    if flags is not None and found_inf is None:
        # The flags are folded into found_inf by the first parameter chunk
        # and every later chunk reads found_inf: it must exist.
        found_inf = torch.zeros((), dtype=torch.float32,
                                device=params[0].device)
    ops = _backend.ops()
    ops.adam_step_inc(steps, found_inf, flags, skips)
    ops.adam_multi(params, [p.grad for p in params],
                   [state[p]['exp_avg'] for p in params],
                   [state[p]['exp_avg_sq'] for p in params], steps, found_inf,
                   float(group['lr']), float(b1), float(b2),
                   float(group['eps']), float(group['weight_decay']))
