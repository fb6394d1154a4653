"""Pure-PyTorch oracles for every native op (CPU path + test reference).

These follow the reference semantics literally (same math, same op order as
``/root/reference/dgmc/models/dgmc.py`` and the PyG/torch_scatter/
torch_spline_conv call sites it relies on).  The HIP kernels in ``csrc/hip``
are validated against these in fp32.
"""
import torch


# --------------------------------------------------------------------------
# Message passing
# --------------------------------------------------------------------------
def spmm(row, col, val, num_rows, x, self_x=None, self_scale=None,
         bias=None, relu=False, out_dtype=torch.float32):
    xf = x.float()
    out = torch.zeros(num_rows, x.size(1), dtype=torch.float32,
                      device=x.device)
    if col.numel() > 0:
        out.index_add_(0, row.long(), val.view(-1, 1) * xf[col.long()])
    if self_x is not None:
        out = out + self_scale.float() * self_x.float()
    if bias is not None:
        out = out + bias.float()
    if relu:
        out = torch.relu(out)
    return out.to(out_dtype)


def spline_basis(pseudo, kernel_size, is_open_spline, degree=1):
    r"""Open/closed B-spline basis (torch_spline_conv ``spline_basis``).

    Returns ``basis [E, S]`` (fp32) and ``weight_index [E, S]`` (int64) with
    ``S = (degree + 1) ** dim``.
    """
    pseudo = pseudo.view(-1, 1) if pseudo.dim() == 1 else pseudo
    E, dim = pseudo.shape
    S = (degree + 1) ** dim
    device = pseudo.device
    s = torch.arange(S, device=device)
    basis = torch.ones(E, S, dtype=torch.float32, device=device)
    wi = torch.zeros(E, S, dtype=torch.long, device=device)
    offset = 1
    for d in range(dim):
        k_mod = (s // ((degree + 1) ** d)) % (degree + 1)          # [S]
        ks = int(kernel_size[d])
        v = pseudo[:, d].float() * (ks - degree * int(is_open_spline[d]))
        fl = v.floor()
        wi = wi + ((fl.long().view(-1, 1) + k_mod.view(1, -1)) % ks) * offset
        offset *= ks
        v = (v - fl).view(-1, 1)
        basis = basis * _basis_fn(v, k_mod.view(1, -1), degree)
    return basis, wi


def _basis_fn(v, k_mod, degree):
    if degree == 1:
        return 1 - v - k_mod + 2 * v * k_mod
    if degree == 2:
        b0 = 0.5 * v * v - v + 0.5
        b1 = -v * v + v + 0.5
        b2 = 0.5 * v * v
        return torch.where(k_mod == 0, b0, torch.where(k_mod == 1, b1, b2))
    if degree == 3:
        b0 = (1 - v) ** 3 / 6.
        b1 = (3 * v ** 3 - 6 * v ** 2 + 4) / 6.
        b2 = (-3 * v ** 3 + 3 * v ** 2 + 3 * v + 1) / 6.
        b3 = v ** 3 / 6.
        return torch.where(k_mod == 0, b0, torch.where(
            k_mod == 1, b1, torch.where(k_mod == 2, b2, b3)))
    raise ValueError('degree must be 1, 2 or 3')


# --------------------------------------------------------------------------
# Dense correspondence (dgmc.py:15-19, 161-183)
# --------------------------------------------------------------------------
def masked_softmax(src, mask, dim=-1):
    out = src.masked_fill(~mask, float('-inf'))
    out = torch.softmax(out, dim=dim)
    out = out.masked_fill(~mask, 0)
    return out


def masked_sinkhorn(src, mask, num_iters=10, tau=1.0):
    r"""Log-domain Sinkhorn normalisation over the valid entries (opt-in
    extension; the reference only uses row softmax).

    Alternates row and column normalisation of ``exp(src / tau)`` and ends
    with a row normalisation, so every valid row sums to 1 like
    :func:`masked_softmax` while columns are pushed towards 1.  Invalid
    entries are 0; fully masked rows/columns stay 0 (no NaN).
    """
    neg = torch.finfo(src.dtype).min / 4
    log = (src / tau).masked_fill(~mask, neg)
    for _ in range(num_iters):
        log = log - torch.logsumexp(log, dim=-1, keepdim=True)
        log = log.masked_fill(~mask, neg)
        log = log - torch.logsumexp(log, dim=-2, keepdim=True)
        log = log.masked_fill(~mask, neg)
    log = log - torch.logsumexp(log, dim=-1, keepdim=True)
    return log.exp().masked_fill(~mask, 0)


def count_mask(n_s, n_t, N_s, N_t):
    """``[B, N_s, N_t]`` validity mask from per-pair node counts."""
    device = n_s.device
    ms = torch.arange(N_s, device=device).view(1, -1) < n_s.view(-1, 1).long()
    mt = torch.arange(N_t, device=device).view(1, -1) < n_t.view(-1, 1).long()
    return ms.view(-1, N_s, 1) & mt.view(-1, 1, N_t)


def consensus_mlp_dense(o_s, o_t, W1, b1, W2, b2):
    """``MLP(o_s[:, :, None] - o_t[:, None])`` exactly as dgmc.py:178-179."""
    B, N_s, R = o_s.shape
    N_t = o_t.size(1)
    D = o_s.view(B, N_s, 1, R) - o_t.view(B, 1, N_t, R)
    h = torch.relu(torch.nn.functional.linear(D, W1, b1))
    return torch.nn.functional.linear(h, W2, b2).squeeze(-1)


def consensus_mlp_sparse(o_s, o_t_gathered, W1, b1, W2, b2):
    """``MLP(o_s[:, :, None] - o_t[S_idx])`` as dgmc.py:219-223."""
    D = o_s.unsqueeze(2) - o_t_gathered
    h = torch.relu(torch.nn.functional.linear(D, W1, b1))
    return torch.nn.functional.linear(h, W2, b2).squeeze(-1)


def top_k(x_s, x_t, k):
    """Indices of the k largest inner products, best first (dgmc.py:85-94)."""
    S_ij = x_s @ x_t.transpose(-1, -2)
    return S_ij.topk(k, dim=2)[1]
