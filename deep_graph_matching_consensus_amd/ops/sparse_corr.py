"""Sparse (top-k) correspondence ops (``/root/reference/dgmc/models/dgmc.py:184-244``).

* :func:`top_k`            - candidate search ``argtopk_j <h_s[b,i], h_t[b,j]>``
  (``dgmc.py:85-94``; KeOps ``argKmin`` in the reference).  On the GPU a fused
  HIP kernel streams ``h_t`` tiles through LDS, computes dot tiles with MFMA
  and keeps a per-row register top-k, so the ``N_s x N_t`` score matrix is
  never materialised.
* :func:`gather_dot`       - ``S_hat[b,i,c] = <h_s[b,i], h_t[b, S_idx[b,i,c]]>``
  (``dgmc.py:197-201``).
* :func:`sparse_transport` - ``r_t = scatter_add(S * r_s, S_idx)``
  (``dgmc.py:209-212``), deterministic (segment sums over a transposed index
  built once per forward, no atomics).
* :func:`consensus_update` - ``S_hat + MLP(o_s[:, :, None] - o_t[S_idx])``
  (``dgmc.py:219-223``; factored ``relu(P_i - Q_idx) . w2 + b2`` on GPU).
"""
import torch
import torch.nn.functional as F

from . import _backend
from . import reference as ref


def top_k(h_s, h_t, k):
    """``[B, N_s, k]`` int64 indices of the k best targets per source row."""
    B, N_s, C = h_s.shape
    N_t = h_t.size(1)
    if _backend.use_hip(h_s) and k <= 64 and C % 4 == 0:
        return _backend.ops().topk_dot(h_s.float().contiguous(),
                                       h_t.float().contiguous(), int(k))
    return ref.top_k(h_s, h_t, k)


# ---------------------------------------------------------------------------
def gather_dot(h_s, h_t, S_idx):
    """``S_hat [B, N_s, k]`` (autograd through both embeddings)."""
    B, N_s, C = h_s.shape
    k = S_idx.size(-1)
    idx = S_idx.reshape(B, N_s * k, 1).expand(-1, -1, C)
    tmp_t = torch.gather(h_t, 1, idx).view(B, N_s, k, C)
    return (h_s.unsqueeze(2) * tmp_t).sum(dim=-1)


# ---------------------------------------------------------------------------
def sparse_transport(S, r_s, S_idx, N_t):
    """``r_t[b, j] = sum_{(i,c): S_idx[b,i,c] = j} S[b,i,c] * r_s[b,i]``."""
    B, N_s, k = S.shape
    R = r_s.size(-1)
    tmp = (r_s.unsqueeze(2) * S.unsqueeze(-1)).reshape(B, N_s * k, R)
    idx = S_idx.reshape(B, N_s * k, 1).expand(-1, -1, R)
    out = torch.zeros(B, N_t, R, dtype=tmp.dtype, device=tmp.device)
    return out.scatter_add(1, idx, tmp)


# ---------------------------------------------------------------------------
def consensus_update(S_hat, o_s, o_t, S_idx, mlp):
    B, N_s, k = S_hat.shape
    R = o_s.size(-1)
    lin1, lin2 = mlp[0], mlp[2]
    idx = S_idx.reshape(B, N_s * k, 1).expand(-1, -1, R)
    if _backend.use_hip(S_hat):
        P = F.linear(o_s, lin1.weight, lin1.bias)            # [B, N_s, R]
        Q = F.linear(o_t, lin1.weight)                        # [B, N_t, R]
        Qg = torch.gather(Q, 1, idx).view(B, N_s, k, R)
        h = torch.relu(P.unsqueeze(2) - Qg)
        return S_hat + F.linear(h, lin2.weight, lin2.bias).squeeze(-1)
    o_t_g = torch.gather(o_t, 1, idx).view(B, N_s, k, R)
    return S_hat + ref.consensus_mlp_sparse(o_s, o_t_g, lin1.weight,
                                            lin1.bias, lin2.weight, lin2.bias)
