"""Dense-correspondence ops of the DGMC consensus loop (per graph pair).

Covers ``/root/reference/dgmc/models/dgmc.py:161-183``:

* ``masked_softmax``          - ``dgmc.py:15-19,165,168,181``;
* ``softmax_transport``       - ``S = masked_softmax(S_hat); r_t = S^T r_s``
                                (``dgmc.py:168-171``), fused per pair;
* ``consensus_update``        - ``S_hat + mask * MLP(o_s[i] - o_t[j])``
                                (``dgmc.py:178-179``).

On the GPU the consensus MLP is evaluated in *factored* form: because the
first layer is linear, ``W1 (o_s_i - o_t_j) + b1 = P_i - Q_j`` with
``P = o_s W1^T + b1`` and ``Q = o_t W1^T`` computed per *node* (two small
GEMMs), and a fused HIP kernel evaluates ``relu(P_i - Q_j) . w2 + b2`` per
pair entry in-place.  The reference materialises ``D [B, N_s, N_t, R]``
(25 MiB per step for PascalVOC shapes); the backward recomputes ``relu`` from
``P``/``Q`` instead of storing it.  Masks are derived from per-pair node
counts (nodes of a pair occupy the leading rows of its padded block), so no
``[B, N_s, N_t]`` mask tensor is stored.
"""
import torch
import torch.nn.functional as F

from . import _backend
from . import reference as ref

# Largest padded graph the per-pair HIP kernels handle (LDS-resident tiles).
MAX_PAIR_NODES = 64


def _hip_ok(x, N_s, N_t):
    return _backend.use_hip(x) and max(N_s, N_t) <= MAX_PAIR_NODES


# ---------------------------------------------------------------------------
class _MaskedSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S_hat, n_s, n_t):
        S = _backend.ops().dense_masked_softmax(S_hat.float().contiguous(),
                                                n_s, n_t)
        ctx.save_for_backward(S, n_s, n_t)
        ctx.dtype = S_hat.dtype
        return S

    @staticmethod
    def backward(ctx, grad):
        S, n_s, n_t = ctx.saved_tensors
        g = _backend.ops().dense_masked_softmax_bwd(
            S, grad.float().contiguous(), n_s, n_t)
        return g.to(ctx.dtype), None, None


def masked_softmax(S_hat, n_s, n_t):
    """Row softmax over valid targets; rows/cols beyond the counts -> 0."""
    B, N_s, N_t = S_hat.shape
    if _hip_ok(S_hat, N_s, N_t):
        return _MaskedSoftmax.apply(S_hat, n_s, n_t)
    mask = ref.count_mask(n_s, n_t, N_s, N_t)
    return ref.masked_softmax(S_hat.float(), mask)


# ---------------------------------------------------------------------------
class _SoftmaxTransport(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S_hat, r_s, n_s, n_t):
        S, r_t = _backend.ops().dense_softmax_transport(
            S_hat.float().contiguous(), r_s.float().contiguous(), n_s, n_t)
        ctx.save_for_backward(S, r_s, n_s, n_t)
        ctx.dtype = S_hat.dtype
        return r_t

    @staticmethod
    def backward(ctx, grad):
        S, r_s, n_s, n_t = ctx.saved_tensors
        g = _backend.ops().dense_softmax_transport_bwd(
            S, r_s.float().contiguous(), grad.float().contiguous(), n_s, n_t)
        return g.to(ctx.dtype), None, None, None


def softmax_transport(S_hat, r_s, n_s, n_t):
    r"""``masked_softmax(S_hat)^T @ r_s`` -> ``r_t [B, N_t, R]``.

    ``r_s`` is a non-differentiable random indicator (as in the reference);
    gradients flow into ``S_hat``.
    """
    B, N_s, N_t = S_hat.shape
    if _hip_ok(S_hat, N_s, N_t):
        return _SoftmaxTransport.apply(S_hat, r_s, n_s, n_t)
    mask = ref.count_mask(n_s, n_t, N_s, N_t)
    S = ref.masked_softmax(S_hat.float(), mask)
    return S.transpose(-1, -2) @ r_s.float()


# ---------------------------------------------------------------------------
class _ConsensusUpdate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S_hat, P, Q, w2, b2, n_s, n_t):
        out = _backend.ops().dense_consensus(
            S_hat.float().contiguous(), P.float().contiguous(),
            Q.float().contiguous(), w2.float().contiguous().view(-1),
            b2.float().contiguous().view(-1), n_s, n_t)
        ctx.save_for_backward(P, Q, w2, n_s, n_t)
        ctx.dtypes = (S_hat.dtype, P.dtype, Q.dtype, w2.dtype, b2.dtype)
        ctx.b2_shape = b2.shape
        return out

    @staticmethod
    def backward(ctx, grad):
        P, Q, w2, n_s, n_t = ctx.saved_tensors
        g = grad.float().contiguous()
        dP, dQ, dw2_part, db2_part = _backend.ops().dense_consensus_bwd(
            g, P.float().contiguous(), Q.float().contiguous(),
            w2.float().contiguous().view(-1), n_s, n_t)
        dw2 = dw2_part.sum(0).view_as(w2)
        db2 = db2_part.sum().view(ctx.b2_shape)
        dt = ctx.dtypes
        return (grad.to(dt[0]), dP.to(dt[1]), dQ.to(dt[2]), dw2.to(dt[3]),
                db2.to(dt[4]), None, None)


def consensus_update(S_hat, o_s, o_t, mlp, n_s, n_t):
    r"""``S_hat + mask * mlp(o_s[:, :, None] - o_t[:, None])``.

    ``mlp`` must be ``Seq(Lin(R, R), ReLU, Lin(R, 1))`` (``dgmc.py:74-78``).
    """
    lin1, lin2 = mlp[0], mlp[2]
    B, N_s, N_t = S_hat.shape
    if _hip_ok(S_hat, N_s, N_t):
        P = F.linear(o_s, lin1.weight, lin1.bias)
        Q = F.linear(o_t, lin1.weight)
        return _ConsensusUpdate.apply(S_hat, P, Q, lin2.weight, lin2.bias,
                                      n_s, n_t)
    mask = ref.count_mask(n_s, n_t, N_s, N_t)
    upd = ref.consensus_mlp_dense(o_s, o_t, lin1.weight, lin1.bias,
                                  lin2.weight, lin2.bias)
    return S_hat + upd.masked_fill(~mask, 0)
