"""Dense-correspondence ops of the DGMC consensus loop (per graph pair).

Covers ``/root/reference/dgmc/models/dgmc.py:161-183``:

* ``masked_softmax``     - ``dgmc.py:15-19,165,168,181``;
* ``softmax_transport``  - ``S = masked_softmax(S_hat); r_t = S^T r_s``
                           (``dgmc.py:168-171``), fused per pair;
* ``consensus_update``   - ``S_hat + mask * MLP(o_s[i] - o_t[j])``
                           (``dgmc.py:178-179``).

Node-level tensors (random indicators ``r_s``/``r_t`` and the consensus
embeddings ``o_s``/``o_t``) stay in the *packed* ``[sum N, R]`` layout the
encoders produce; the per-pair kernels address them through int32 row offsets
``ptr`` (one workgroup per pair), so the reference's ``to_sparse``/
``to_dense`` round trips (``dgmc.py:173,176``) disappear.

The consensus MLP is evaluated in *factored* form on the GPU: the first layer
is linear, so ``W1 (o_s_i - o_t_j) + b1 = P_i - Q_j + b1`` with
``[P; Q] = [o_s; o_t] W1^T`` computed by ONE node-level GEMM (bf16 under
autocast) and the fused kernel evaluates ``relu(P_i - Q_j + b1) . w2 + b2``
per pair entry.  The reference materialises ``D [B, N_s, N_t, R]`` (25 MiB
per step for PascalVOC shapes); the backward recomputes the ReLU from
``P``/``Q``.  Masks come from per-pair node counts.
"""

import torch

from . import _backend
from . import reference as ref
from .gemm import _col_sum, lowp_weight_t, mixed_matmul
from ..runtime import loopgrad

# Largest padded graph the per-pair HIP kernels handle (LDS-resident tiles).
MAX_PAIR_NODES = 64
# Consensus update of step l fused with the softmax transport of step l + 1
# (one per-pair kernel each way); FUSE_STEPS = False keeps them apart (tests).
FUSE_STEPS = True


def _hip_ok(x, N_s, N_t):
    return _backend.use_hip(x) and max(N_s, N_t) <= MAX_PAIR_NODES


def _count_mask(lay_s, lay_t):
    return ref.count_mask(lay_s.counts, lay_t.counts, lay_s.N, lay_t.N)


# ---------------------------------------------------------------------------
class _PairScores(torch.autograd.Function):
    """``S_hat = h_s h_t^T`` per pair straight from the packed joint encoder
    output (csrc/hip/pair_scores.hip); the backward returns the joint
    gradient (padding rows zero) - no dense layouts, no slice backward."""

    @staticmethod
    def forward(ctx, h, t_off, ptr_s, ptr_t, N_s, N_t, two):
        S = _backend.ops().pair_scores(h, t_off, ptr_s, ptr_t, N_s, N_t)
        ctx.save_for_backward(h, ptr_s, ptr_t)
        ctx.t_off = t_off
        ctx.set_materialize_grads(False)
        if two:
            # Two handles on S_hat for its two consumers (objective / loop):
            # their gradients meet in the backward kernel, not in an
            # autograd add.
            return S, S.view_as(S)
        return S

    @staticmethod
    def backward(ctx, grad, grad2=None):
        h, ptr_s, ptr_t = ctx.saved_tensors
        if grad is None:
            grad, grad2 = grad2, None
        if grad is None:
            return (None, ) * 7
        dh = _backend.ops().pair_scores_bwd(
            grad.float().contiguous(), h, ctx.t_off, ptr_s, ptr_t,
            None if grad2 is None else grad2.float().contiguous())
        return dh, None, None, None, None, None, None


def pair_scores_supported(h, lay_s, lay_t):
    # (mirrors pair_scores_bwd's contract: C % 4, 16-byte aligned rows)
    return (_hip_ok(h, lay_s.N, lay_t.N) and h.dim() == 2 and
            h.is_contiguous() and h.dtype in (torch.bfloat16, torch.float32)
            and h.size(1) <= 256 and h.size(1) % 4 == 0 and
            h.data_ptr() % 16 == 0 and lay_s.N >= 1 and lay_t.N >= 1)


def pair_scores(h, t_off, lay_s, lay_t, two=False):
    r"""Dense initial scores ``[B, N_s, N_t]`` (fp32) of the joint encoder
    output ``h = [h_s; h_t]`` (target rows from ``t_off``): entry
    ``(b, i, j) = <h_s[ptr_s[b] + i], h_t[ptr_t[b] + j]>``, zero outside
    each pair's ``n_s x n_t`` block (``dgmc.py:154-163``).  ``two``: return
    two aliases (one per consumer; gradients summed in the backward
    kernel)."""
    return _PairScores.apply(h, int(t_off), lay_s.ptr, lay_t.ptr, lay_s.N,
                             lay_t.N, bool(two))


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


def masked_softmax(S_hat, lay_s, lay_t):
    """Row softmax over valid targets; rows/cols beyond the counts -> 0."""
    B, N_s, N_t = S_hat.shape
    if _hip_ok(S_hat, N_s, N_t):
        return _MaskedSoftmax.apply(S_hat, lay_s.counts, lay_t.counts)
    return ref.masked_softmax(S_hat, _count_mask(lay_s, lay_t))


class _MaskedSoftmaxPacked(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S_hat, index, n_s, n_t):
        S = _backend.ops().masked_softmax_packed(S_hat.float().contiguous(),
                                                 index, n_s, n_t)
        ctx.save_for_backward(S, index)
        ctx.shape, ctx.dtype = tuple(S_hat.shape), S_hat.dtype
        return S

    @staticmethod
    def backward(ctx, grad):
        S, index = ctx.saved_tensors
        B, N_s, _ = ctx.shape
        g = _backend.ops().masked_softmax_packed_bwd(
            S, grad.float().contiguous(), index, B, N_s)
        return g.to(ctx.dtype), None, None, None


def masked_softmax_packed(S_hat, lay_s, lay_t):
    r"""``lay_s.to_sparse(masked_softmax(S_hat))`` - the packed
    ``[sum N_s, N_t]`` correspondence output (``dgmc.py:165,181``) in one
    kernel on the GPU (its backward is a row scatter, no ``index_add``)."""
    index = getattr(lay_s, 'index', None)
    if (_backend.use_hip(S_hat) and torch.is_tensor(index) and
            index.dtype == torch.long and index.is_cuda):
        return _MaskedSoftmaxPacked.apply(S_hat, index.contiguous(),
                                          lay_s.counts, lay_t.counts)
    return lay_s.to_sparse(masked_softmax(S_hat, lay_s, lay_t))


class _SoftmaxNLL(torch.autograd.Function):
    """Masked row softmax + NLL (+ Hits@1) on the dense scores in one fused
    kernel (csrc/hip/loss.hip::softmax_nll_*) for one or two score tiles
    (the objective's ``S_L`` and ``S_0`` in the same launch);
    ``aux = [count, correct, count of the second tile]``."""

    @staticmethod
    def forward(ctx, S_hat, S_hat2, ptr_s, n_t, y, mask, eps, stats):
        S_hat = S_hat.float().contiguous()
        if S_hat2 is not None:
            S_hat2 = S_hat2.float().contiguous()
        loss, aux = _backend.ops().softmax_nll_fwd(S_hat, S_hat2, ptr_s, n_t,
                                                   y, mask, eps, stats)
        ctx.save_for_backward(S_hat, S_hat2, ptr_s, n_t, y, mask, aux)
        ctx.eps = eps
        ctx.mark_non_differentiable(aux)
        ctx.set_materialize_grads(False)
        return loss, aux

    @staticmethod
    def backward(ctx, grad, grad_aux):
        if grad is None:
            return (None, ) * 8
        S_hat, S_hat2, ptr_s, n_t, y, mask, aux = ctx.saved_tensors
        dS, dS2 = _backend.ops().softmax_nll_bwd(
            grad.float().reshape(1), S_hat, S_hat2, ptr_s, n_t, y, mask, aux,
            ctx.eps)
        return (dS, dS2 if S_hat2 is not None else None) + (None, ) * 6


def softmax_nll_supported(S_hat, lay_s):
    return (_backend.use_hip(S_hat) and S_hat.dim() == 3 and
            torch.is_tensor(getattr(lay_s, 'ptr', None)) and
            lay_s.ptr.is_cuda)


def softmax_nll(S_hat, lay_s, lay_t, y_col, mask, eps, S_hat2=None,
                stats=None):
    r"""``(loss, aux)``: mean of ``-log(masked_softmax(S_hat)[r, y_col[r]] +
    eps)`` over the packed source rows ``r`` (weights ``mask``) - plus the
    same term of ``S_hat2`` when given - and ``aux = [count, correct top-1,
    count]`` (``DGMC.loss`` / ``DGMC.correct`` of
    ``masked_softmax_packed(S_hat)`` with ``y = (arange, y_col)``).
    ``stats`` (fp64 device tensor, optional) receives ``+= [loss, correct,
    count]`` inside the fold kernel."""
    return _SoftmaxNLL.apply(S_hat, S_hat2, lay_s.ptr, lay_t.counts, y_col,
                             mask, float(eps), stats)


# ---------------------------------------------------------------------------
class _Sinkhorn(torch.autograd.Function):
    """Masked log-domain Sinkhorn per pair (csrc/hip/sinkhorn.hip): the
    forward keeps each half-step's potentials, the backward rebuilds the
    half-step outputs from them and applies the normalisation Jacobians in
    reverse."""

    @staticmethod
    def forward(ctx, S_hat, n_s, n_t, iters, tau):
        S_hat = S_hat.float().contiguous()
        P, ah, bh = _backend.ops().sinkhorn_fwd(S_hat, n_s, n_t, int(iters),
                                                float(tau))
        ctx.save_for_backward(S_hat, n_s, n_t, ah, bh)
        ctx.iters, ctx.tau = int(iters), float(tau)
        return P

    @staticmethod
    def backward(ctx, grad):
        S_hat, n_s, n_t, ah, bh = ctx.saved_tensors
        dS = _backend.ops().sinkhorn_bwd(grad.float().contiguous(), S_hat,
                                         n_s, n_t, ah, bh, ctx.iters,
                                         ctx.tau)
        return dS, None, None, None, None


def masked_sinkhorn(S_hat, lay_s, lay_t, iters=10, tau=1.0):
    r"""Sinkhorn normalisation of the dense scores ``[B, N_s, N_t]`` over
    each pair's valid ``n_s x n_t`` block (``iters`` row + column rounds and
    a final row step, so rows sum to 1 like the reference's masked softmax;
    zeros outside).  HIP kernel on the GPU, :func:`.reference.masked_sinkhorn`
    elsewhere (the oracle of ``tests/test_sinkhorn.py``)."""
    B, N_s, N_t = S_hat.shape
    if _hip_ok(S_hat, N_s, N_t):
        return _Sinkhorn.apply(S_hat, lay_s.counts, lay_t.counts, iters, tau)
    return ref.masked_sinkhorn(S_hat, _count_mask(lay_s, lay_t), iters, tau)


class _SinkhornTransportJoint(torch.autograd.Function):
    """``[r_s; sinkhorn(S_hat)^T r_s]`` (and optionally the normalised
    ``P`` itself) from one per-pair kernel (csrc/hip/sinkhorn.hip::
    sinkhorn_transport); the backward forms ``dL/dP = G_P + r_s g_t^T``
    inside the Sinkhorn backward kernel (plus ``S_hat``'s passthrough
    gradient) - no batched GEMMs, pack / unpack or gradient adds."""

    @staticmethod
    def forward(ctx, S_hat, r_s, ptr_s, ptr_t, rows_t, iters, tau, with_prob,
                passthrough):
        S_hat = S_hat.float().contiguous()
        r_s = r_s.float().contiguous()
        joint, P, ah, bh = _backend.ops().sinkhorn_transport(
            S_hat, r_s, ptr_s, ptr_t, int(rows_t), int(iters), float(tau),
            bool(with_prob))
        ctx.save_for_backward(S_hat, r_s, ptr_s, ptr_t, ah, bh)
        ctx.iters, ctx.tau = int(iters), float(tau)
        ctx.with_prob, ctx.passthrough = bool(with_prob), bool(passthrough)
        ctx.joint_shape = tuple(joint.shape)
        ctx.set_materialize_grads(False)
        out = (joint, )
        if with_prob:
            out = out + (P, )
        if passthrough:
            out = out + (S_hat.view_as(S_hat), )
        return out if len(out) > 1 else joint

    @staticmethod
    def backward(ctx, gj, *rest):
        S_hat, r_s, ptr_s, ptr_t, ah, bh = ctx.saved_tensors
        rest = list(rest)
        gP = rest.pop(0) if ctx.with_prob else None
        gpass = rest.pop(0) if ctx.passthrough else None
        if gj is None:
            gj = torch.zeros(ctx.joint_shape, device=S_hat.device)
        dS = _backend.ops().sinkhorn_transport_bwd(
            None if gP is None else gP.float().contiguous(),
            gj.float().contiguous(), r_s, S_hat, ptr_s, ptr_t, ah, bh,
            ctx.iters, ctx.tau,
            None if gpass is None else gpass.float().contiguous())
        return (dS, ) + (None, ) * 8


def sinkhorn_transport_supported(S_hat, r_s, lay_s, lay_t):
    B, N_s, N_t = S_hat.shape
    return (_hip_ok(S_hat, N_s, N_t) and r_s.dim() == 2 and
            r_s.size(1) in (64, 128, 256) and
            torch.is_tensor(getattr(lay_s, 'ptr', None)) and
            torch.is_tensor(getattr(lay_t, 'ptr', None)))


def sinkhorn_transport_joint(S_hat, r_s, lay_s, lay_t, iters=10, tau=1.0,
                             with_prob=False, passthrough=False):
    r"""``joint = [r_s; masked_sinkhorn(S_hat)^T r_s]`` packed
    ``[sum N_s + sum N_t, R]`` fp32 (psi_2's fused input), differentiable
    w.r.t. ``S_hat``.  ``with_prob`` also returns the dense normalised
    ``P`` (``masked_sinkhorn(S_hat)``); ``passthrough`` an alias of
    ``S_hat`` whose gradient is summed inside the backward kernel.
    Returns ``joint`` or the tuple ``(joint[, P][, S_hat'])``."""
    return _SinkhornTransportJoint.apply(S_hat, r_s, lay_s.ptr, lay_t.ptr,
                                         lay_t.num_nodes, iters, tau,
                                         with_prob, passthrough)


# ---------------------------------------------------------------------------
class _SoftmaxTransport(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S_hat, r_s, ptr_s, ptr_t, rows_t):
        S, r_t = _backend.ops().dense_softmax_transport(
            S_hat.float().contiguous(), r_s.contiguous(), ptr_s, ptr_t,
            rows_t)
        ctx.save_for_backward(S, r_s, ptr_s, ptr_t)
        ctx.dtype = S_hat.dtype
        return r_t

    @staticmethod
    def backward(ctx, grad):
        S, r_s, ptr_s, ptr_t = ctx.saved_tensors
        g = _backend.ops().dense_softmax_transport_bwd(
            S, r_s.contiguous(), grad.to(r_s.dtype).contiguous(), ptr_s,
            ptr_t)
        return g.to(ctx.dtype), None, None, None, None


class _SoftmaxTransportJoint(torch.autograd.Function):
    """Returns ``[r_s; r_t]`` (psi_2's fused input) from one kernel: the
    transport kernel also copies ``r_s`` - no concatenation kernel.  With
    ``passthrough`` it also returns an alias of ``S_hat`` for S_hat's other
    consumer (the consensus update): that gradient is added inside the
    backward kernel instead of by a separate autograd add."""

    @staticmethod
    def forward(ctx, S_hat, r_s, ptr_s, ptr_t, rows_t, passthrough=False,
                planes=False):
        r_s = r_s.contiguous()
        pl = _joint_planes(r_s, rows_t) if planes else None
        S, joint = _backend.ops().dense_softmax_transport(
            S_hat.float().contiguous(), r_s, ptr_s, ptr_t, rows_t, True, pl)
        _attach_planes(joint, pl)
        ctx.save_for_backward(S, r_s, ptr_s, ptr_t)
        ctx.dtype = S_hat.dtype
        ctx.n_s = r_s.size(0)
        if passthrough:
            return joint, S_hat.view_as(S_hat)
        return joint

    @staticmethod
    def backward(ctx, grad, gpass=None):
        S, r_s, ptr_s, ptr_t = ctx.saved_tensors
        add = gpass if (gpass is not None and
                        gpass.dtype == torch.float32 and
                        gpass.is_contiguous() and
                        gpass.shape == S.shape) else None
        g = _backend.ops().dense_softmax_transport_bwd(
            S, r_s.contiguous(), grad[ctx.n_s:].to(r_s.dtype).contiguous(),
            ptr_s, ptr_t, add)
        g = g.to(ctx.dtype)
        if gpass is not None and add is None:
            g = g + gpass
        return g, None, None, None, None, None, None


def _joint_planes(r_s, rows_t):
    """bf16x6 planes buffer ``[3, rows_s + rows_t, R]`` for the joint
    ``[r_s; r_t]`` (written by the transport kernel), or None when the joint
    is not fp32."""
    if r_s.dtype != torch.float32 or r_s.size(1) % 4 != 0:
        return None
    return torch.empty((3, r_s.size(0) + rows_t, r_s.size(1)),
                       dtype=torch.bfloat16, device=r_s.device)


def _attach_planes(joint, planes):
    # (the record psi_2's first slot conv checks: shape and version of x)
    if planes is not None:
        joint._dgmc_x6 = (planes, joint._version)


def transport_joint_supported(S_hat, lay_s, lay_t):
    B, N_s, N_t = S_hat.shape
    return _hip_ok(S_hat, N_s, N_t)


def softmax_transport_joint(S_hat, r_s, lay_s, lay_t, passthrough=False,
                            planes=False):
    r"""``[r_s; masked_softmax(S_hat)^T r_s]`` as one packed
    ``[sum N_s + sum N_t, R]`` tensor (differentiable w.r.t. ``S_hat``).
    ``passthrough`` returns ``(joint, S_hat')`` with ``S_hat'`` an alias of
    ``S_hat`` whose gradient is summed inside this op's backward kernel.
    ``planes``: the consumer is a bf16x6 slot conv - the kernel also writes
    the joint's operand planes (fp32; attached to ``joint``)."""
    return _SoftmaxTransportJoint.apply(S_hat, r_s, lay_s.ptr, lay_t.ptr,
                                        lay_t.num_nodes, passthrough, planes)


def softmax_transport(S_hat, r_s, lay_s, lay_t):
    r"""``masked_softmax(S_hat)^T r_s`` with packed ``r_s [sum N_s, R]``;
    returns packed ``r_t [sum N_t, R]`` in ``r_s``'s dtype (fp32 or bf16;
    accumulation in fp32).  ``r_s`` is a non-differentiable random indicator
    (as in the reference); gradients flow into ``S_hat``.
    """
    B, N_s, N_t = S_hat.shape
    if _hip_ok(S_hat, N_s, N_t):
        return _SoftmaxTransport.apply(S_hat, r_s, lay_s.ptr, lay_t.ptr,
                                       lay_t.num_nodes)
    S = ref.masked_softmax(S_hat, _count_mask(lay_s, lay_t))
    r_t = S.transpose(-1, -2) @ lay_s.to_dense(r_s.to(S.dtype))
    return lay_t.to_sparse(r_t)


# ---------------------------------------------------------------------------
class _ConsensusUpdate(torch.autograd.Function):
    """``P``/``Q`` separately, or ``P`` = joint ``[P; Q]`` with ``Q`` an int
    row split (then the joint gradient buffer is produced directly - no
    slice-backward fill + copies)."""

    @staticmethod
    def forward(ctx, S_hat, P, Q, b1, w2, b2, ptr_s, ptr_t, loop):
        ctx.split = None
        if isinstance(Q, int):
            ctx.split = Q
            P, Q = P[:Q], P[Q:]
        out = _backend.ops().dense_consensus(
            S_hat.float().contiguous(), P.contiguous(), Q.contiguous(),
            b1.float().contiguous(), w2.float().contiguous().view(-1),
            b2.float().contiguous().view(-1), ptr_s, ptr_t)
        ctx.save_for_backward(P, Q, b1, w2, ptr_s, ptr_t)
        ctx.meta = (S_hat.dtype, b1.dtype, w2.dtype, b2.dtype, b2.shape)
        ctx.loop = loop
        ctx.idx = loop.register() if loop is not None else None
        return out

    @staticmethod
    def backward(ctx, grad):
        P, Q, b1, w2, ptr_s, ptr_t = ctx.saved_tensors
        dPQ = None
        if ctx.split is not None:
            dPQ = torch.empty((P.size(0) + Q.size(0), P.size(1)),
                              dtype=P.dtype, device=P.device)
        part, accum = _loop_part(ctx.loop, grad.size(0), P.size(1),
                                 grad.device)
        dP, dQ, dw2_part, db2_part = _backend.ops().dense_consensus_bwd(
            grad.float().contiguous(), P.contiguous(), Q.contiguous(),
            b1.float().contiguous(), w2.float().contiguous().view(-1), ptr_s,
            ptr_t, dPQ, part, accum)
        dP_rows = dP                    # db1 = column sum over P rows only
        if dPQ is not None:
            dP, dQ = dPQ, None
        s_dt, b1_dt, w2_dt, b2_dt, b2_shape = ctx.meta
        db1, dw2, db2 = _consensus_param_grads(ctx.loop, ctx.idx, dP_rows,
                                               dw2_part, db2_part)
        if db1 is not None:
            db1 = db1.to(b1_dt)
            dw2 = dw2.view_as(w2).to(w2_dt)
            db2 = db2.view(b2_shape).to(b2_dt)
        return (grad.to(s_dt), dP, dQ, db1, dw2, db2, None, None, None)


class _ConsensusTransport(torch.autograd.Function):
    """Consensus update of step ``l`` fused with the softmax transport of step
    ``l + 1`` (``dense_consensus_transport``): returns ``(joint, S_hat')``
    with ``joint = [r_s; masked_softmax(S_hat')^T r_s]`` for the next psi_2
    call.  The backward kernel forms S_hat''s total gradient (transport
    backward + the next step's identity path) and runs the consensus backward
    on it in the same workgroup."""

    @staticmethod
    def forward(ctx, S_hat, PQ, split, b1, w2, b2, r_s, ptr_s, ptr_t, rows_t,
                loop, planes=False):
        P, Q = PQ[:split], PQ[split:]
        r_s = r_s.contiguous()
        pl = _joint_planes(r_s, rows_t) if planes else None
        S_new, S_prob, joint = _backend.ops().dense_consensus_transport(
            S_hat.float().contiguous(), P, Q, b1.float().contiguous(),
            w2.float().contiguous().view(-1), b2.float().contiguous().view(-1),
            r_s, ptr_s, ptr_t, rows_t, pl)
        _attach_planes(joint, pl)
        ctx.save_for_backward(S_prob, r_s, P, Q, b1, w2, ptr_s, ptr_t)
        ctx.meta = (S_hat.dtype, b1.dtype, w2.dtype, b2.dtype, b2.shape)
        ctx.n_s = r_s.size(0)
        ctx.loop = loop
        ctx.idx = loop.register() if loop is not None else None
        ctx.set_materialize_grads(False)
        return joint, S_new

    @staticmethod
    def backward(ctx, g_joint, g_S):
        S_prob, r_s, P, Q, b1, w2, ptr_s, ptr_t = ctx.saved_tensors
        R = P.size(1)
        if g_joint is None:
            g_t = r_s.new_zeros((Q.size(0), R))
        else:
            g_t = g_joint[ctx.n_s:].to(r_s.dtype).contiguous()
        add = None
        if g_S is not None:
            add = g_S.float().contiguous()
        dPQ = torch.empty((P.size(0) + Q.size(0), R), dtype=P.dtype,
                          device=P.device)
        part, accum = _loop_part(ctx.loop, S_prob.size(0), R, P.device)
        G, dP, _, dw2_part, db2_part = \
            _backend.ops().dense_transport_consensus_bwd(
                S_prob, r_s.contiguous(), g_t, add, P, Q,
                b1.float().contiguous(), w2.float().contiguous().view(-1),
                ptr_s, ptr_t, dPQ, part, accum)
        s_dt, b1_dt, w2_dt, b2_dt, b2_shape = ctx.meta
        db1, dw2, db2 = _consensus_param_grads(
            ctx.loop, ctx.idx, dP, dw2_part, db2_part)
        if db1 is not None:
            db1 = db1.to(b1_dt)
            dw2 = dw2.view_as(w2).to(w2_dt)
            db2 = db2.view(b2_shape).to(b2_dt)
        return (G.to(s_dt), dPQ, None, db1, dw2, db2, None, None, None, None,
                None, None)


def _loop_part(loop, B, R, device):
    """``(part, accumulate)``: the loop's ``[B, 2R + 1]`` fp32 accumulator of
    per-pair ``[db1 | dw2 | db2]`` partials, written by the backward kernels
    of every use in turn (``(None, False)`` outside a loop)."""
    if loop is None:
        return None, False
    return loop.acc('pq_part', (B, 2 * R + 1), device)


def _consensus_param_grads(loop, idx, dP, dw2_part, db2_part):
    """``(db1, dw2, db2)`` of one consensus use; inside a loop the kernels
    accumulated them into the loop's part buffer and the use completing the
    set folds it with ONE column sum (``None`` for the others)."""
    if loop is None:
        parts = (dP, dw2_part, db2_part.view(-1, 1))
        return tuple(_col_sum(t) for t in parts)
    if loop.arrive():
        part = loop.get_acc('pq_part')
        R = (part.size(1) - 1) // 2
        tot = _col_sum(part)
        loop.release()
        return tot[:R], tot[R:2 * R], tot[2 * R:]
    return None, None, None


def consensus_transport_supported(PQ, r_s, S_hat):
    B, N_s, N_t = S_hat.shape
    return (_hip_ok(S_hat, N_s, N_t) and
            PQ.dtype in (torch.bfloat16, torch.float32) and
            r_s.dtype == PQ.dtype and PQ.is_contiguous() and
            PQ.size(1) == r_s.size(1))


class _CatMatmul(torch.autograd.Function):
    """``[X_0 | X_1 | ...] @ W`` (bf16, ``W = w [K, 128]``) without forming
    the concatenation for the product (``cat_gemm``); the kernel writes the
    concatenation once into the loop's stacked weight-gradient operand.
    Backward: ``g W^T`` split into column views (no copies) and, when the
    last loop use arrives, ONE long-K ``dW`` GEMM over all uses."""

    @staticmethod
    def forward(ctx, w, w_n, w_nt, loop, total, *parts):
        M = parts[0].size(0)
        K = sum(p.size(1) for p in parts)
        ctx.loop, ctx.widths = loop, [p.size(1) for p in parts]
        ctx.w_dtype = w.dtype
        # (grad mode is off inside forward: needs_input_grad alone says
        # whether the backward will want dW.)
        need_w = ctx.needs_input_grad[0]
        if loop is not None:
            ctx.idx = loop.register()
            ocat = loop.slot_total('x', ctx.idx, (M, K), w_n.dtype,
                                   w_n.device, total)
        else:
            ctx.idx = None
            ocat = torch.empty((M, K), dtype=w_n.dtype, device=w_n.device) \
                if need_w else None
        out = _backend.ops().cat_gemm(list(parts), w_n, ocat)
        ctx.save_for_backward(w_n, w_nt)
        ctx.ocat = ocat if loop is None else None
        return out

    @staticmethod
    def backward(ctx, g):
        from .gemm import matmul_tn_fp32
        w_n, w_nt = ctx.saved_tensors
        g = g.contiguous()
        if g.dtype != w_n.dtype:
            g = g.to(w_n.dtype)
        # g W^T = [M, 128] x [128, K] on the same kernel (W^T staged in LDS).
        if w_nt.size(0) in (128, 256, 384) and \
                g.data_ptr() % 16 == 0:
            gx = _backend.ops().cat_gemm([g], w_nt, None)    # [M, K]
        else:
            gx = g @ w_n                                     # [M, K]
        grads, off = [], 0
        for i, wd in enumerate(ctx.widths):
            grads.append(gx[:, off:off + wd]
                         if ctx.needs_input_grad[5 + i] else None)
            off += wd
        gw = None
        loop = ctx.loop
        if loop is None:
            if ctx.needs_input_grad[0]:
                gw = matmul_tn_fp32(ctx.ocat, g).to(ctx.w_dtype)
        else:
            loop.keep('g', ctx.idx, g)
            if loop.arrive():
                if ctx.needs_input_grad[0]:
                    X = loop.stack('x')
                    gl = loop.kept_list('g')
                    if dense_wgrad_supported(X, gl):
                        gw = dense_wgrad(list(X.unbind(0)), gl).to(
                            ctx.w_dtype)
                    else:
                        gw = matmul_tn_fp32(X.view(-1, X.size(-1)),
                                            loop.kept('g')).to(ctx.w_dtype)
                loop.release()
        return (gw, None, None, None, None) + tuple(grads)


def dense_wgrad_supported(X, gs):
    return (_backend.use_hip(X) and X.dtype == torch.bfloat16
            and X.dim() == 3 and X.size(-1) % 128 == 0 and
            X.size(-1) <= 512 and X.is_contiguous() and
            X.data_ptr() % 16 == 0 and len(gs) == X.size(0) and
            all(g.dtype == torch.bfloat16 and g.is_contiguous() and
                g.shape == (X.size(1), 128) and g.data_ptr() % 16 == 0
                for g in gs))


def dense_wgrad(xs, gs, nsplit=None, out=None, accumulate=False):
    r"""``sum_u xs[u]^T gs[u]`` (fp32 ``[Kx, Kg]``) for bf16 ``xs[u] [N, Kx]``
    and ``gs[u] [N, Kg]`` (multiples of 128) read in place
    (csrc/hip/slot_wgrad.hip::dense_wgrad: TN MFMA over row chunks, per-split
    partials folded by ``reduce_add_rows``, optionally into ``out``)."""
    Kx, Kg = xs[0].size(1), gs[0].size(1)
    blocks = (Kx // 128) * (Kg // 128)
    n = xs[0].size(0)
    nsplit = nsplit or max(1, min(256 // blocks, (n + 127) // 128))
    if out is None:
        out = torch.empty(Kx * Kg, dtype=torch.float32, device=xs[0].device)
        accumulate = False
    flat = out.view(-1)
    for i in range(0, len(xs), 16):
        part = _backend.ops().dense_wgrad(list(xs[i:i + 16]),
                                          list(gs[i:i + 16]), nsplit)
        _backend.ops().reduce_add_rows(part.view(nsplit, Kx * Kg), flat,
                                       accumulate or i > 0)
    return out.view(Kx, Kg)


def cat_matmul_supported(parts, w_t):
    return (all(_backend.use_hip(p) and p.dtype == torch.bfloat16 and
                p.dim() == 2 and p.stride(1) == 1 and p.size(1) % 32 == 0 and
                p.stride(0) % 8 == 0 and p.data_ptr() % 16 == 0
                for p in parts) and
            1 <= len(parts) <= 4 and w_t.size(1) == 128 and
            w_t.size(0) == sum(p.size(1) for p in parts) and
            w_t.size(0) in (128, 256, 384))


def cat_matmul(parts, w_t, lp, key, total):
    """``cat(parts, -1) @ w_t`` with ``w_t [K, 128]`` (fp32, receives the
    gradient) - see :class:`_CatMatmul`; ``total`` = uses of ``key``'s loop
    collector in this forward (the consensus steps)."""
    w_n = lp.get('n')
    if w_n is None:
        w_n = lp['n'] = w_t.detach().t().to(torch.bfloat16).contiguous()
        lp['nt'] = w_n.t().contiguous()
    loop = loopgrad.group(('catmm', ) + key + (parts[0].size(0), )) \
        if total else None
    with torch.autocast(device_type='cuda', enabled=False):
        return _CatMatmul.apply(w_t, w_n, lp['nt'], loop, total, *parts)


_SEG01 = {}


def _seg01(M, device):
    """Device int32 ``[0, M]`` (one "slot" covering all rows) for the dense
    weight-gradient kernel; created outside graph capture (the warm-up
    steps) and reused by the captured replays."""
    key = (str(device), int(M))
    t = _SEG01.get(key)
    if t is None:
        t = _SEG01[key] = torch.tensor([0, int(M)], dtype=torch.int32,
                                       device=device)
    return t


# The folded projection's NT products on bf16x6 (fp32 parts split in the
# kernel's registers; error vs fp64 below the exact-f32 MFMA kernel's:
# tests/test_slot_gemm_x6.py) or on the exact-f32 MFMA kernel.
NT_X6 = True


def _nt_x6():
    from . import slot_gemm
    return NT_X6 and slot_gemm.X6


def _nt(ops, parts, bt, b3=None):
    """``[parts] @ bt^T``; ``b3``: bf16x6 planes of ``bt`` (split once per
    forward scope), used by the bf16x6 kernel."""
    if _nt_x6():
        return ops.dense_nt_x6(parts, bt, b3)
    return ops.dense_nt_f32(parts, bt)


class _CatMatmulF32(torch.autograd.Function):
    """fp32 ``[X_0 | X_1 | ...] @ W`` (``W = w_t [128 n, 128]``) on the
    LDS-DMA MFMA GEMM reading psi_2's feature parts in place
    (``csrc/hip/slot_gemm.hip::dense_nt_f32``: no concatenation); backward
    ``g W^T`` on the same kernel (part gradients are column views), and
    inside a consensus loop the weight gradient of all uses as ONE dense TN
    launch over the kept parts (``dense_wgrad_f32``: no stacked copies)."""

    @staticmethod
    def forward(ctx, w_t, loop, *parts):
        from ..runtime.cache import cached
        ops = _backend.ops()
        # Both B operands (w_t^T for the forward, w_t itself for the input
        # gradient, k-contiguous) and their bf16x6 planes: built once per
        # forward scope, shared by the consensus loop's uses.
        key = ('cat_f32_w', w_t.data_ptr(), w_t._version, tuple(w_t.shape),
               tuple(w_t.stride()))
        bt = cached(key + ('t', ), lambda: w_t.detach().t().contiguous())
        wc = cached(key, lambda: w_t.detach().contiguous())
        x6 = _nt_x6()
        bt3 = cached(key + ('t3', ), lambda: ops.split3(bt)) if x6 else None
        wc3 = cached(key + ('3', ), lambda: ops.split3(wc)) if x6 else None
        out = _nt(ops, list(parts), bt, bt3)
        ctx.loop, ctx.np = loop, len(parts)
        # The parts go through save_for_backward (autograd's version check
        # catches an in-place write to a part before the weight gradient).
        keep = tuple(parts) if ctx.needs_input_grad[0] else ()
        ctx.wc3 = wc3
        ctx.save_for_backward(w_t, wc, *keep)
        ctx.idx = loop.register() if loop is not None else None
        return out

    @staticmethod
    def backward(ctx, g):
        w_t, wc, *kept = ctx.saved_tensors
        ctx.parts = tuple(kept) if kept else None
        ops = _backend.ops()
        g = g.float().contiguous()
        gx = _nt(ops, [g], wc, ctx.wc3)                         # [M, 128 n]
        ctx.wc3 = None
        grads = tuple(gx[:, 128 * i:128 * (i + 1)]
                      if ctx.needs_input_grad[2 + i] else None
                      for i in range(ctx.np))
        need_w = ctx.needs_input_grad[0]
        seg = _seg01(g.size(0), g.device)
        gw, loop = None, ctx.loop
        if loop is None:
            if need_w:
                gw = ops.dense_wgrad_f32(list(ctx.parts), ctx.np, [g], seg)
        else:
            if need_w:
                loop.keep('g', ctx.idx, g)
                loop.keep('xp', ctx.idx, ctx.parts)
            ctx.parts = None
            if loop.arrive():
                if need_w:
                    xps, gs = loop.kept_list('xp'), loop.kept_list('g')
                    for i in range(0, len(gs), 16):
                        part = ops.dense_wgrad_f32(
                            [p for t in xps[i:i + 16] for p in t], ctx.np,
                            gs[i:i + 16], seg)
                        gw = part if gw is None else gw.add_(part)
                loop.release()
        if gw is not None:
            gw = gw.to(w_t.dtype)
        return (gw, None) + grads


def cat_matmul_f32_supported(parts, w_t):
    return (1 <= len(parts) <= 4 and w_t.dtype == torch.float32 and
            tuple(w_t.shape) == (128 * len(parts), 128) and
            parts[0].size(0) % 32 == 0 and
            all(_backend.use_hip(p) and p.dtype == torch.float32 and
                p.dim() == 2 and p.is_contiguous() and p.size(1) == 128 and
                p.size(0) == parts[0].size(0) and p.data_ptr() % 16 == 0
                for p in parts))


def cat_matmul_f32(parts, w_t, key, total):
    """``cat(parts, -1) @ w_t`` in fp32 without the concatenation (see
    :class:`_CatMatmulF32`); ``total`` = uses of ``key``'s loop collector
    in this forward (the consensus steps)."""
    loop = loopgrad.group(('catmm32', ) + key + (parts[0].size(0), )) \
        if total else None
    with torch.autocast(device_type='cuda', enabled=False):
        return _CatMatmulF32.apply(w_t, loop, *parts)


def consensus_update(S_hat, o_s, o_t, mlp, lay_s, lay_t, o_joint=None,
                     w1_fold=None, next_r_s=None, planes=False):
    r"""``S_hat + mask * mlp(o_s[:, :, None] - o_t[:, None])`` for packed
    ``o_s [sum N_s, R]`` / ``o_t [sum N_t, R]``.  ``o_joint`` may pass the
    concatenation ``[o_s; o_t]`` (fused encoder output) to compute both
    projections with one GEMM.  ``mlp`` must be ``Seq(Lin(R, R), ReLU,
    Lin(R, 1))`` (``dgmc.py:74-78``).  ``w1_fold = (W^T, lp_cache, key)``
    replaces ``W1^T`` by a folded ``[K, R]`` map applied to ``o_joint``
    (the encoder's pre-projection features; see ``DGMC._forward``).
    ``next_r_s`` / ``planes``: see :class:`_ConsensusTransport` /
    :func:`softmax_transport_joint`.
    """
    lin1, lin2 = mlp[0], mlp[2]
    B, N_s, N_t = S_hat.shape
    if w1_fold is not None and (o_joint is None or
                                not _hip_ok(S_hat, N_s, N_t)):
        raise ValueError('w1_fold needs the joint HIP path')
    if w1_fold is not None:
        w_t, lp, key, total = w1_fold
        parts = getattr(o_joint, 'parts', None)
        if parts is not None and cat_matmul_supported(parts, w_t):
            PQ = cat_matmul(parts, w_t, lp, key, total)
        elif parts is not None and cat_matmul_f32_supported(parts, w_t):
            PQ = cat_matmul_f32(parts, w_t, key, total)
        else:
            if parts is not None:
                o_joint = o_joint.cat()
            w_lp = lp.get(o_joint.dtype)
            if w_lp is None:
                w_lp = lp[o_joint.dtype] = w_t.detach().to(o_joint.dtype)
            PQ = mixed_matmul(o_joint, w_t, w_lp, loop_key=key + (
                o_joint.size(0), ))
        loop = loopgrad.group(('consensus', id(mlp)))
        if next_r_s is not None and FUSE_STEPS and \
                consensus_transport_supported(PQ, next_r_s, S_hat):
            # (joint input of the next psi_2 call, S_hat')
            return _ConsensusTransport.apply(
                S_hat, PQ, lay_s.num_nodes, lin1.bias, lin2.weight,
                lin2.bias, next_r_s, lay_s.ptr, lay_t.ptr,
                lay_t.num_nodes, loop, planes)
        return _ConsensusUpdate.apply(S_hat, PQ, lay_s.num_nodes, lin1.bias,
                                      lin2.weight, lin2.bias, lay_s.ptr,
                                      lay_t.ptr, loop)
    if _hip_ok(S_hat, N_s, N_t):
        w1t = lin1.weight.t()
        key = (id(lin1.weight), )
        if o_joint is not None:
            PQ = mixed_matmul(o_joint, w1t,
                              lowp_weight_t(lin1.weight, o_joint.dtype),
                              loop_key=key + (o_joint.size(0), ))
            P, Q = PQ, lay_s.num_nodes   # joint: split inside the op
        else:
            P = mixed_matmul(o_s, w1t, lowp_weight_t(lin1.weight, o_s.dtype),
                             loop_key=key + (o_s.size(0), ))
            Q = mixed_matmul(o_t, w1t, lowp_weight_t(lin1.weight, o_t.dtype),
                             loop_key=key + (o_t.size(0), ))
        loop = loopgrad.group(('consensus', id(mlp)))
        return _ConsensusUpdate.apply(S_hat, P, Q, lin1.bias, lin2.weight,
                                      lin2.bias, lay_s.ptr, lay_t.ptr, loop)
    o_s_d = lay_s.to_dense(o_s.to(S_hat.dtype))
    o_t_d = lay_t.to_dense(o_t.to(S_hat.dtype))
    upd = ref.consensus_mlp_dense(o_s_d, o_t_d, lin1.weight, lin1.bias,
                                  lin2.weight, lin2.bias)
    return S_hat + upd.masked_fill(~_count_mask(lay_s, lay_t), 0)
