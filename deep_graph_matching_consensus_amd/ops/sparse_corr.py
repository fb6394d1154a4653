"""Sparse (top-k) correspondence ops
(``/root/reference/dgmc/models/dgmc.py:184-244``).

* :func:`top_k`      - candidate search ``argtopk_j <h_s[b,i], h_t[b,j]>``
  (``dgmc.py:85-94``; KeOps ``argKmin`` in the reference).  On the GPU a fused
  HIP kernel streams ``h_t`` tiles through LDS, computes the dot tiles on
  MFMA and keeps a per-row register top-k, so the ``N_s x N_t`` score matrix
  is never materialised.  The default is EXACT fp32 selection (the
  reference's fp32 KeOps ``argKmin``) at split-bf16 speed: a split-bf16
  ("bf16x3") pass keeps 32 approximate candidates per row, every one within
  a proven error margin of the k-th is re-scored with the exact fp32 chain,
  and rows whose margin is not covered are recomputed exhaustively
  (``csrc/hip/topk.hip::topk_refine_kernel``) - indices identical to the
  brute-force exact-f32 MFMA kernel.  ``exact=False`` returns the unrefined
  split-bf16 selection.
* :class:`CandidateGraph`  - the candidate set ``S_idx [B, N_s, k]`` as a CSR
  matrix over flattened source rows (global target columns ``b*N_t + idx``)
  plus its transpose, built once per forward.
* :func:`gather_dot` - ``S_hat[b,i,c] = <h_s[b,i], h_t[b, S_idx[b,i,c]]>``
  (``dgmc.py:197-201``): an SDDMM kernel; backward = two SpMMs.
* :func:`sparse_transport` - ``r_t = scatter_add(S * r_s, S_idx)``
  (``dgmc.py:209-212``): SpMM over the transpose (deterministic, no atomics);
  backward w.r.t. ``S`` = SDDMM.
* :func:`consensus_update` - ``S_hat + MLP(o_s[:, :, None] - o_t[S_idx])``
  (``dgmc.py:219-223``) in factored form ``relu(P_i + b1 - Q_idx) . w2 + b2``
  with ``P = o_s W1^T``, ``Q = o_t W1^T`` computed per node.

The reference quirks are kept: no masking of padded targets or rows in the
sparse path (``dgmc.py:202,223``).
"""

import torch
import torch.nn.functional as F

from . import _backend
from . import reference as ref
from .gemm import _col_sum
from ..runtime import loopgrad
from .sparse import SparseOperator, piece_plan


TOPK_EXACT = True


def top_k(h_s, h_t, k, exact=None, brute_force=False, warm=None):
    """``[B, N_s, k]`` int64 indices of the k best targets per source row
    (best first, ties to the lower index).

    ``exact`` (default :data:`TOPK_EXACT`, on): exact fp32 selection
    (filter + exact re-score on the GPU); ``exact=False``: split-bf16
    scores (~2^-16 relative error - near-ties can rank differently).
    ``brute_force``: the exact-f32 MFMA kernel over every target (the test
    oracle of the refined path).  ``warm``: optional persistent int64
    ``[B, N_s, 32]`` state (exact path, k <= 10): the filter's candidate
    lists are kept there and the next call's filter starts from a proven
    lower bound of every row's threshold computed from them - same output,
    far fewer list insertions when consecutive calls see similar
    embeddings (training steps)."""
    B, N_s, C = h_s.shape
    if exact is None:
        exact = TOPK_EXACT
    if _backend.use_hip(h_s) and k <= 64 and C % 4 == 0 and C <= 256 \
            and h_s.dtype == torch.float32:
        mode = 1 if brute_force else (2 if exact else 0)
        return _backend.ops().topk_dot(h_s.contiguous(), h_t.contiguous(),
                                       int(k), mode,
                                       warm if mode == 2 else None)
    return ref.top_k(h_s, h_t, k)


class CandidateGraph(object):
    """CSR/CSC view of ``S_idx [B, N_s, k]`` over targets ``[B * N_t]``."""

    def __init__(self, S_idx, N_t):
        B, N_s, k = S_idx.shape
        dev = S_idx.device
        self.B, self.N_s, self.N_t, self.k = B, N_s, N_t, k
        self.rows, self.cols = B * N_s, B * N_t
        if _backend.use_hip(S_idx):
            # prep + stable radix sort by column + pointers: 5 launches
            # (csrc/hip/candidates.hip::candidate_csc).
            (self.col, self.rowptr, self.colptr, self.perm32,
             self.row_of) = _backend.ops().candidate_csc(
                 S_idx.contiguous(), N_t)
            self.perm = self.perm32
            nnz = self.col.numel()
        else:
            offs = (torch.arange(B, device=dev) * N_t).view(B, 1, 1)
            col = (S_idx + offs).reshape(-1)
            self.rowptr = (torch.arange(self.rows + 1, device=dev) * k).to(
                torch.int32)
            self.col = col.to(torch.int32)
            self.perm = torch.argsort(col, stable=True)
            counts = torch.zeros(self.cols, dtype=torch.long, device=dev)
            counts.index_add_(0, col, torch.ones_like(col))
            colptr = torch.zeros(self.cols + 1, dtype=torch.long, device=dev)
            torch.cumsum(counts, 0, out=colptr[1:])
            self.colptr = colptr.to(torch.int32)
            self.row_of = (self.perm // k).to(torch.int32)
            self.perm32 = self.perm.to(torch.int32)
            nnz = col.numel()
        # Column walks (transport, consensus dQ, gather-dot dB) in pieces of
        # <= sparse.PIECE entries: with random-init embeddings a few
        # targets sit in
        # the top-k of thousands of rows (hubness), which would serialise a
        # column-per-wave kernel.
        self.col_pieces = piece_plan(self.colptr, nnz)

    def op(self, val):
        """``[rows, cols]`` operator with per-entry values ``val``."""
        return SparseOperator(self.rowptr, self.col, val, self.rows,
                              self.cols)

    def op_t(self, val):
        """Transposed operator ``[cols, rows]``."""
        return SparseOperator(self.colptr, self.row_of, val[self.perm],
                              self.cols, self.rows)


def _spmm(op, x):
    return _backend.ops().spmm_csr(op.rowptr, op.col, op.val, x.contiguous(),
                                   None, None, None, False, torch.float32)


def _spmm_t(cand, val, x):
    """``op_t(val) @ x`` (targets <- sources) by the piece-balanced SpMM over
    the CSC, reading ``val`` through the CSC permutation in place."""
    x = x.contiguous()
    out = torch.empty((cand.cols, x.size(1)), dtype=torch.float32,
                      device=x.device)
    _backend.ops().spmm_pieces_out(cand.colptr, cand.row_of, val.contiguous(),
                                   cand.perm32, *cand.col_pieces, x, None,
                                   None, None, False, out)
    return out


# ---------------------------------------------------------------------------
class _GatherDot(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, Bm, cand):
        ctx.cand = cand
        ctx.save_for_backward(A, Bm)
        return _backend.ops().sddmm(cand.rowptr, cand.col, A, Bm)

    @staticmethod
    def backward(ctx, g):
        A, Bm = ctx.saved_tensors
        cand = ctx.cand
        g = g.contiguous().float()
        dA = _spmm(cand.op(g), Bm) if ctx.needs_input_grad[0] else None
        dB = _spmm_t(cand, g, A) if ctx.needs_input_grad[1] else None
        return dA, dB, None


def gather_dot(h_s, h_t, S_idx, cand=None):
    """``S_hat [B, N_s, k]`` (autograd through both embeddings)."""
    B, N_s, C = h_s.shape
    k = S_idx.size(-1)
    if cand is not None and _backend.use_hip(h_s) and C <= 512:
        out = _GatherDot.apply(h_s.reshape(-1, C).float().contiguous(),
                               h_t.reshape(-1, C).float().contiguous(), cand)
        return out.view(B, N_s, k)
    idx = S_idx.reshape(B, N_s * k, 1).expand(-1, -1, C)
    tmp_t = torch.gather(h_t, 1, idx).view(B, N_s, k, C)
    return (h_s.unsqueeze(2) * tmp_t).sum(dim=-1)


# ---------------------------------------------------------------------------
class _SparseTransport(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S, r_s, cand):
        ctx.cand = cand
        ctx.save_for_backward(r_s)
        return _spmm_t(cand, S, r_s)

    @staticmethod
    def backward(ctx, g):
        r_s, = ctx.saved_tensors
        cand = ctx.cand
        dS = _backend.ops().sddmm(cand.rowptr, cand.col, r_s,
                                  g.contiguous().float())
        return dS, None, None


def sparse_transport(S, r_s, S_idx, N_t, cand=None):
    """``r_t[b, j] = sum_{(i,c): S_idx[b,i,c] = j} S[b,i,c] * r_s[b,i]``."""
    B, N_s, k = S.shape
    R = r_s.size(-1)
    if cand is not None and _backend.use_hip(S) and R <= 512:
        out = _SparseTransport.apply(S.reshape(-1).float().contiguous(),
                                     r_s.reshape(-1, R).float().contiguous(),
                                     cand)
        return out.view(B, N_t, R)
    tmp = (r_s.unsqueeze(2) * S.unsqueeze(-1)).reshape(B, N_s * k, R)
    idx = S_idx.reshape(B, N_s * k, 1).expand(-1, -1, R)
    out = torch.zeros(B, N_t, R, dtype=tmp.dtype, device=tmp.device)
    return out.scatter_add(1, idx, tmp)


# ---------------------------------------------------------------------------
class _SparseConsensus(torch.autograd.Function):
    """Consensus update from the joint node projections ``PQ = [P; Q]``
    (``P = PQ[:n_s]``, ``Q = PQ[n_s:]``): the backward writes ``[dP; dQ]``
    into one buffer (no slice-backward zero fills, copies and adds), and its
    row kernel also emits the per-block partials of the MLP's b1 / w2 / b2
    gradients.  Inside a loop scope those partials are kept per use and
    folded once by the last use (runtime/loopgrad.py): no per-step
    reductions and no AccumulateGrad adds.  ``soft_k > 0`` (uniform rows of
    ``soft_k`` candidates) also returns the row softmax of the update - the
    next step's ``S`` - from the same kernel; its backward (softmax backward
    + the pass-through add) runs inside the consensus backward kernel."""

    @staticmethod
    def forward(ctx, S_hat, PQ, n_s, b1, w2, b2, cand, loop=None, soft_k=0):
        ctx.cand = cand
        ctx.n_s = n_s
        ctx.meta = (b1.dtype, w2.dtype, b2.dtype, b2.shape)
        ctx.loop = loop
        ctx.idx = loop.register() if loop is not None else None
        ctx.soft = bool(soft_k)
        ctx.set_materialize_grads(False)
        b1f = b1.float().contiguous()
        w2f = w2.float().contiguous().view(-1)
        b2f = b2.float().contiguous().view(-1)
        P, Q = PQ[:n_s], PQ[n_s:]
        if soft_k:
            out, prob = _backend.ops().sparse_consensus_fwd_prob(
                cand.rowptr, cand.col, S_hat, P, Q, b1f, w2f, b2f,
                int(soft_k))
            ctx.save_for_backward(PQ, b1, w2, prob)
            return out, prob
        ctx.save_for_backward(PQ, b1, w2)
        return _backend.ops().sparse_consensus_fwd(
            cand.rowptr, cand.col, S_hat, P, Q, b1f, w2f, b2f)

    @staticmethod
    def backward(ctx, g, gS=None):
        if ctx.soft:
            PQ, b1, w2, prob = ctx.saved_tensors
        else:
            PQ, b1, w2 = ctx.saved_tensors
            prob = None
        cand, n_s = ctx.cand, ctx.n_s
        P, Q = PQ[:n_s], PQ[n_s:]
        if g is None:
            g = torch.zeros(cand.col.numel(), dtype=torch.float32,
                            device=PQ.device)
        g = g.contiguous().float()
        soft = prob is not None and gS is not None
        dPQ = torch.empty_like(PQ)
        _, _, part, g = _backend.ops().sparse_consensus_bwd(
            cand.rowptr, cand.col, cand.colptr, cand.row_of, cand.perm32, g,
            P, Q, b1.float().contiguous(), w2.float().contiguous().view(-1),
            *cand.col_pieces, prob if soft else None,
            gS.contiguous().float() if soft else None, dPQ)
        b1_dt, w2_dt, b2_dt, b2_shape = ctx.meta
        R = PQ.size(1)
        nones = (None, None, None)

        def split(tot):     # [dw2 | db1 | db2, 0, 0, 0]
            return (tot[R:2 * R].to(b1_dt), tot[:R].view_as(w2).to(w2_dt),
                    tot[2 * R].view(b2_shape).to(b2_dt))
        loop = ctx.loop
        if loop is None:
            db1, dw2, db2 = split(_col_sum(part))
            return (g, dPQ, None, db1, dw2, db2) + nones
        loop.keep('part', ctx.idx, part)
        db1 = dw2 = db2 = None
        if loop.arrive():
            db1, dw2, db2 = split(_col_sum(loop.kept('part')))
            loop.release()
        return (g, dPQ, None, db1, dw2, db2) + nones


def soft_fusable(k, R):
    """Can the consensus kernel also emit the row softmax (rows of ``k``
    candidates, ``R`` channels)?  (sparse_corr.hip::soft_max_k)"""
    if R % 4 or R > 256 or R == 0:
        return False
    G = 1
    while G * 4 < R:
        G *= 2
    return 1 <= k <= min(64, 8 * (64 // G))


def consensus_update_pq(S_hat, PQ, n_s, mlp, cand, with_prob=False):
    """``S_hat + relu(P_i + b1 - Q_idx) . w2 + b2`` from the joint node-level
    projections ``PQ = [P; Q]``: ``P = PQ[:n_s]`` (``[B * N_s, R]``), ``Q =
    PQ[n_s:]`` (``[B * N_t, R]``) - the folded form ``P = o_s W1^T`` with
    psi_2's final Linear inside, models/dgmc.py.
    ``with_prob``: returns ``(S_hat', softmax(S_hat'))`` from one kernel."""
    B, N_s, k = S_hat.shape
    lin1, lin2 = mlp[0], mlp[2]
    res = _SparseConsensus.apply(S_hat.reshape(-1).float().contiguous(),
                                 PQ.float().contiguous(), n_s, lin1.bias,
                                 lin2.weight, lin2.bias, cand,
                                 _consensus_loop(lin1),
                                 k if with_prob else 0)
    if with_prob:
        return res[0].view(B, N_s, k), res[1].view(B, N_s, k)
    return res.view(B, N_s, k)


def _consensus_loop(lin1):
    """Loop collector of the consensus MLP's vector gradients (taken here:
    grad mode is off inside ``Function.forward``)."""
    return loopgrad.group(('sparse_consensus', id(lin1.bias)))


def consensus_update(S_hat, o_s, o_t, S_idx, mlp, cand=None):
    """``S_hat + MLP(o_s[:, :, None] - o_t[S_idx])`` on dense ``o_s
    [B, N_s, R]`` / ``o_t [B, N_t, R]``."""
    B, N_s, k = S_hat.shape
    R = o_s.size(-1)
    lin1, lin2 = mlp[0], mlp[2]
    if cand is not None and _backend.use_hip(S_hat) and R <= 512:
        PQ = F.linear(torch.cat([o_s.reshape(-1, R), o_t.reshape(-1, R)]
                                ).float(), lin1.weight.float())
        out = _SparseConsensus.apply(S_hat.reshape(-1).float().contiguous(),
                                     PQ.contiguous(), B * N_s,
                                     lin1.bias, lin2.weight, lin2.bias, cand,
                                     _consensus_loop(lin1))
        return out.view(B, N_s, k)
    idx = S_idx.reshape(B, N_s * k, 1).expand(-1, -1, R)
    o_t_g = torch.gather(o_t, 1, idx).view(B, N_s, k, R)
    return S_hat + ref.consensus_mlp_sparse(o_s, o_t_g, lin1.weight,
                                            lin1.bias, lin2.weight, lin2.bias)
