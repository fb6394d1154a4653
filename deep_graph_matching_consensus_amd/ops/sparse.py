"""Sparse operators: the single primitive all message passing reduces to.

Every aggregation on the reference's hot path is a *fixed* sparse linear map
applied to a dense feature matrix:

* SplineConv message+mean+root (``/root/reference/dgmc/models/spline.py:49``,
  PyG ``SplineConv`` over torch_spline_conv) =
  ``A_spline @ (x @ [W_0 .. W_{K-1} | root])`` where ``A_spline`` has one entry
  per (edge, B-spline slot) with value ``basis / deg`` plus a root diagonal;
* GINConv sum (``gin.py:49``) = ``A_adj @ x + (1 + eps) x``;
* RelConv two-flow mean (``rel.py:26-31``) =
  ``A_rel @ (x @ [lin1 | lin2 | root])``.

``SparseOperator`` stores such a map in CSR (int32 ``rowptr``/``col``, fp32
``val``) and lazily materialises its transpose, so the backward of
``spmm`` is the same deterministic gather-reduce kernel on ``A^T`` - no float
atomics anywhere (the reference's torch_scatter / spline_weighting backward
use atomicAdd).  Plans are built once per batch and reused by every layer and
every consensus step.
"""
import torch

from . import _backend
from . import reference as ref


class SparseOperator(object):
    r"""Fixed-structure, fixed-value CSR matrix of shape ``[R, C]``."""

    def __init__(self, rowptr, col, val, num_rows, num_cols, row=None):
        self.rowptr = rowptr.to(torch.int32).contiguous()
        self.col = col.to(torch.int32).contiguous()
        self.val = val.to(torch.float32).contiguous()
        self.num_rows = int(num_rows)
        self.num_cols = int(num_cols)
        self._row = row
        self._t = None

    @property
    def nnz(self):
        return self.col.numel()

    @property
    def device(self):
        return self.col.device

    @property
    def row(self):
        """int64 row id of every stored entry (CSR expanded)."""
        if self._row is None:
            counts = (self.rowptr[1:] - self.rowptr[:-1]).long()
            self._row = torch.repeat_interleave(
                torch.arange(self.num_rows, device=self.device), counts,
                output_size=self.nnz)
        return self._row

    @staticmethod
    def from_coo(row, col, val, num_rows, num_cols):
        """Build from unsorted COO (stable sort by row; no host sync)."""
        row = row.long()
        perm = torch.argsort(row, stable=True)
        row, col, val = row[perm], col[perm], val[perm]
        counts = torch.zeros(num_rows, dtype=torch.long, device=row.device)
        counts.index_add_(0, row, torch.ones_like(row))
        rowptr = torch.zeros(num_rows + 1, dtype=torch.long,
                             device=row.device)
        torch.cumsum(counts, 0, out=rowptr[1:])
        return SparseOperator(rowptr, col, val, num_rows, num_cols, row=row)

    def t(self):
        """Transpose (cached)."""
        if self._t is None:
            self._t = SparseOperator.from_coo(self.col.long(), self.row,
                                              self.val, self.num_cols,
                                              self.num_rows)
            self._t._t = self
        return self._t

    def to_dense(self):
        out = torch.zeros(self.num_rows, self.num_cols, device=self.device)
        out.index_put_((self.row, self.col.long()), self.val, accumulate=True)
        return out

    def __repr__(self):
        return 'SparseOperator(shape=[{}, {}], nnz={})'.format(
            self.num_rows, self.num_cols, self.nnz)


def _spmm_raw(op, x, self_x, self_scale, bias, relu, out_dtype):
    if _backend.use_hip(x):
        return _backend.ops().spmm_csr(
            op.rowptr, op.col, op.val, x.contiguous(),
            self_x.contiguous() if self_x is not None else None,
            self_scale, bias, relu, out_dtype)
    return ref.spmm(op.row, op.col, op.val, op.num_rows, x, self_x,
                    self_scale, bias, relu, out_dtype)


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, self_x, self_scale, bias, op, relu, out_dtype):
        out = _spmm_raw(op, x, self_x, self_scale, bias, relu, out_dtype)
        ctx.op, ctx.relu = op, relu
        ctx.x_dtype = x.dtype
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.save_for_backward(self_x, self_scale, out if relu else None)
        return out

    @staticmethod
    def backward(ctx, grad):
        self_x, self_scale, out = ctx.saved_tensors
        grad = grad.contiguous()
        gbias = None
        need_bias = ctx.bias_dtype is not None and ctx.needs_input_grad[3]
        if _backend.use_hip(grad) and (ctx.relu or need_bias):
            # Fused: g = grad * (out > 0) and per-block bias partials.
            g, part = _backend.ops().relu_bias_bwd(
                grad, out if ctx.relu else grad, ctx.relu, ctx.x_dtype)
            if need_bias:
                gbias = part.sum(0).to(ctx.bias_dtype)
        else:
            g = grad.float()
            if ctx.relu:
                g = g * (out > 0)
            if need_bias:
                gbias = g.sum(0).to(ctx.bias_dtype)
        gx = gself = gscale = None
        if ctx.needs_input_grad[0]:
            gx = _spmm_raw(ctx.op.t(), g, None, None, None, False,
                           ctx.x_dtype)
        if self_x is not None:
            gf = g.float()
            if ctx.needs_input_grad[1]:
                gself = (gf * self_scale.float()).to(self_x.dtype)
            if ctx.needs_input_grad[2]:
                gscale = (gf * self_x.float()).sum().view_as(self_scale)
                gscale = gscale.to(self_scale.dtype)
        return gx, gself, gscale, gbias, None, None, None


def spmm(op, x, self_x=None, self_scale=None, bias=None, relu=False,
         out_dtype=None):
    r"""``act(op @ x + self_scale * self_x + bias)`` with fp32 accumulation.

    ``x`` may be fp32 or bf16 (e.g. the output of a bf16 GEMM).  The result
    keeps bf16/fp16 inputs in their dtype (so the next GEMM needs no cast and
    the backward moves half the bytes) and is fp32 otherwise; override with
    ``out_dtype``.  Gradients flow to ``x``, ``self_x``, ``self_scale`` and
    ``bias``.
    """
    assert x.dim() == 2 and x.size(0) == op.num_cols, (x.shape, op)
    if self_x is not None:
        assert self_x.size(0) == op.num_rows and self_scale is not None
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) \
            else torch.float32
    return _SpMM.apply(x, self_x, self_scale, bias, op, relu, out_dtype)
