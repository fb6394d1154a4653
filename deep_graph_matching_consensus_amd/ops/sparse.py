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


PIECE = 16   # entries per piece of the balanced SpMM (spmm.hip)


def piece_plan(rowptr, nnz, T=PIECE):
    """Cut every CSR row into pieces of at most ``T`` entries (an empty row
    keeps one empty piece, so every row is written).  Returns int32
    ``pptr [R + 1]`` (first piece of each row) and, per piece slot
    (``R + nnz // T + 1`` of them, a static bound - no host sync),
    ``prow`` (the row, bit-inverted ``~r`` when the row has several pieces;
    ``R`` for unused slots), ``pbeg`` / ``pend`` (entry range).  Built by one
    HIP kernel on the GPU (``spmm.hip::piece_plan``)."""
    if _backend.use_hip(rowptr):
        return tuple(_backend.ops().piece_plan(rowptr, int(nnz), int(T)))
    R = rowptr.numel() - 1
    dev = rowptr.device
    rowptr = rowptr.to(torch.int32)
    counts = rowptr[1:] - rowptr[:-1]
    npc = torch.clamp_min(torch.div(counts + (T - 1), T,
                                    rounding_mode='floor'), 1)
    pptr = torch.zeros(R + 1, dtype=torch.int32, device=dev)
    torch.cumsum(npc, 0, dtype=torch.int32, out=pptr[1:])
    P = R + int(nnz) // T + 1
    v = torch.arange(P, dtype=torch.int32, device=dev)
    row = torch.searchsorted(pptr[1:], v, right=True, out_int32=True)
    used = row < R
    r = torch.where(used, row, torch.zeros_like(row)).long()
    beg = rowptr[r] + (v - pptr[r]) * T
    end = torch.minimum(rowptr[r + 1], beg + T)
    code = torch.where(npc[r] > 1, -row - 1, row)
    prow = torch.where(used, code, torch.full_like(row, R))
    pbeg = torch.where(used, beg, torch.zeros_like(beg))
    pend = torch.where(used, end, torch.zeros_like(end))
    return pptr, prow, pbeg.to(torch.int32), pend.to(torch.int32)


class SparseOperator(object):
    r"""Fixed-structure, fixed-value CSR matrix of shape ``[R, C]``.

    ``balanced``: rows can be long and skewed (knowledge-graph hubs), so the
    HIP SpMM walks them in pieces of :data:`PIECE` entries
    (:func:`piece_plan`, ``spmm.hip::spmm_piece_kernel``) instead of one
    lane group per row.  Inherited by the transpose."""

    def __init__(self, rowptr, col, val, num_rows, num_cols, row=None,
                 balanced=False):
        self.rowptr = rowptr.to(torch.int32).contiguous()
        self.col = col.to(torch.int32).contiguous()
        self.val = val.to(torch.float32).contiguous()
        self.num_rows = int(num_rows)
        self.num_cols = int(num_cols)
        self._row = row
        self._t = None
        self.balanced = balanced
        # static: the structure outlives one step (e.g. a KG relational
        # plan), so a once-per-operator host split of its rows pays.
        self.static = False
        self._pieces = None
        self._split = None

    def pieces(self):
        """``(pptr, prow, pbeg, pend)`` of :func:`piece_plan` (cached)."""
        if self._pieces is None:
            self._pieces = piece_plan(self.rowptr, self.nnz)
        return self._pieces

    def split_rows(self):
        """``(short_rows, long_rows)`` int32: rows of at most / more than
        :data:`PIECE` entries (``spmm.hip::spmm_split_kernel``), or None
        while a graph is being captured before the split exists (it needs
        one host synchronisation).  Cached."""
        if self._split is None:
            if self.rowptr.is_cuda and \
                    torch.cuda.is_current_stream_capturing():
                return None
            counts = self.rowptr[1:] - self.rowptr[:-1]
            long_ = counts > PIECE
            self._split = (
                torch.nonzero(~long_).view(-1).to(torch.int32).contiguous(),
                torch.nonzero(long_).view(-1).to(torch.int32).contiguous())
        return self._split

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
            self._t.balanced = self.balanced
            self._t.static = self.static
        return self._t

    def slot_csr(self, num_slots):
        """``[R * S, C / S]`` re-indexing of a slot-structured operator
        (columns ``j * S + k``): row ``i * S + k`` lists the source nodes
        ``j`` of slot ``k`` - the gather order of :func:`gemm_spmm`'s fused
        kernel.  Cached."""
        cache = self.__dict__.setdefault('_slot_csr', {})
        sc = cache.get(num_slots)
        if sc is None:
            S = int(num_slots)
            col = self.col.long()
            sc = SparseOperator.from_coo(self.row * S + col % S, col // S,
                                         self.val, self.num_rows * S,
                                         self.num_cols // S)
            cache[num_slots] = sc
        return sc

    def to_dense(self):
        out = torch.zeros(self.num_rows, self.num_cols, device=self.device)
        out.index_put_((self.row, self.col.long()), self.val, accumulate=True)
        return out

    def __repr__(self):
        return 'SparseOperator(shape=[{}, {}], nnz={})'.format(
            self.num_rows, self.num_cols, self.nnz)


def _split_ok(x):
    """Rows of at most 16 16-byte vectors (spmm_split_kernel's lanes)."""
    width = 4 if x.dtype == torch.float32 else 8
    return (x.dim() == 2 and x.size(1) % width == 0 and
            x.size(1) // width <= 16 and x.is_contiguous() and
            x.data_ptr() % 16 == 0 and x.dtype in (torch.float32,
                                                   torch.bfloat16))


def spmm_out(op, x, out, self_x=None, self_scale=None, bias=None,
             relu=False):
    """HIP SpMM into ``out`` (piece-balanced for ``op.balanced``; for a
    static balanced operator with narrow rows, the one-launch short / long
    row split)."""
    split = op.split_rows() if (op.balanced and op.static and
                                _split_ok(x)) else None
    if split is not None:
        _backend.ops().spmm_split_out(op.rowptr, op.col, op.val, split[0],
                                      split[1], x, self_x, self_scale, bias,
                                      relu, out)
    elif op.balanced:
        _backend.ops().spmm_pieces_out(
            op.rowptr, op.col, op.val, None, *op.pieces(), x, self_x,
            self_scale, bias, relu, out)
    else:
        _backend.ops().spmm_csr_out(op.rowptr, op.col, op.val, x, self_x,
                                    self_scale, bias, relu, out)
    return out


def _spmm_raw(op, x, self_x, self_scale, bias, relu, out_dtype):
    if _backend.use_hip(x) and op.balanced:
        x = x.contiguous()
        out = torch.empty((op.num_rows, x.size(1)), dtype=out_dtype,
                          device=x.device)
        return spmm_out(op, x, out, self_x.contiguous()
                        if self_x is not None else None, self_scale, bias,
                        relu)
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
            # Fused: g = grad * (out > 0) and the bias gradient.
            g, db = _backend.ops().relu_bias_bwd(
                grad, out if ctx.relu else grad, ctx.relu, ctx.x_dtype)
            if need_bias:
                gbias = db.to(ctx.bias_dtype)
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


# ---------------------------------------------------------------------------
# Fused "GEMM then aggregate" layer (SplineConv / RelConv shape)
# ---------------------------------------------------------------------------
class _GemmSpMM(torch.autograd.Function):
    """``out = act(A @ view(x @ W, [-1, C]) + bias)`` as ONE autograd node.

    Backward: ``g' = grad * relu'`` and ``dbias`` (one fused kernel),
    ``dY = A^T g'`` (written straight into the loop stack when ``loop`` is
    set), ``dx = dY W^T``, ``dW = x^T dY`` - deferred to one long-K GEMM over
    all loop uses (see :mod:`..runtime.loopgrad`).
    """

    @staticmethod
    def forward(ctx, x, w, w_lp, bias, op, relu, C, loop, passthrough=False):
        xc = x if x.dtype == w_lp.dtype else x.to(w_lp.dtype)
        ctx.passthrough = passthrough
        K = xc.size(1)
        S = w_lp.size(1) // C
        ctx.img_b = None
        ctx.slot = _slot_conv_ok(op, xc, K, C, S)
        if ctx.slot:
            # Graph-closed tiles: Z_k = A_k x and Z_k W_k on MFMA, Y and Z
            # never materialised (csrc/hip/slot_conv.hip).
            img = slot_conv_image(w_lp, C, trans=False)
            if loop is not None:
                ctx.img_b = slot_conv_image(w_lp, C, trans=True)
            out = _backend.ops().slot_conv(
                xc.contiguous(), *slot_tile_plan(op, S), S, img, False, bias,
                relu, xc.dtype, None)
        else:
            from .gemm import nt_f32, nt_f32_supported
            if nt_f32_supported([xc], w_lp.t()):
                # chunked NT MFMA GEMM (bf16x6 unless DGMC_AMD_X6=0), x read
                # in place (csrc/hip/gemm_f32.hip)
                y = nt_f32([xc], w_lp.t()).view(-1, C)
            else:
                y = (xc @ w_lp).view(-1, C)
            out_dtype = y.dtype if y.dtype in (torch.bfloat16,
                                               torch.float16) \
                else torch.float32
            out = _spmm_raw(op, y, None, None, bias, relu, out_dtype)
        ctx.save_for_backward(xc, w_lp, out if relu else None)
        ctx.op, ctx.relu, ctx.C, ctx.loop = op, relu, C, loop
        ctx.x_dtype, ctx.w_dtype = x.dtype, w.dtype
        ctx.w_transposed = w.dim() == 2 and w.size(0) > 1 and \
            w.size(1) > 1 and w.stride(0) == 1 and w.stride(1) == w.size(0)
        # Gradient carrier token of nn/conv.py::_StackedSplineWeight (an
        # expanded 1-element tensor): its node can take the loop-folded
        # weight gradient in slot-major layout directly (no permute copy, no
        # unpack kernel).
        node = w.grad_fn if (w.dim() == 2 and w.stride() == (0, 0)) \
            else None
        ctx.w_node = node if hasattr(node, 'takes_slot_major') else None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.idx = loop.register() if loop is not None else None
        if passthrough:
            # A second consumer reads x through this alias: its gradient
            # arrives here and is fused into dx (no autograd add kernel).
            return out, x.view_as(x)
        return out

    @staticmethod
    def _slot_loop_backward(ctx, grad, gpass, xc, out, op, K, S, need_b):
        """Consensus-loop use on the fused slot kernels: g' (ReLU mask), the
        bias gradient's tile partials and dx in ONE transposed slot conv
        (``slot_conv_relu_bwd``); dW later from the kept (x, g') pairs of all
        uses (``slot_weight_grad``)."""
        from .gemm import loop_col_total
        loop, idx, C = ctx.loop, ctx.idx, ctx.C
        plan = slot_tile_plan(op, S)
        if (grad.stride(-1) != 1 or grad.stride(0) < C or
                grad.stride(0) % 8 or grad.data_ptr() % 16):
            grad = grad.contiguous()
        part = loop.slot('b', idx, (plan[0].size(0), C), torch.float32,
                         grad.device) if need_b else None
        g = torch.empty((grad.size(0), C), dtype=torch.bfloat16,
                        device=grad.device)
        add = gpass if _addend_ok(gpass, g) else None
        gx = _backend.ops().slot_conv_relu_bwd(
            grad, out if ctx.relu else None, *plan, S, ctx.img_b, g.dtype,
            add, g, part)
        if add is not None:
            gpass = None
        if gx.dtype != ctx.x_dtype:
            gx = gx.to(ctx.x_dtype)
        gx = _add_pass(gx, gpass) if ctx.needs_input_grad[0] else None
        loop.keep('x', idx, xc)
        loop.keep('g', idx, g)
        gw = gb = None
        if loop.arrive():
            need_w = ctx.needs_input_grad[1]
            xs, gs = loop.kept_list('x'), loop.kept_list('g')
            if need_w:
                dW = slot_weight_grad(xs, gs, op, S, loop.uses)
            if need_b:
                gb = loop_col_total(loop, 'b').to(ctx.bias_dtype)
            if need_w:
                if ctx.w_node is not None:
                    # Slot-major [S, in, out] straight to the stacked-weight
                    # node (nn/conv.py): weight / root gradients are views.
                    ctx.w_node.slot_major = dW
                else:
                    gw = dW.permute(1, 0, 2).reshape(K, S * C).to(
                        ctx.w_dtype)
            loop.release()
        return (gx, gw, None, gb) + (None, ) * 5

    @staticmethod
    def backward(ctx, grad, gpass=None):
        from .gemm import col_partial_rows, loop_col_total, matmul_tn_fp32
        nones = (None, ) * 5
        xc, w_lp, out = ctx.saved_tensors
        loop, idx, C = ctx.loop, ctx.idx, ctx.C
        dev = grad.device
        need_b = ctx.bias_dtype is not None and ctx.needs_input_grad[3]
        hip = _backend.use_hip(grad)
        op = ctx.op
        K = xc.size(1)
        S = w_lp.size(1) // C
        if (hip and ctx.slot and loop is not None and
                ctx.img_b is not None and
                grad.dtype == torch.bfloat16 and w_lp.dtype == torch.bfloat16
                and (out is None or out.dtype == torch.bfloat16)):
            return _GemmSpMM._slot_loop_backward(ctx, grad, gpass, xc, out,
                                                 op, K, S, need_b)
        if not hip or grad.stride(-1) != 1 or grad.stride(0) < grad.size(1):
            grad = grad.contiguous()    # (the kernel reads column slices)
        # 1. g' = grad * relu'(out) and the bias gradient.
        db = None
        if hip:
            # Loop uses keep per-block bias partials (folded once at the
            # end); a single use folds right away.
            part = loop.slot('b', idx, (col_partial_rows(grad.size(0)), C),
                             torch.float32, dev) \
                if (loop is not None and need_b) else None
            g, db = _backend.ops().relu_bias_bwd(
                grad, out if ctx.relu else grad, ctx.relu, w_lp.dtype, None,
                False, part)
        else:
            g = grad.float()
            if ctx.relu:
                g = g * (out > 0)
            if need_b:
                db = g.sum(0)
                if loop is not None:
                    loop.add_to('b', db)
            g = g.to(w_lp.dtype)
        if (ctx.slot and loop is not None and
                g.dtype == torch.bfloat16 and ctx.img_b is not None):
            # 2'. dx by the transposed slot conv; dW from the kept (x, g')
            #     pairs of all uses - dY is never formed.
            gx = gw = gb = None
            if ctx.needs_input_grad[0]:
                add = gpass if _addend_ok(gpass, g) else None
                gx = _backend.ops().slot_conv(
                    g.contiguous(), *slot_tile_plan(op, S), S, ctx.img_b,
                    True, None, False, g.dtype, None, add)
                if add is not None:
                    gpass = None
                if gx.dtype != ctx.x_dtype:
                    gx = gx.to(ctx.x_dtype)
                gx = _add_pass(gx, gpass)
            loop.keep('x', idx, xc)
            loop.keep('g', idx, g)
            if loop.arrive():
                if ctx.needs_input_grad[1]:
                    dW = slot_weight_grad(loop.kept_list('x'),
                                          loop.kept_list('g'), op, S,
                                          loop.uses)
                    gw = dW.permute(1, 0, 2).reshape(K, S * C)
                    gw = gw.to(ctx.w_dtype)
                if need_b:
                    gb = loop_col_total(loop, 'b').to(ctx.bias_dtype)
                loop.release()
            return (gx, gw, None, gb) + nones
        # 2. dY = A^T g' (and dx = sum_k dY_k W_k^T, fused when possible).
        slot = ctx.img_b is not None and ctx.needs_input_grad[0] and \
            g.dtype == torch.bfloat16
        opt = None if slot else op.t()
        rows_t = op.num_cols
        if loop is not None:
            dy = loop.slot('dy', idx, (rows_t, C), w_lp.dtype, dev)
            loop.keep('x', idx, xc)      # concatenated once at the end
        elif slot:
            dy = torch.empty((rows_t, C), dtype=w_lp.dtype, device=dev)
        else:
            dy = None
        gx = gw = gb = None
        if slot:
            # Same tiles, A_k^T and W_k^T: dx in one kernel, which also
            # writes dY = A^T g' for the weight gradient.
            gx = _backend.ops().slot_conv(
                g.contiguous(), *slot_tile_plan(op, S), S, ctx.img_b, True,
                None, False, g.dtype, dy)
            if gx.dtype != ctx.x_dtype:
                gx = gx.to(ctx.x_dtype)
        elif dy is not None and hip:
            spmm_out(opt, g, dy)
        elif dy is not None:
            dy.copy_(_spmm_raw(opt, g, None, None, None, False, w_lp.dtype))
        else:
            dy = _spmm_raw(opt, g, None, None, None, False, w_lp.dtype)
        dY = dy.view(xc.size(0), -1)
        # 3. dx (unfused path) and dW.  A passthrough consumer's gradient
        #    enters the GEMM epilogue (beta = 1): no separate add kernel.
        if ctx.needs_input_grad[0] and gx is None and hip and \
                dY.dtype == torch.float32 and ctx.x_dtype == torch.float32:
            # fp32 (RelConv's stacked map, ψ₁ of the DBP15K config): dx =
            # dY [N, 3C] @ W_stacked [3C, K] on the chunked NT GEMM; a
            # passthrough consumer's gradient is accumulated in place by its
            # epilogue (beta = 1, ``passthrough='cat'``) - no library GEMM.
            from .gemm import nt_f32, nt_f32_supported
            bt = w_lp.contiguous()                   # [K, 3C]
            if nt_f32_supported([dY], bt):
                if ctx.passthrough == 'cat' and gpass is not None and \
                        gpass.dtype == torch.float32 and \
                        gpass.shape == (dY.size(0), bt.size(0)) and \
                        gpass.dim() == 2 and gpass.stride(1) == 1 and \
                        gpass.stride(0) % 4 == 0 and \
                        gpass.data_ptr() % 16 == 0:
                    gx = nt_f32([dY], bt, out=gpass, accumulate=True)
                    gpass = None
                else:
                    gx = nt_f32([dY], bt)
        if ctx.needs_input_grad[0] and gx is None:
            if gpass is not None and gpass.dtype == dY.dtype == \
                    ctx.x_dtype and gpass.shape == (dY.size(0),
                                                    w_lp.size(0)):
                if ctx.passthrough == 'cat' and gpass.dim() == 2 and \
                        gpass.stride(1) == 1 and \
                        gpass.stride(0) >= gpass.size(1):
                    # In place (opt-in, ``passthrough='cat'``: the caller
                    # guarantees the alias feeds exactly one torch.cat, so
                    # gpass is this op's own slice of the concatenation's
                    # gradient - CatBackward hands out disjoint column views
                    # nothing else reads): the GEMM accumulates into it with
                    # beta = 1, no copy of gpass into a fresh output first.
                    gx = gpass.addmm_(dY, w_lp.t())
                else:
                    gx = torch.addmm(gpass, dY, w_lp.t())
                gpass = None
            else:
                gx = (dY @ w_lp.t()).to(ctx.x_dtype)
        # w = (stacked weights).t() (RelConv): the gradient is produced in
        # the stacked [3C, K] layout and handed back transposed, so the
        # concatenation's backward gives each Linear a contiguous slice that
        # AccumulateGrad keeps without a layout copy.
        wt = ctx.w_transposed
        if loop is None:
            if ctx.needs_input_grad[1]:
                gw = (matmul_tn_fp32(dY, xc.contiguous()).t() if wt else
                      matmul_tn_fp32(xc.contiguous(), dY)).to(ctx.w_dtype)
            if need_b:
                gb = db.to(ctx.bias_dtype)
        elif loop.arrive():
            if ctx.needs_input_grad[1]:
                X = loop.kept('x').contiguous()
                dYs = loop.stack('dy').view(X.size(0), -1)
                gw = matmul_tn_fp32(dYs, X).t() if wt else \
                    matmul_tn_fp32(X, dYs)
                gw = gw.to(ctx.w_dtype)
            if need_b:
                gb = loop_col_total(loop, 'b').to(ctx.bias_dtype)
            loop.release()
        return (_add_pass(gx, gpass), gw, None, gb) + nones


def _addend_ok(a, g):
    """Can the slot conv epilogue add ``a`` into its bf16 output?"""
    return (a is not None and a.dtype == torch.bfloat16 and
            a.device == g.device and a.dim() == 2 and
            a.size(0) == g.size(0) and a.size(1) == _SLOT_C and
            a.stride(1) == 1 and a.stride(0) % 4 == 0 and
            a.data_ptr() % 8 == 0)


def _add_pass(gx, gpass):
    if gx is None or gpass is None:
        return gx
    return gx + gpass


# Fused slot convolution on graph-closed row tiles (csrc/hip/slot_conv.hip,
# bf16): used whenever the operator carries graph-start flags (static
# batches, datasets/static_batch.py) and the layer is 128 -> 128 wide (psi_2
# of the PascalVOC/WILLOW configs).  Forward: the fused kernel; consensus-loop
# backward: the transposed slot conv (ReLU mask, g', bias partials and dx in
# one kernel) + the slot weight gradient from the kept (x, g') pairs of every
# use (csrc/hip/slot_wgrad.hip; no dY stack).  Measured on MI355X:
# docs/performance.md.  SLOT_CONV = False selects GEMM + SpMM (tests).
SLOT_CONV = True
_SLOT_C = 128
_SLOT_MAX_S = 62    # one wave lane per slot offset (csrc/hip/slot_conv.hip)
_SLOT_ERR = {}
_SLOT_PERM = {}


def _slot_conv_ok(op, x, K, C, S):
    return (SLOT_CONV and getattr(op, 'tile_flag', None) is not None and
            K == _SLOT_C and C == _SLOT_C and S <= _SLOT_MAX_S and
            x.dtype == torch.bfloat16 and _backend.use_hip(x))


def slot_conv_error(device):
    """Persistent int32 [1] flag the slot-conv kernel sets if a tile breaks
    its contract (bit 0: > 64 rows, bit 1: an entry leaves its tile,
    bit 2: > 65535 entries in one tile)."""
    key = str(device)
    err = _SLOT_ERR.get(key)
    if err is None:
        err = _SLOT_ERR[key] = torch.zeros(1, dtype=torch.int32,
                                           device=device)
    return err


def slot_tile_plan(op, S):
    """``(tiles, soff, ecode, eval)`` of ``op`` for the slot conv: tile
    bounds and the tiles' entries bucketed by slot, built once per operator
    (one launch per training step, shared by every psi_2 use and backward)."""
    plan = op.__dict__.setdefault('_slot_plan', {})
    p = plan.get(S)
    if p is None:
        p = plan[S] = tuple(_backend.ops().slot_tile_plan(
            op.tile_flag, op.rowptr, op.col, op.val, op.tile_window, S,
            slot_conv_error(op.device)))
    return p


def slot_pair_lists(op, S):
    """``(esrc, edst, evals, soff)``: the entries of ``op`` grouped by slot
    (source node, target node, value; slot offsets), built once per operator
    on the device without host synchronisation."""
    cache = op.__dict__.setdefault('_slot_pairs', {})
    p = cache.get(S)
    if p is None and _backend.use_hip(op.col) and S <= 64:
        # Stable device counting sort (csrc/hip/slot_wgrad.hip).
        p = cache[S] = tuple(_backend.ops().slot_pair_lists(
            op.rowptr, op.col, op.val, op.row.contiguous(), S))
    if p is None:
        col = op.col.long()
        k = col % S
        perm = torch.argsort(k, stable=True)
        cnt = torch.zeros(S, dtype=torch.long, device=col.device)
        cnt.index_add_(0, k, torch.ones_like(k))
        soff = torch.zeros(S + 1, dtype=torch.int32, device=col.device)
        soff[1:] = torch.cumsum(cnt, 0).to(torch.int32)
        p = cache[S] = ((col // S)[perm].to(torch.int32).contiguous(),
                        op.row[perm].to(torch.int32).contiguous(),
                        op.val[perm].contiguous(), soff)
    return p


# Split partials of the slot weight gradient (64 measured best among
# 24..128, docs/performance.md).
SLOT_WGRAD_SPLITS = 64
_SLOT_WGRAD_MAX_LIST = 16    # pointer table size (csrc/hip/slot_wgrad.hip)


def slot_weight_grad(X, G, op, S, uses, nsplit=None):
    """``dW [S, C, C]`` (fp32) with ``dW_k = sum_u sum_{e in k} a_e
    X_u[j_e]^T G_u[i_e]`` for use-major stacks ``X, G [uses * N, C]`` or
    lists of the ``uses`` per-use ``[N, C]`` tensors (read in place)."""
    nsplit = nsplit or SLOT_WGRAD_SPLITS
    lists = slot_pair_lists(op, S)
    M = _SLOT_WGRAD_MAX_LIST
    stacked = not isinstance(X, (list, tuple))
    if stacked and uses > M:
        # More uses than the kernel's pointer table (num_steps > 16): per-use
        # row views of the stacks, chunked below.
        X, G = list(X.chunk(uses, 0)), list(G.chunk(uses, 0))
        stacked = False
    dev = X.device if stacked else X[0].device
    out = torch.empty(S * _SLOT_C, _SLOT_C, dtype=torch.float32, device=dev)
    if stacked:
        chunks = [None]
    else:
        X = [x.contiguous() for x in X]
        G = [g.contiguous() for g in G]
        chunks = range(0, len(X), M)
    # <= M uses per launch; the chunks' split partials are folded into the
    # same output in order (deterministic, no atomics).
    for i, c in enumerate(chunks):
        if c is None:
            part = _backend.ops().slot_wgrad(X.contiguous(), G.contiguous(),
                                             *lists, uses, nsplit)
        else:
            part = _backend.ops().slot_wgrad_list(X[c:c + M], G[c:c + M],
                                                  *lists, nsplit)
        _backend.ops().reduce_add_rows(
            part.view(nsplit, S * _SLOT_C, _SLOT_C), out, i > 0)
    return out.view(S, _SLOT_C, _SLOT_C)


def slot_k_order(device):
    """Position -> channel map of the kernel's 128-wide K axis: inside each
    32-wide chunk, lane group q holds channels 4q..4q+3 and 16+4q..16+4q+3
    (the rows an MFMA accumulator leaves in a lane, reused as the next
    product's B operand without a shuffle)."""
    key = str(device)
    p = _SLOT_PERM.get(key)
    if p is None:
        c = torch.arange(4).view(4, 1, 1)
        q = torch.arange(4).view(1, 4, 1)
        j = torch.arange(8).view(1, 1, 8)
        ch = 32 * c + torch.where(j < 4, 4 * q + j, 12 + 4 * q + j)
        p = _SLOT_PERM[key] = ch.reshape(-1).to(device)
    return p


def _slot_img_key(w_lp, trans):
    # Keyed by storage, not object: autograd hands every use a fresh
    # ``detach()`` view of the same cached low-precision weight (the entry
    # keeps it alive, so the address cannot be recycled within the scope).
    return ('slot_img', w_lp.data_ptr(), w_lp._version, tuple(w_lp.shape),
            bool(trans))


def prime_slot_images(w_lp, weight, root):
    """Compute both slot-conv weight images of a 128 -> 128 SplineConv from
    its parameters in ONE kernel (``spline_slot_images``) and store them in
    the forward scope under ``w_lp``'s keys, so :func:`slot_conv_image` finds
    them instead of permuting ``w_lp`` twice."""
    from ..runtime.cache import prime
    img_f, img_t = _backend.ops().spline_slot_images(
        weight.detach(), root.detach() if root is not None else None,
        slot_k_order(weight.device))
    # Looked up from _GemmSpMM.forward, i.e. with grad mode off.
    prime(_slot_img_key(w_lp, False), (w_lp, img_f), any_grad_mode=True)
    prime(_slot_img_key(w_lp, True), (w_lp, img_t), any_grad_mode=True)


def slot_conv_image(w_lp, C, trans):
    """``[S, C, C]`` weight image of the slot conv, memoised per forward
    scope: forward rows = output channels, backward (``trans``) rows = input
    channels; the K axis in :func:`slot_k_order`."""
    from ..runtime.cache import cached

    def build():
        w3 = w_lp.view(w_lp.size(0), -1, C)          # [in, S, out]
        img = w3.permute(1, 0, 2) if trans else w3.permute(1, 2, 0)
        return (w_lp, img[:, :, slot_k_order(w_lp.device)].contiguous())
    return cached(_slot_img_key(w_lp, trans), build)[1]


def gemm_spmm(op, x, w, w_lp, out_channels, bias=None, relu=False,
              loop_key=None, passthrough=False):
    r"""``act(op @ (x @ w).view(-1, out_channels) + bias)``.

    ``w [in, S * out]`` is the fp32 stacked weight (receives the gradient),
    ``w_lp`` its compute-dtype copy; ``op`` maps the ``S`` slot rows of
    every node to the output rows.  ``loop_key`` enables loop-shared gradient
    accumulation inside :func:`~..runtime.loopgrad.loop_scope`.
    ``passthrough`` returns ``(out, x')`` where ``x'`` aliases ``x``: give
    ``x'`` to x's other consumers and their gradient is accumulated inside
    this node's backward (fused into the slot conv epilogue).
    ``passthrough='cat'`` additionally promises that ``x'`` feeds exactly
    one ``torch.cat`` (nothing else), which lets the backward accumulate
    into that gradient slice in place.
    """
    from ..runtime import loopgrad
    assert x.dim() == 2 and x.size(0) * (w.size(1) // out_channels) == \
        op.num_cols, (x.shape, w.shape, op)
    loop = loopgrad.group(('gemm_spmm', ) + loop_key) \
        if loop_key is not None else None
    with torch.autocast(device_type='cuda' if x.is_cuda else 'cpu',
                        enabled=False):
        return _GemmSpMM.apply(x, w, w_lp.detach(), bias, op, relu,
                               out_channels, loop, passthrough)
