"""fp32 SplineConv on the (node, slot) pairs the edges use
(csrc/hip/slot_gemm.hip).

Reference: ``/root/reference/dgmc/models/spline.py:21,49`` (PyG SplineConv
over torch_spline_conv, fp32).  With ``A [N, N*S]`` the layer's message
operator (columns ``j*S + k``: source ``j``, B-spline slot ``k``, root =
slot ``S-1``; :func:`~.plans.spline_plan`)::

    out = act(A (X W) + bias)

The dense form multiplies every node by every slot's weight; only 42 % of
those ``(j, k)`` pairs carry an entry on PascalVOC-shaped batches, so this
path forms exactly those rows (``Y_c = X[src] W_slot``, a segmented gathered
GEMM on fp32 MFMA) and aggregates them with the CSR SpMM over ``A``'s
re-indexed columns.  Backward: ``dY_c = A^T g'`` (row-mapped SpMM over the
assembled transpose), ``dX = sum_k (dY_c W_k^T)`` (same GEMM kernel with
``W^T`` + a per-node gather-sum), ``dW_k = X[src]^T dY_c`` (gathered TN
GEMM, per-slot fixed-order fold).  Everything is exact fp32 (the MFMA is a
k-ordered ``fmaf`` chain) and deterministic.

Inside a :func:`~..runtime.loopgrad.loop_scope` (psi_2 in the consensus
loop) the weight gradient of all uses is ONE launch over the kept ``(X_u,
dY_c,u)`` pairs.
"""
import os
import weakref

import torch

from . import _backend
from ..runtime.cache import cached
from .gemm import col_partial_rows, loop_col_total

BM = 128                      # compact tile unit (slot_gemm.hip)
SEG = 256                     # slot segment alignment (256-row x6 tiles)
MAX_USES = 16                 # pointer table of slot_wgrad_f32
ENABLED = True                # (tests compare against the GEMM + SpMM path)
# fp32 products on the bf16 matrix cores ("bf16x6", csrc/hip/slot_gemm_x6.hip):
# every operand split into three bf16 terms, six products, two fp32
# accumulators - max error vs fp64 BELOW the exact-f32 MFMA kernels on every
# headline shape (tests/test_slot_gemm_x6.py).
X6 = os.environ.get('DGMC_AMD_X6', '1') == '1'
# Under in-step data parallelism a single-use weight gradient of at least
# PIECE_BYTES (psi_1 layer 0: 25 MiB, the last gradient of the backward) is
# produced in PIECES slot ranges and each piece's all-reduce starts as soon
# as it is written (parallel/ddp.py::grad_sink), instead of the whole bucket
# waiting for the last launch.  Without a reducer one launch is cheaper
# (+0.03 ms per PascalVOC step for the extra fold); PIECES_ALWAYS=1 pieces
# regardless (tests compare a one-rank RCCL run bit-for-bit with that).
PIECES = 2
PIECES_ALWAYS = os.environ.get('DGMC_AMD_WGRAD_PIECES_ALWAYS', '0') == '1'
PIECE_BYTES = 8 << 20
# bf16x6 backward on fp32 dY_c (split inside the dX / dW kernels' LDS
# staging) instead of the rowmap SpMM writing three bf16 planes.
F32DY = True
# Rowmap SpMM entries from a per-step inline (col, val) table.
ROWMAP_ELL = True
# bf16x6 forward on fp32 X (gathered rows split in the GEMM's staging) for
# in <= F32X_KMAX (tools/bench_slot_gemm_x6.py with the 32 x 128 wave tiles
# of the fp32-A kernel: 128->128 42.9 -> 38.0 us, 256->256 115 -> 113,
# 1024->256 351 -> 346 vs bf16 planes; the earlier 64 x 64 tiles were slower
# than planes beyond K = 128).
F32X = True
F32X_KMAX = 4096
# (The weight gradient keeps reading bf16 planes of X: an fp32-X weight
# gradient measured slower - PascalVOC 5.57 -> 5.66 ms, both operands'
# column reads + splits cost more than the 1/3 of X traffic they save - and
# was removed in round 6.)


class CompactPlan(object):
    """Used-column layout of one operator (built once, cached on it)."""

    def __init__(self, op, S):
        N = op.num_cols // S
        ncols = op.num_cols
        cap = op.col.numel()
        P_cap = (min(cap, ncols) + S * SEG + SEG - 1) // SEG * SEG
        (self.src, self.seg, self.col_c, self.posmap, self.cinv,
         self.counts) = _backend.ops().slot_compact_plan(
             op.rowptr, op.col, N, S, P_cap)
        self.S, self.N, self.P_cap = S, N, P_cap


def dx_tiles(plan, row0, unit=BM):
    """Row-tile list (``unit``-row tiles) of the dX pass for sources
    ``j >= row0`` (cached)."""
    cache = plan.__dict__.setdefault('_dx_tiles', {})
    t = cache.get((row0, unit))
    if t is None:
        t = cache[(row0, unit)] = _backend.ops().slot_dx_tiles(
            plan.src, plan.seg, plan.N, row0, plan.P_cap, unit)
    return t


def rowmap_ranges(plan, At):
    """A^T entries of every compact row, built once per plan and transposed
    operator (shared by the step's rowmap SpMMs): the ``[P_cap, 8]`` inline
    entry table (``ROWMAP_ELL``: up to three (col, val) pairs per row, one
    dependent load round fewer) or ``[P_cap, 2]`` int32 ranges."""
    cache = plan.__dict__.setdefault('_ranges', {})
    key = (At.rowptr.data_ptr(), At.col.data_ptr(), At.val.data_ptr(),
           ROWMAP_ELL)
    r = cache.get(key)
    if r is None:
        ops = _backend.ops()
        r = cache[key] = ops.slot_rowmap_ell(
            At.rowptr, At.col, At.val, plan.cinv) if ROWMAP_ELL else \
            ops.slot_rowmap_ranges(At.rowptr, plan.cinv)
    return r


def compact_plan(op, S):
    cache = op.__dict__.setdefault('_compact_plan', {})
    p = cache.get(S)
    if p is None:
        p = cache[S] = CompactPlan(op, S)
    return p


def supported(op, x, weight, root):
    """Shapes / dtypes served by the fp32 slot GEMM path."""
    if not (ENABLED and _backend.use_hip(x) and x.dtype == torch.float32 and
            weight.dtype == torch.float32 and weight.dim() == 3):
        return False
    S = weight.size(0) + (1 if root is not None else 0)
    cin, cout = weight.size(1), weight.size(2)
    return (cin % 128 == 0 and cout % 128 == 0 and S <= 64 and
            x.dim() == 2 and x.size(1) == cin and
            op.num_cols == x.size(0) * S and op.num_rows == x.size(0))


def weight_grad(xs, dys, plan, cin, cout):
    """``dW [S, in, out]`` = ``sum_u X_u[src]^T dY_c,u`` per slot: balanced
    work items (one round of resident workgroups for a single 128x128 output
    tile, two otherwise), per-item partials folded in item order."""
    ops = _backend.ops()
    # Rounds of resident workgroups the items are sized for, by output tiles
    # (tools/bench_slot_gemm.py sweep, 1 / 2 / 3 / 4 / 6 rounds: 128->128
    # 387 / 407 / 420 / 440 / 467 us, 256->256 178 / 174 / 179 / 184 / 205
    # us, 1024->256 737 / 720 / 599 / 623 / 573 us; 8 / 12 / 16 rounds: 587
    # / 623 / 653 us).
    tiles = (cin // 128) * (cout // 128)
    rounds = 1 if tiles == 1 else (2 if tiles <= 4 else 6)
    out = None
    for i in range(0, len(xs), MAX_USES):
        part = ops.slot_wgrad_f32(list(xs[i:i + MAX_USES]),
                                  list(dys[i:i + MAX_USES]), plan.src,
                                  plan.seg, rounds)
        out = part if out is None else out.add_(part)
    return out


def _x6_rounds(tiles):
    """Rounds of resident workgroups the bf16x6 weight gradient's slot-range
    items are sized for (more items: better balance, more partial bytes
    for the fold)."""
    if tiles == 1:
        return X6_WGRAD_ROUNDS_ONE
    return 2 if tiles <= 4 else X6_WGRAD_ROUNDS_BIG


X6_WGRAD_ROUNDS_BIG = 6
# (single-tile shapes, psi_2's 10-use gradient: 1 / 2 / 3 rounds measured
# 5.637 / 5.658 / 5.68 ms per PascalVOC step)
X6_WGRAD_ROUNDS_ONE = 1


def weight_grad_x6(x3s, dy3s, plan, cin, cout):
    """:func:`weight_grad` on bf16x6 operand planes (``[3, N, in]`` /
    ``[3, P_cap, out]``)."""
    ops = _backend.ops()
    tiles = (cin // 128) * (cout // 128)
    rounds = _x6_rounds(tiles)
    out = None
    for i in range(0, len(x3s), MAX_USES):
        part = ops.slot_wgrad_x6(list(x3s[i:i + MAX_USES]),
                                 list(dy3s[i:i + MAX_USES]), plan.src,
                                 plan.seg, rounds)
        out = part if out is None else out.add_(part)
    return out


def _x6_images(weight, root, need_dx=True):
    """bf16x6 weight images of the forward (W^T) and the input gradient (W,
    only when ``need_dx``: psi_1 layer 0's input needs no gradient), built
    once per forward scope and shared by the consensus loop's uses."""
    ops = _backend.ops()
    w = weight.detach().contiguous()
    r = root.detach().contiguous() if root is not None else None
    return (cached(('slot_wt3', id(weight)),
                   lambda: ops.slot_weight_x3(w, r, True)),
            cached(('slot_w3', id(weight)),
                   lambda: ops.slot_weight_x3(w, r, False))
            if need_dx else None)


class _SlotGemmSpMM(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, weight, root, bias, op, relu, loop, passthrough,
                dx_row0=0, planes_out=False, uses=None):
        S = weight.size(0) + (1 if root is not None else 0)
        plan = compact_plan(op, S)
        xc = x.contiguous()
        ops = _backend.ops()
        ctx.x6 = X6
        if X6:
            # bf16x6: X split once (the planes are also the weight
            # gradient's operand), weight images once per forward scope.
            wt3, ctx.w3 = _x6_images(weight, root, ctx.needs_input_grad[0])
            # (planes written by the producing SpMM when it was another
            # slot conv; valid while x is unmodified)
            pl = getattr(x, '_dgmc_x6', None)
            planes = pl[0] if (pl is not None and pl[1] == x._version and
                               tuple(pl[0].shape) == (3, ) + tuple(x.shape)) \
                else None
            if F32X and x.size(1) <= F32X_KMAX:
                if xc.data_ptr() % 16 != 0:
                    xc = xc.clone()          # (16-byte row DMA)
                # The GEMM gathers fp32 X rows and splits them in its LDS
                # staging (4 instead of 6 bytes per gathered element); the
                # weight gradient reads X's planes.
                Y = ops.slot_gemm_x6(xc, plan.src, plan.seg, wt3, True, None)
                if planes is None and (ctx.needs_input_grad[1] or (
                        root is not None and ctx.needs_input_grad[2])):
                    planes = ops.split3(xc)
                xc = planes
            else:
                xc = planes if planes is not None else ops.split3(xc)
                Y = ops.slot_gemm_x6(xc, plan.src, plan.seg, wt3, True,
                                     None)
        else:
            # W^T images [S, out, in] (k-contiguous B operand), built once
            # per forward scope and shared by the consensus loop's uses.
            wt = cached(('slot_wt', id(weight)), lambda: ops.slot_weight_t(
                weight.detach().contiguous(),
                root.detach().contiguous() if root is not None else None))
            Y = ops.slot_gemm2(xc, plan.src, plan.seg, wt, None, True)
        if X6 and planes_out:
            # The consumer is another bf16x6 slot conv: the SpMM also
            # writes its operand planes (no split pass there).
            out, planes = ops.spmm_csr_planes(op.rowptr, plan.col_c, op.val,
                                              Y, bias, relu)
            out._dgmc_x6 = (planes, out._version)
        else:
            out = ops.spmm_csr(op.rowptr, plan.col_c, op.val, Y, None, None,
                               bias, relu, torch.float32)
        ctx.save_for_backward(xc, weight, root, out if relu else None)
        ctx.op, ctx.plan, ctx.relu, ctx.loop = op, plan, relu, loop
        # Forward uses of this weight in the current forward scope: the
        # pieced DP weight gradient writes the weight's flat gradient view
        # and starts its all-reduce, which is only valid for a weight used
        # once per step (a second use would add into the view in flight).
        ctx.uses = uses
        ctx.dx_row0 = int(dx_row0)
        ctx.has_root = root is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.idx = loop.register() if loop is not None else None
        # Fused ReLU / bias backward: the NEXT slot conv's gather-sum (the
        # dX producing this output's gradient) applies this layer's ReLU mask
        # and deposits its bias-gradient partials into this use's loop slot
        # (bit-identical to relu_bias_bwd; csrc/hip/slot_gemm.hip
        # sg_gather_sum_kernel<RB>).  ``out`` carries the hand-off record,
        # the consumer keeps the record of its input.
        ctx.rb = None
        if RB_FUSE and relu and loop is not None and ctx.x6:
            ctx.rb = _ReluBiasHandoff(out, loop, ctx.idx, ctx.bias_dtype
                                      is not None and ctx.needs_input_grad[3])
            out._dgmc_rb = ctx.rb
        ctx.in_rb = getattr(x, '_dgmc_rb', None)
        if passthrough:
            return out, x.view_as(x)
        return out

    @staticmethod
    def backward(ctx, grad, gpass=None):
        x, weight, root, out = ctx.saved_tensors
        nones = (None, ) * 7
        op, plan, loop, idx = ctx.op, ctx.plan, ctx.loop, ctx.idx
        ops = _backend.ops()
        need_b = ctx.bias_dtype is not None and ctx.needs_input_grad[3]
        if grad.stride(-1) != 1 or grad.stride(0) < grad.size(1) or \
                grad.dtype != torch.float32:
            grad = grad.float().contiguous()
        rb = ctx.rb
        if rb is not None and rb.accepts(grad):
            # ReLU mask applied and bias partials deposited by the consumer's
            # gather-sum
            g, db = grad, None
        else:
            part = loop.slot('b', idx, (col_partial_rows(grad.size(0)),
                                        grad.size(1)), torch.float32,
                             grad.device) if (loop is not None and need_b) \
                else None
            g, db = ops.relu_bias_bwd(grad, out if ctx.relu else grad,
                                      ctx.relu, torch.float32, None, False,
                                      part)
        if rb is not None:
            rb.g = None
        At = op.t()
        dyc = ops.slot_spmm_rowmap(At.rowptr, At.col, At.val, plan.cinv, g,
                                    plan.seg, rowmap_ranges(plan, At),
                                    ctx.x6 and not F32DY)
        gx = None
        if ctx.needs_input_grad[0] and ctx.x6:
            # dY_c planes straight from the rowmap SpMM; 256-row tiles of
            # the sources >= dx_row0 only.
            row0 = ctx.dx_row0
            Z = ops.slot_gemm_x6(dyc, plan.src, plan.seg, ctx.w3, False,
                                 dx_tiles(plan, row0, SEG) if row0 > 0
                                 else None)
            add = gpass if (gpass is not None and
                            gpass.dtype == torch.float32 and gpass.dim() == 2
                            and gpass.stride(1) == 1 and
                            gpass.stride(0) % 4 == 0 and
                            gpass.data_ptr() % 16 == 0) else None
            rb = ctx.in_rb
            if rb is not None and (gpass is None or add is not None):
                fused = rb.fuse_args(plan.N, Z.size(1), Z.device)
                if fused is not None:
                    gx = ops.slot_gather_sum(plan.posmap, Z, plan.N, plan.S,
                                             add, row0, *fused)
                    rb.hand(gx)
            if gx is None:
                gx = ops.slot_gather_sum(plan.posmap, Z, plan.N, plan.S, add,
                                         row0)
            if gpass is not None and add is None:
                gx = gx + gpass
        elif ctx.needs_input_grad[0]:
            # K = 128 (psi_2): the register-staged v1 kernel streams dY_c
            # faster than the LDS-DMA one (51 vs 57 us per call,
            # tools/bench_slot_gemm.py); longer K: v2.  Rows below
            # ``dx_row0`` (psi_2's random r_s half) need no input gradient:
            # only the row tiles of sources >= dx_row0 are multiplied.
            row0 = ctx.dx_row0 if weight.size(2) < 256 else 0
            wc = weight.contiguous()
            rc = root.contiguous() if root is not None else None
            if weight.size(2) >= 256:
                Z = ops.slot_gemm2(dyc, plan.src, plan.seg, wc, rc, False)
            else:
                Z = ops.slot_gemm(dyc, plan.src, plan.seg, wc, rc, True,
                                  dx_tiles(plan, row0) if row0 > 0 else None)
            add = gpass if (gpass is not None and
                            gpass.dtype == torch.float32 and gpass.dim() == 2
                            and gpass.stride(1) == 1 and
                            gpass.stride(0) % 4 == 0 and
                            gpass.data_ptr() % 16 == 0) else None
            gx = ops.slot_gather_sum(plan.posmap, Z, plan.N, plan.S, add,
                                     row0)
            if gpass is not None and add is None:
                gx = gx + gpass
        elif gpass is not None:
            gx = gpass
        need_w = ctx.needs_input_grad[1] or (ctx.has_root and
                                             ctx.needs_input_grad[2])
        cin, cout = weight.size(1), weight.size(2)
        gw = gr = gb = None
        wgrad = weight_grad_x6 if ctx.x6 else weight_grad
        if loop is None:
            if need_w and ctx.x6 and PIECES > 1 and \
                    weight.numel() * 4 >= PIECE_BYTES and \
                    ctx.needs_input_grad[1] and ctx.uses is not None and \
                    ctx.uses[0] == 1 and (PIECES_ALWAYS or
                                          _has_sink(weight)):
                gw, gr = _weight_grad_pieces(x, dyc, plan, weight, root,
                                             ctx.has_root and
                                             ctx.needs_input_grad[2])
                need_w = False
            elif need_w:
                dW = wgrad([x], [dyc], plan, cin, cout)
            if need_b:
                gb = db.to(ctx.bias_dtype)
        else:
            if need_w:
                loop.keep('x', idx, x)
                loop.keep('dy', idx, dyc)
            if not loop.arrive():
                return (gx, None, None, None) + nones
            if need_w:
                dW = wgrad(loop.kept_list('x'), loop.kept_list('dy'), plan,
                           cin, cout)
            if need_b:
                gb = loop_col_total(loop, 'b').to(ctx.bias_dtype)
            loop.release()
        if need_w:
            nw = weight.size(0)
            if ctx.needs_input_grad[1]:
                gw = dW[:nw]
            if ctx.has_root and ctx.needs_input_grad[2]:
                gr = dW[nw]
        return (gx, gw, gr, gb) + nones


# Fused ReLU / bias backward of a slot conv into the next slot conv's
# gather-sum (PascalVOC: psi_2 layer 0's relu_bias_bwd, 10 launches a step).
RB_FUSE = True


class _ReluBiasHandoff(object):
    """Hand-off record between a ReLU slot conv (producer) and the slot conv
    that consumes its output: the consumer's dX gather-sum writes the masked
    gradient ``g`` and the producer's bias partials; the producer's backward
    takes ``g`` as is only if autograd hands it over unchanged (same tensor,
    same version - no other consumer's gradient was added), and otherwise
    recomputes both (the ReLU mask is idempotent and the partials are
    overwritten, so the fallback stays exact)."""

    def __init__(self, out, loop, idx, need_b):
        self.out = weakref.ref(out)
        self.loop, self.idx, self.need_b = loop, idx, need_b
        self.g = None
        self.gv = None

    def fuse_args(self, N, C, device):
        out = self.out()
        if out is None or self.g is not None or out.dtype != torch.float32 \
                or not out.is_contiguous() or tuple(out.shape) != (N, C) or \
                out.data_ptr() % 16 != 0 or not (256 <= N <= 16384) or \
                not (64 <= C <= 256):
            return None
        shape = (col_partial_rows(N), C)
        part = self.loop.slot('b', self.idx, shape, torch.float32, device) \
            if self.need_b else torch.empty(shape, device=device)
        return out, part

    def hand(self, g):
        self.g, self.gv = g, g._version

    def accepts(self, grad):
        return self.g is not None and grad is self.g and \
            grad._version == self.gv


def _forward_uses(weight):
    """Shared per-forward-scope counter of ``weight``'s uses (``[n]``,
    final once the forward has run), or None outside a forward scope (then
    single use cannot be proven)."""
    from ..runtime.cache import in_forward_scope
    if not (in_forward_scope() and torch.is_grad_enabled()):
        return None
    cnt = cached(('slot_gemm_uses', id(weight)), lambda: [0])
    cnt[0] += 1
    return cnt


def _has_sink(weight):
    from ..parallel.ddp import grad_sink
    return grad_sink(weight) is not None


def _weight_grad_pieces(x3, dy3, plan, weight, root, need_root):
    """``dW`` of one use in ``PIECES`` slot ranges, each written into the
    weight's flat DP gradient view (when an in-step reducer owns it) and
    all-reduced right away; returns ``(gw, gr)``."""
    from ..parallel.ddp import grad_sink
    ops = _backend.ops()
    nw, cin, cout = weight.shape
    S = plan.S
    tiles = (cin // 128) * (cout // 128)
    rounds = _x6_rounds(tiles)
    sink = grad_sink(weight)
    if sink is not None and sink.is_pre_reduced(weight):
        raise RuntimeError('pieced weight gradient: the weight\'s flat '
                           'gradient is already being reduced this step')
    gw = sink.grad_view(weight) if sink is not None else \
        torch.empty_like(weight)
    gr = None
    per = cin * cout
    bounds = [nw * i // PIECES for i in range(PIECES)] + [S]
    for c in range(PIECES):
        s0, s1 = bounds[c], bounds[c + 1]
        part = ops.slot_wgrad_x6([x3], [dy3], plan.src, plan.seg[s0:s1 + 1],
                                 rounds)
        w1 = min(s1, nw)
        gw[s0:w1].copy_(part[:w1 - s0])
        if sink is not None:
            sink.reduce_piece(weight, s0 * per, w1 * per)
        if s1 > nw and need_root:
            gr = part[nw - s0]
    if sink is not None:
        sink.mark_reduced(weight)
    return gw, gr


def slot_gemm_spmm(op, x, weight, root, bias=None, relu=False, loop_key=None,
                   passthrough=False, dx_row0=0, planes_out=False):
    r"""``act(A (x @ [W_0 | .. | W_{K-1} | root]).view(-1, C) + bias)`` in
    fp32 on the used ``(node, slot)`` pairs only; ``weight [K, in, out]``,
    ``root [in, out]`` are read in place (reference checkpoint layout).
    ``passthrough`` returns ``(out, x')`` (``x'`` aliases ``x``; its
    gradient is added inside this op's dX kernel).  ``dx_row0``: the input
    gradient of rows ``< dx_row0`` is not needed (returned as zeros).
    ``planes_out``: the output feeds another slot conv - on the bf16x6 path
    the aggregation also writes its operand planes."""
    from ..runtime import loopgrad
    loop = loopgrad.group(('slot_gemm', ) + tuple(loop_key)) \
        if loop_key is not None else None
    # (counted here: inside Function.forward grad mode is off)
    uses = _forward_uses(weight) if (loop is None and
                                     weight.requires_grad) else None
    with torch.autocast(device_type='cuda', enabled=False):
        return _SlotGemmSpMM.apply(x, weight, root, bias, op, relu, loop,
                                   passthrough, dx_row0, planes_out, uses)
