"""Mixed-precision GEMM with split-K weight gradients.

The encoder GEMMs are plain library GEMMs (hipBLASLt via ``torch.matmul``),
but their *weight-gradient* products have a tiny output and a huge reduction
dimension: for psi_2's SplineConv, ``dW = X^T dY`` is ``[128, 9216] x
[9216, 3328]`` - 52 output tiles for 256 CUs.  hipBLASLt's heuristic picks a
non-split kernel (~76 us, 100 TF/s measured on MI355X).  Splitting K into a
batch of ``s`` GEMMs with fp32 outputs and summing them runs the same product
in ~33 us (s=16) and accumulates directly in fp32 for the fp32 master weight
(no bf16 rounding of the weight gradient).  Measurements:
``tools/gemm_bench.py`` / ``profiles/gemm_bench_r1.txt``.

``mixed_matmul(x, w, w_lp)`` computes ``x @ w`` in the autocast dtype with
``w_lp`` an (optionally cached) low-precision copy of the fp32 parameter
``w``; gradients flow to ``x`` and to the fp32 ``w``.  Inside a
:func:`~..runtime.loopgrad.loop_scope` the weight/bias gradients of repeated
uses are accumulated in place by the split-K combine / column-sum kernels.
"""
import os

import torch

from . import _backend
from ..runtime import loopgrad
from ..runtime.cache import cached

def _rows16(t):
    return (t.dim() == 2 and t.dtype == torch.float32 and t.stride(1) == 1
            and t.size(1) % 4 == 0 and t.stride(0) % 4 == 0 and
            t.data_ptr() % 16 == 0)


def nt_f32_supported(parts, bt):
    """``[parts] @ bt^T`` on the chunked NT GEMM (``csrc/hip/gemm_f32.hip``):
    fp32 device operands with 16-byte rows, output width a multiple of 4
    (a partial last tile column block is masked), K <= 3072."""
    if not (parts and _backend.use_hip(parts[0]) and _rows16(bt) and
            bt.size(0) % 4 == 0):
        return False
    M = parts[0].size(0)
    chunks = 0
    for p in parts:
        if not (_rows16(p) and p.size(0) == M):
            return False
        chunks += (p.size(1) + 127) // 128
    return (chunks <= 24 and bt.size(1) == sum(p.size(1) for p in parts)
            and M > 0)


# fp32 products of the chunked NT GEMM on the bf16 matrix cores as bf16x6
# (three bf16 terms per operand, six products, two fp32 accumulators; error
# below the exact-f32 MFMA chain's, tests/test_gemm_f32.py) - the same
# switch as ops/slot_gemm.py::X6 (DGMC_AMD_X6=0: exact-f32 kernels).
NT_X6 = os.environ.get('DGMC_AMD_X6', '1') == '1'
# bf16x6 NT kernel with the fragment splits scheduled against the previous
# block's MFMAs (csrc/hip/gemm_f32.hip, SCHED; tools/bench_gemm_nt.py: 2-10 %
# faster on the DBP15K psi_1 shapes, bit-identical).
NT_SCHED = 1


def nt_f32(parts, bt, bias=None, relu=False, out=None, x6=None,
           accumulate=False, sched=None):
    """``act([parts] @ bt^T + bias)`` (fp32, no autograd; parts read in
    place, never concatenated).  ``x6``: bf16x6 products (default
    :data:`NT_X6`) or the exact-f32 chain.  ``accumulate``: add the product
    into ``out`` (beta = 1) instead of overwriting it."""
    b = None
    if bias is not None:
        b = bias.detach()
        if not b.is_contiguous():
            b = b.contiguous()
    return _backend.ops().gemm_nt_f32(list(parts), bt, b, relu, out,
                                      NT_X6 if x6 is None else bool(x6),
                                      bool(accumulate),
                                      NT_SCHED if sched is None else
                                      int(sched))


def _tn_part_ok(t, K):
    return (t.dim() == 2 and t.size(0) == K and t.dtype == torch.float32 and
            t.is_cuda and t.stride(1) == 1 and t.size(1) % 4 == 0 and
            (t.stride(0) % 4 == 0 or K <= 1) and t.data_ptr() % 16 == 0)


def tn_f32_supported(a_parts, b_parts):
    """``[a_parts]^T [b_parts]`` on the split-K TN GEMM
    (``csrc/hip/gemm_tn.hip``): fp32 device parts ``[K, w]`` with 16-byte
    rows, widths multiples of 4, at most 8 parts per operand."""
    if not (a_parts and b_parts and len(a_parts) <= 8 and len(b_parts) <= 8
            and _backend.use_hip(a_parts[0])):
        return False
    K = a_parts[0].size(0)
    return all(_tn_part_ok(t, K) for t in list(a_parts) + list(b_parts))


def tn_f32(a_parts, b_parts, out=None, accumulate=False, x6=None, cfg=0):
    """``[a_parts]^T [b_parts]`` (fp32 ``[M, N]``; written, or added into
    ``out``).  bf16x6 products unless ``x6=False`` / ``DGMC_AMD_X6=0``.
    ``cfg``: kernel staging variant (measurement hook; 0 = default)."""
    return _backend.ops().gemm_tn_f32(list(a_parts), list(b_parts), out,
                                      bool(accumulate),
                                      NT_X6 if x6 is None else bool(x6), 0,
                                      int(cfg))


class _LinearParts(torch.autograd.Function):
    """``torch.cat(parts, -1) @ W^T + b`` without the concatenation: the
    chunked NT GEMM (bf16x6 unless ``DGMC_AMD_X6=0``) reads the parts in
    place.  Backward on the same kernels: the input gradients of the parts
    that need one are ONE NT product ``g W[:, lo:hi]`` (handed out as column
    slices), the weight gradient ONE split-K TN product ``g^T [parts]``."""

    @staticmethod
    def forward(ctx, weight, bias, *parts):
        w = weight.detach()
        out = nt_f32(parts, w, bias)
        ctx.widths = [p.size(1) for p in parts]
        ctx.has_bias = bias is not None
        ctx.save_for_backward(weight, *parts)
        return out

    @staticmethod
    def backward(ctx, g):
        weight, *parts = ctx.saved_tensors
        g = g.contiguous()
        need = [ctx.needs_input_grad[2 + i] for i in range(len(parts))]
        grads = [None] * len(parts)
        offs = [0]
        for w in ctx.widths:
            offs.append(offs[-1] + w)
        if any(need):
            lo = offs[need.index(True)]
            hi = offs[len(need) - need[::-1].index(True)]
            wt = weight.detach().t().contiguous()        # [in, out]
            if nt_f32_supported([g], wt[lo:hi]):
                dx = nt_f32([g], wt[lo:hi])
            else:
                dx = g @ weight[:, lo:hi]
            for i, w in enumerate(ctx.widths):
                if need[i]:
                    grads[i] = dx[:, offs[i] - lo:offs[i] - lo + w]
        gw = gb = None
        if ctx.needs_input_grad[0]:
            if tn_f32_supported([g], parts):
                gw = tn_f32([g], parts)
            else:
                gw = torch.cat([matmul_tn_fp32(g, p.contiguous())
                                for p in parts], 1)
        if ctx.has_bias and ctx.needs_input_grad[1]:
            gb = _col_sum(g)
        return (gw, gb) + tuple(grads)


def linear_parts(parts, weight, bias=None):
    """``F.linear(torch.cat(parts, -1), weight, bias)``; on the GPU (fp32)
    the parts are read in place by one chunked NT GEMM (bf16x6 unless
    ``DGMC_AMD_X6=0``; no concatenation)."""
    parts = list(parts)
    ok = nt_f32_supported(parts, weight) and (
        bias is None or (bias.dtype == torch.float32 and
                         bias.is_contiguous() and bias.data_ptr() % 16 == 0))
    if not ok:
        return linear(torch.cat(parts, -1), weight, bias)
    if torch.is_grad_enabled() and (
            weight.requires_grad or any(p.requires_grad for p in parts) or
            (bias is not None and bias.requires_grad)):
        return _LinearParts.apply(weight, bias, *parts)
    return nt_f32(parts, weight, bias)


def _split_factor(m, n, k):
    elems = m * n
    if elems >= (4 << 20) or k < 2048:
        return 1
    # Small outputs get many splits: 64 x [384, 128] partials of the 92k-row
    # consensus weight gradient run 55 us vs 69 us at 16 (tools/
    # bench_wgrad_tn.py).
    s = 8 if elems >= (1 << 20) else (16 if elems >= (1 << 17) else 64)
    while s > 1 and k // s < 512:
        s //= 2
    return s


def _dense_tn_ok(a, b):
    if not (a.is_cuda and _backend.use_hip(a)):
        return False
    K, M = a.shape
    N = b.shape[1]
    return (a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and
            M % 128 == 0 and N % 128 == 0 and M * N <= 512 * 512 and
            K >= 1024 and b.shape[0] == K and
            all(t.stride(1) == 1 and t.stride(0) % 8 == 0 and
                t.data_ptr() % 16 == 0 for t in (a, b)))


def matmul_tn_fp32(a, b, out=None, accumulate=False):
    """``a^T @ b`` (``a [K, M]``, ``b [K, N]``) with fp32 output, split-K.

    With ``out`` (fp32 ``[M, N]``) the product is written (or added, when
    ``accumulate``) there; on the GPU the split-K combine does the
    accumulation, so it costs no extra kernel.
    """
    K, M = a.shape
    N = b.shape[1]
    if _dense_tn_ok(a, b):
        # Small bf16 outputs: the MFMA TN kernel (ops/dense.py::dense_wgrad)
        # instead of a skinny split-K library GEMM.
        from .dense import dense_wgrad
        return dense_wgrad([a], [b], out=out, accumulate=accumulate)
    if _dense_tn_f32_ok(a, b):
        # fp32: the LDS-DMA MFMA TN kernel over balanced row ranges (a
        # batched split-K library GEMM with M x N = 256 x 256 ran as 16
        # workgroups: 152 us for psi_1's final Linear).
        from .dense import _seg01
        res = _backend.ops().dense_wgrad_f32([a], 1, [b],
                                             _seg01(K, a.device))
    elif tn_f32_supported([a], [b]):
        # fp32, any width: the split-K TN MFMA kernel (csrc/hip/gemm_tn.hip;
        # the deterministic fold writes / adds ``out`` directly).
        return tn_f32([a], [b], out=out, accumulate=accumulate)
    elif not a.is_cuda:
        res = a.float().t() @ b.float()
    else:
        # (low-precision inputs accumulate into fp32; fp32 / fp64 - the
        # reference-mode oracle - stay in their own dtype)
        low = a.dtype in (torch.bfloat16, torch.float16)
        s = _split_factor(M, N, K)
        if s == 1:
            res = torch.mm(a.t(), b, out_dtype=torch.float32) if low \
                else a.t() @ b
        else:
            k = K // s
            main = k * s
            a3 = a[:main].view(s, k, M).transpose(1, 2)
            b3 = b[:main].view(s, k, N)
            if not low:
                part = torch.bmm(a3, b3)
            else:
                part = torch.bmm(a3, b3, out_dtype=torch.float32)
            if main < K:   # fold the remainder rows into the first split
                tail = torch.mm(a[main:].t(), b[main:],
                                out_dtype=torch.float32) if low \
                    else a[main:].t() @ b[main:]
                part[0].add_(tail)
            if _backend.hip_available() and part.dtype == torch.float32:
                if out is None:
                    out = torch.empty((M, N), dtype=torch.float32,
                                      device=a.device)
                    accumulate = False
                _backend.ops().reduce_add_rows(part, out, accumulate)
                return out
            res = part.sum(0)
    if out is None:
        return res
    if accumulate:
        out.add_(res)
    else:
        out.copy_(res)
    return out


def _dense_tn_f32_ok(a, b):
    return (_backend.use_hip(a) and a.dtype == torch.float32 and
            b.dtype == torch.float32 and a.dim() == 2 and b.dim() == 2 and
            a.is_contiguous() and b.is_contiguous() and
            a.size(0) == b.size(0) and a.size(0) % 32 == 0 and
            a.size(1) % 128 == 0 and a.size(1) <= 512 and
            b.size(1) % 128 == 0 and a.data_ptr() % 16 == 0 and
            b.data_ptr() % 16 == 0)


class _MixedMatmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, w_lp, bias, loop):
        xc = x if x.dtype == w_lp.dtype else x.to(w_lp.dtype)
        # w = weight.t() of an fp32 [out, in] parameter: the exact-f32
        # chunked NT kernel reads the weight in place (GIN / MLP / encoder
        # Linears, /root/reference/dgmc/models/gin.py:49, mlp.py:35)
        wt = w_lp.t() if w_lp.dim() == 2 else None
        if wt is not None and xc.dtype == torch.float32 and \
                wt.is_contiguous() and nt_f32_supported([xc], wt) and \
                (bias is None or (bias.dtype == torch.float32 and
                                  bias.is_contiguous() and
                                  bias.data_ptr() % 16 == 0)):
            out = nt_f32([xc], wt, bias)
        elif bias is not None:
            # Bias in the GEMM epilogue (hipBLASLt), cast once per forward.
            b_lp = bias if bias.dtype == w_lp.dtype else cached(
                ('bias_lp', id(bias), w_lp.dtype),
                lambda: (bias, bias.detach().to(w_lp.dtype)))[1]
            out = torch.addmm(b_lp, xc, w_lp)
        else:
            out = xc @ w_lp
        ctx.save_for_backward(xc, w_lp)
        ctx.x_dtype, ctx.w_dtype = x.dtype, w.dtype
        ctx.w_transposed = w.dim() == 2 and w.size(0) > 1 and \
            w.size(1) > 1 and w.stride(0) == 1 and w.stride(1) == w.size(0)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.loop = loop
        ctx.idx = loop.register() if loop is not None else None
        return out

    @staticmethod
    def backward(ctx, g):
        xc, w_lp = ctx.saved_tensors
        g = g.contiguous()
        if g.dtype != w_lp.dtype:
            g = g.to(w_lp.dtype)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            # dX = g W: NT with Bt = W^T = w_lp ([in, out]); a transposed
            # view (linear's weight.t()) is made contiguous (<= 1 MB copy)
            wb = w_lp if (w_lp.dim() != 2 or w_lp.is_contiguous() or
                          w_lp.numel() > (1 << 18)) else w_lp.contiguous()
            if g.dtype == torch.float32 and wb.dim() == 2 and \
                    wb.is_contiguous() and nt_f32_supported([g], wb):
                gx = nt_f32([g], wb).to(ctx.x_dtype)
            else:
                gx = (g @ w_lp.t()).to(ctx.x_dtype)
        need_w = ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[3]
        loop = ctx.loop
        if loop is None:
            if need_w and ctx.w_transposed:
                # w = weight.t(): produce the gradient in the parameter's own
                # layout ([out, in] contiguous) and hand back its transpose,
                # so AccumulateGrad keeps it without a layout copy.
                gw = matmul_tn_fp32(g, xc.contiguous()).to(ctx.w_dtype).t()
            elif need_w:
                gw = matmul_tn_fp32(xc.contiguous(), g).to(ctx.w_dtype)
            if need_b:
                gb = _col_sum(g).to(ctx.bias_dtype)
            return gx, gw, None, gb, None
        # Kept: reference x and g per use; ONE long-K GEMM (and column sum)
        # over the concatenation when the last use arrives.
        loop.keep('x', ctx.idx, xc)
        loop.keep('g', ctx.idx, g)
        if loop.arrive():
            G = loop.kept('g')
            if need_w:
                gw = matmul_tn_fp32(loop.kept('x').contiguous(), G)
                gw = gw.to(ctx.w_dtype)
            if need_b:
                gb = _col_sum(G).to(ctx.bias_dtype)
            loop.release()
        return gx, gw, None, gb, None


# (= csrc/hip/elementwise.hip::kMaxColBlocks)
_COL_MAX_BLOCKS = 1024


def col_partial_rows(rows):
    """Per-block partial rows of the HIP column reductions (keep in sync
    with csrc/hip/elementwise.hip::colsum_blocks)."""
    return max(1, min((rows + 15) // 16, _COL_MAX_BLOCKS))


def loop_col_sum(loop, name, idx, src):
    """Deposit ``src.sum(0)`` of loop use ``idx`` as per-block partials in
    stack ``name`` (folded once by :func:`loop_col_total`)."""
    if _backend.use_hip(src):
        slot = loop.slot(name, idx, (col_partial_rows(src.size(0)),
                                     src.size(1)), torch.float32, src.device)
        _backend.ops().col_sum(src.contiguous(), None, False, slot)
    else:
        loop.add_to(name, src.float().sum(0))


def loop_col_total(loop, name):
    """Total of the contributions deposited by :func:`loop_col_sum`."""
    if name in loop._stacks:
        st = loop.stack(name)
        return _col_sum(st.view(-1, st.size(-1)))
    return loop.get_acc(name)


def _col_sum(src, out=None, accumulate=False):
    """Column sum of a 2-D tensor in fp32 (optionally into ``out``)."""
    if _backend.use_hip(src):
        return _backend.ops().col_sum(src.contiguous(), out, accumulate)
    res = src.float().sum(0)
    if out is None:
        return res
    if accumulate:
        out.add_(res)
    else:
        out.copy_(res)
    return out


def compute_dtype(x):
    dev = 'cuda' if x.is_cuda else 'cpu'
    if torch.is_autocast_enabled(dev):
        return torch.get_autocast_dtype(dev)
    return x.dtype


def mixed_matmul(x, w, w_lp=None, bias=None, loop_key=None):
    r"""``x @ w (+ bias)`` in the autocast dtype; fp32 gradient for ``w``.

    Args:
        x: ``[N, K]`` activations.
        w: ``[K, M]`` fp32 weight (receives the gradient).
        w_lp: optional pre-cast copy of ``w`` in the compute dtype.
        bias: optional ``[M]``.
        loop_key: identifies the op instance inside a
            :func:`~..runtime.loopgrad.loop_scope` (gradient accumulation
            across loop iterations).
    """
    dtype = compute_dtype(x)
    if w_lp is None:
        w_lp = w.detach().to(dtype)
    loop = loopgrad.group(('mm', ) + loop_key) if loop_key is not None \
        else None
    with torch.autocast(device_type='cuda' if x.is_cuda else 'cpu',
                        enabled=False):
        return _MixedMatmul.apply(x, w, w_lp.detach(), bias, loop)


def lowp_weight_t(weight, dtype):
    """``weight.t()`` cast to ``dtype``, memoised per forward scope for
    parameters (the cache entry keeps the parameter alive, so its ``id``
    cannot be recycled within the scope)."""
    if not isinstance(weight, torch.nn.Parameter):
        return weight.detach().t().to(dtype)
    return cached(('w_lp_t', id(weight), dtype),
                  lambda: (weight, weight.detach().t().to(dtype)))[1]


def linear(x, weight, bias=None):
    """``F.linear`` with split-K fp32 weight gradients (``weight [out, in]``).
    Parameters reused inside a loop scope accumulate their gradient in
    place."""
    w_lp = lowp_weight_t(weight, compute_dtype(x))
    key = (id(weight), ) if isinstance(weight, torch.nn.Parameter) else None
    return mixed_matmul(x, weight.t(), w_lp, bias, loop_key=key)
