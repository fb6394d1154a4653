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
``w``; gradients flow to ``x`` and to the fp32 ``w``.
"""
import torch

from . import _backend


def _split_factor(m, n, k):
    elems = m * n
    if elems >= (4 << 20) or k < 2048:
        return 1
    s = 8 if elems >= (1 << 20) else 16
    while s > 1 and k // s < 512:
        s //= 2
    return s


def matmul_tn_fp32(a, b):
    """``a^T @ b`` (``a [K, M]``, ``b [K, N]``) with fp32 output, split-K."""
    K, M = a.shape
    N = b.shape[1]
    s = _split_factor(M, N, K) if a.is_cuda else 1
    if not a.is_cuda:
        return a.float().t() @ b.float()
    if s == 1:
        return torch.mm(a.t(), b, out_dtype=torch.float32) \
            if a.dtype != torch.float32 else a.t() @ b
    k = K // s
    main = k * s
    a3 = a[:main].view(s, k, M).transpose(1, 2)
    b3 = b[:main].view(s, k, N)
    if a.dtype == torch.float32:
        part = torch.bmm(a3, b3)
    else:
        part = torch.bmm(a3, b3, out_dtype=torch.float32)
    if _backend.hip_available():
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
        _backend.ops().reduce_add_rows(part, out, False)
    else:
        out = part.sum(0)
    if main < K:
        tail = a[main:].t() @ b[main:]
        out = out + tail.float()
    return out


class _MixedMatmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, w_lp, bias):
        xc = x if x.dtype == w_lp.dtype else x.to(w_lp.dtype)
        out = xc @ w_lp
        if bias is not None:
            out = out + bias.to(out.dtype)
        ctx.save_for_backward(xc, w_lp)
        ctx.x_dtype, ctx.w_dtype = x.dtype, w.dtype
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        return out

    @staticmethod
    def backward(ctx, g):
        xc, w_lp = ctx.saved_tensors
        g = g.contiguous()
        if g.dtype != w_lp.dtype:
            g = g.to(w_lp.dtype)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = (g @ w_lp.t()).to(ctx.x_dtype)
        if ctx.needs_input_grad[1]:
            gw = matmul_tn_fp32(xc.contiguous(), g).to(ctx.w_dtype)
        if ctx.has_bias and ctx.needs_input_grad[3]:
            gb = g.float().sum(0).to(ctx.bias_dtype)
        return gx, gw, None, gb


def compute_dtype(x):
    dev = 'cuda' if x.is_cuda else 'cpu'
    if torch.is_autocast_enabled(dev):
        return torch.get_autocast_dtype(dev)
    return x.dtype


def mixed_matmul(x, w, w_lp=None, bias=None):
    r"""``x @ w (+ bias)`` in the autocast dtype; fp32 gradient for ``w``.

    Args:
        x: ``[N, K]`` activations.
        w: ``[K, M]`` fp32 weight (receives the gradient).
        w_lp: optional pre-cast copy of ``w`` in the compute dtype.
        bias: optional ``[M]``.
    """
    dtype = compute_dtype(x)
    if w_lp is None:
        w_lp = w.detach().to(dtype)
    with torch.autocast(device_type='cuda' if x.is_cuda else 'cpu',
                        enabled=False):
        return _MixedMatmul.apply(x, w, w_lp.detach(), bias)


def linear(x, weight, bias=None):
    """``F.linear`` with split-K fp32 weight gradients (``weight [out, in]``)."""
    return mixed_matmul(x, weight.t(), None, bias)
