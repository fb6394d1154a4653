"""Message-passing layers (PyG-free), each = one GEMM + one sparse operator.

* :class:`SplineConv` - PyG 1.4 ``SplineConv`` semantics as used at
  ``/root/reference/dgmc/models/spline.py:21,49`` (open B-splines,
  ``aggr='mean'``, root weight, bias; checkpoint keys ``weight
  [K, in, out]``, ``root [in, out]``, ``bias [out]`` plus the buffers
  ``kernel_size`` (int64) and ``is_open_spline`` (uint8)).
* :class:`GINConv` - PyG 1.4 ``GINConv(nn, train_eps=True)`` as used at
  ``/root/reference/dgmc/models/gin.py:22,49``:
  ``nn((1 + eps) x + sum_{j->i} x_j)`` with self-loops removed.

MI355X formulation: instead of per-edge weighting kernels (torch_spline_conv
runs one thread per (edge, channel) with atomicAdd backward), SplineConv is
``A_spline @ (x @ [W_0 | ... | W_24 | root])``: one large MFMA GEMM
(hipBLASLt, bf16 under autocast) followed by a single fused deterministic
gather-reduce kernel that applies basis weights, mean normalisation, the
root term, bias and (optionally) ReLU.  Its backward is the same kernel on
``A^T`` followed by two GEMMs; no float atomics.
"""
import torch
from torch.nn import Parameter

from ..ops import _backend
from ..ops import slot_gemm
from ..ops.plans import spline_plan, adjacency_plan
from ..ops.gemm import compute_dtype
from ..ops.sparse import SLOT_CONV, gemm_spmm, prime_slot_images, spmm
from ..runtime.cache import cached
from .inits import reset, uniform


def repeat(src, length):
    if isinstance(src, (list, tuple)):
        assert len(src) == length
        return list(src)
    return [src] * length


class _StackedSplineWeight(torch.autograd.Function):
    """``(w, w_lp)`` for :func:`~..ops.sparse.gemm_spmm` straight from the
    parameters (csrc/hip/weights.hip): ``w_lp [in, S * out]`` is the stacked
    low-precision GEMM operand written by ONE kernel (no fp32 permute / cat
    intermediates), ``w`` an fp32 placeholder of the same shape that only
    carries the stacked fp32 gradient back - mapped to ``weight`` / ``root``
    by one unpack kernel."""

    @staticmethod
    def forward(ctx, weight, root, dtype):
        w_lp = _backend.ops().spline_weight_pack(weight, root, dtype)
        ctx.K, ctx.has_root = weight.size(0), root is not None
        token = weight.new_empty(1).expand(w_lp.shape)
        ctx.takes_slot_major = True     # see backward
        ctx.slot_major = None
        ctx.mark_non_differentiable(w_lp)
        # w_lp never receives a gradient: do not materialise a zero one.
        ctx.set_materialize_grads(False)
        return token, w_lp

    @staticmethod
    def backward(ctx, g, _):
        # A slot-major [S, in, out] gradient deposited on this node by the
        # fused slot conv's loop fold (ops/sparse.py): weight / root are
        # views (AccumulateGrad steals them - no kernel).
        pend, ctx.slot_major = ctx.slot_major, None
        if g is None and pend is None:
            return None, None, None
        gw = gr = None
        if g is not None:
            gw, gr = _backend.ops().spline_weight_unpack(
                g.float().contiguous(), ctx.K, ctx.has_root)
        if pend is not None:
            pw, pr = pend[:ctx.K], pend[ctx.K] if ctx.has_root else None
            gw = pw if gw is None else gw + pw
            if ctx.has_root:
                gr = pr if gr is None else gr + pr
        return gw, (gr if ctx.has_root else None), None


class SplineConv(torch.nn.Module):
    r"""Spline-based convolution (Fey et al., CVPR 2018).

    Args:
        in_channels, out_channels (int): feature sizes.
        dim (int): pseudo-coordinate dimensionality.
        kernel_size (int or list): kernel size per dimension.
        is_open_spline (bool or list): open vs closed B-splines.
        degree (int): B-spline degree (1, 2 or 3).
        aggr (str): only ``'mean'`` (the reference configuration).
        root_weight (bool), bias (bool).
    """

    def __init__(self, in_channels, out_channels, dim, kernel_size,
                 is_open_spline=True, degree=1, aggr='mean',
                 root_weight=True, bias=True):
        super(SplineConv, self).__init__()
        assert aggr == 'mean', 'only mean aggregation is supported'
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.dim = dim
        self.degree = degree
        self.aggr = aggr

        kernel_size = torch.tensor(repeat(kernel_size, dim), dtype=torch.long)
        self.register_buffer('kernel_size', kernel_size)
        is_open_spline = torch.tensor(repeat(is_open_spline, dim),
                                      dtype=torch.uint8)
        self.register_buffer('is_open_spline', is_open_spline)
        self._ks = tuple(int(k) for k in kernel_size.tolist())
        self._open = tuple(int(v) for v in is_open_spline.tolist())

        K = int(kernel_size.prod().item())
        self.weight = Parameter(torch.Tensor(K, in_channels, out_channels))
        if root_weight:
            self.root = Parameter(torch.Tensor(in_channels, out_channels))
        else:
            self.register_parameter('root', None)
        if bias:
            self.bias = Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        size = self.in_channels * self.weight.size(0)
        uniform(size, self.weight)
        uniform(size, self.root)
        uniform(size, self.bias)

    def _load_from_state_dict(self, *args, **kwargs):
        super(SplineConv, self)._load_from_state_dict(*args, **kwargs)
        self._ks = tuple(int(k) for k in self.kernel_size.tolist())
        self._open = tuple(int(v) for v in self.is_open_spline.tolist())

    def stacked_weight(self):
        """``[in, (K + root) * out]`` fp32 GEMM operand (slot-major columns),
        memoised per forward scope (:mod:`..runtime.cache`)."""
        def build():
            K, cin, cout = self.weight.shape
            w = self.weight.permute(1, 0, 2).reshape(cin, K * cout)
            if self.root is not None:
                w = torch.cat([w, self.root], dim=1)
            return w
        return cached(('spline_w', id(self)), build)

    def stacked_operands(self, dtype, like, plan=None):
        """``(w, w_lp)``: the fp32 stacked weight (gradient carrier) and its
        ``dtype`` copy, memoised per forward scope."""
        if (_backend.use_hip(like) and self.weight.is_cuda and
                dtype in (torch.bfloat16, torch.float32) and
                self.out_channels % 4 == 0):
            def build():
                w, w_lp = _StackedSplineWeight.apply(self.weight, self.root,
                                                     dtype)
                if (dtype == torch.bfloat16 and self.in_channels == 128 and
                        self.out_channels == 128 and SLOT_CONV and
                        getattr(plan, 'tile_flag', None) is not None):
                    # psi_2-shaped: the fused slot conv's two weight images
                    # from the parameters in one kernel (ops/sparse.py).
                    prime_slot_images(w_lp, self.weight, self.root)
                return w, w_lp
            return cached(('spline_w_pack', id(self), dtype), build)
        w = self.stacked_weight()
        return w, cached(('spline_w_lp', id(self), dtype),
                         lambda: w.detach().to(dtype))

    def forward(self, x, edge_index, pseudo, act=None, passthrough=False,
                planes_out=False):
        x = x.unsqueeze(-1) if x.dim() == 1 else x
        pseudo = pseudo.unsqueeze(-1) if pseudo.dim() == 1 else pseudo
        N = x.size(0)
        plan = spline_plan(edge_index, pseudo, N, self._ks, self._open,
                           self.degree, root=self.root is not None,
                           device_params=(self.kernel_size,
                                          self.is_open_spline))
        dtype = compute_dtype(x)
        if dtype == torch.float32 and slot_gemm.supported(
                plan, x, self.weight, self.root):
            # fp32: only the (node, slot) pairs edges use are multiplied
            # (ops/slot_gemm.py, csrc/hip/slot_gemm.hip).
            return slot_gemm.slot_gemm_spmm(
                plan, x, self.weight, self.root, self.bias,
                relu=(act == 'relu'), loop_key=(id(self), N, plan.num_cols),
                passthrough=passthrough,
                dx_row0=getattr(x, '_dgmc_dx_row0', 0),
                planes_out=planes_out)
        w, w_lp = self.stacked_operands(dtype, x, plan)
        return gemm_spmm(plan, x, w, w_lp, self.out_channels, bias=self.bias,
                         relu=(act == 'relu'),
                         loop_key=(id(self), N, plan.num_cols),
                         passthrough=passthrough)

    def __repr__(self):
        return '{}({}, {}, dim={})'.format(self.__class__.__name__,
                                           self.in_channels,
                                           self.out_channels, self.dim)


class GINConv(torch.nn.Module):
    r"""Graph isomorphism operator ``nn((1 + eps) x + sum_{j->i} x_j)``."""

    def __init__(self, nn, eps=0., train_eps=False):
        super(GINConv, self).__init__()
        self.nn = nn
        self.initial_eps = eps
        if train_eps:
            self.eps = Parameter(torch.Tensor([eps]))
        else:
            self.register_buffer('eps', torch.Tensor([eps]))
        self.reset_parameters()

    def reset_parameters(self):
        reset(self.nn)
        self.eps.data.fill_(self.initial_eps)

    def forward(self, x, edge_index):
        x = x.unsqueeze(-1) if x.dim() == 1 else x
        plan = adjacency_plan(edge_index, x.size(0), remove_self_loops=True)
        one_plus_eps = 1 + self.eps
        out = spmm(plan, x, self_x=x, self_scale=one_plus_eps)
        return self.nn(out.to(x.dtype))

    def __repr__(self):
        return '{}(nn={})'.format(self.__class__.__name__, self.nn)


__all__ = ['SplineConv', 'GINConv']
