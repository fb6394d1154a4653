"""Fused RelCNN consensus encoder (psi_2 of the DBP15K config) on the HIP
kernels of ``csrc/hip/relconv.hip``.

Reference: ``/root/reference/dgmc/models/rel.py:25-99`` (RelConv / RelCNN)
as used by ``/root/reference/examples/dbp15k.py:29-33`` - psi_2 =
``RelCNN(32, 32, 3, batch_norm=False, cat=True, lin=True, dropout=0)`` -
inside DGMC's sparse consensus loop (``dgmc/models/dgmc.py:204-223``), with
psi_2's final Linear folded into the consensus MLP's first layer
(``models/dgmc.py``: ``[P; Q] = feat (W1 W_f)^T``).

One consensus step on the joint graph (source and target entities, N rows):

* forward - three layer kernels (gather both mean aggregations of the layer
  input + ``[W1 | W2 | Wr]`` on exact-f32 MFMA + bias + ReLU), writing the
  concatenation ``feat = [r | h1 | h2 | h3]`` column by column; the last one
  also computes ``PQ = feat fold^T`` (``fold = W1_mlp W_f``) - no hipBLASLt,
  no concatenation kernel, no separate projection GEMM;
* backward - one projection kernel (``dfeat = dPQ fold``, fold-gradient
  partials) and three layer kernels (each gathers the transposed
  aggregations of its ``g'``, multiplies by ``[W1; W2; Wr]``, adds the
  result into the previous feature slice's gradient and applies that
  slice's ReLU mask, and deposits weight / bias gradient partials).

The weight gradients of the ``num_steps`` uses accumulate into per-tile
partial buffers (``runtime/loopgrad.py``) folded once by the last use.
"""
import torch

from . import _backend
from .plans import _CACHE

# Rows whose in- + out-lists hold more than this many entries are gathered
# by a whole wave (entries split over its 8 lane groups) instead of one lane
# group: 455 / 691 of the 19.4k / 19.6k entities of the DBP15K-shaped graphs
# (datasets/kg.py), at most 288 entries.
HUB_THRESHOLD = 32
ROWS = 64                 # rows per tile (relconv.hip::kRcRows)
PART = 3 * 32 * 32 + 32   # per-tile partial (relconv.hip::kRcPart)


class RelPlan(object):
    """Joint neighbour lists of one graph for the fused kernels (static;
    built once - the hub split needs no host synchronisation, but the
    lists' sort does run on the device before any capture).

    * forward: row i = in-neighbours (edges j -> i), then out-neighbours
      (i -> j) from ``split_f[i]``;
    * backward: row j = out-neighbours i weighted ``1 / deg_in(i)`` (the
      transposed in-flow mean), then in-neighbours weighted
      ``1 / deg_out(i)`` from ``split_b[j]``.
    """

    def __init__(self, edge_index, N, hub_threshold=HUB_THRESHOLD):
        dev = edge_index.device
        src, dst = edge_index[0].long(), edge_index[1].long()
        N = self.N = int(N)
        E = src.numel()
        deg_in = torch.bincount(dst, minlength=N)
        deg_out = torch.bincount(src, minlength=N)
        deg = deg_in + deg_out
        ptr = torch.zeros(N + 1, dtype=torch.long, device=dev)
        torch.cumsum(deg, 0, out=ptr[1:])
        # Joint entries: key = 2 * row + list (stable: edge order inside).
        rows_f = torch.cat([dst * 2, src * 2 + 1])
        cols_f = torch.cat([src, dst])
        perm = torch.argsort(rows_f, stable=True)
        self.col_f = cols_f[perm].int().contiguous()
        seg_f = rows_f[perm] % (2 * ROWS)      # segment inside the row tile
        rows_b = torch.cat([src * 2, dst * 2 + 1])
        cols_b = torch.cat([dst, src])
        perm = torch.argsort(rows_b, stable=True)
        col_b = cols_b[perm]
        seg_b = rows_b[perm] % (2 * ROWS)
        inv_in = 1.0 / deg_in.clamp(min=1).float()
        inv_out = 1.0 / deg_out.clamp(min=1).float()
        first = torch.cat([torch.ones(E, dtype=torch.bool, device=dev),
                           torch.zeros(E, dtype=torch.bool, device=dev)])
        # (list 0 of the backward: out-neighbours, weight 1 / deg_in)
        w_b = torch.where(first[perm], inv_in[col_b], inv_out[col_b])
        # one trailing dummy entry: the kernels' clamped (branch-free) list
        # loads stay in bounds for edgeless tiles and graphs
        pad_i = torch.zeros(1, dtype=torch.int32, device=dev)
        self.col_f = torch.cat([self.col_f, pad_i])
        self.col_b = torch.cat([col_b.int(), pad_i])
        self.w_b = torch.cat([w_b, torch.zeros(1, device=dev)])
        # kernel lists: column | tile segment (2 (row % 64) + list) << 24, so
        # a gathering lane sees segment changes without a search
        assert N < (1 << 24), 'RelPlan: at most 2^24 - 1 rows'
        self.pk_f = torch.cat([(self.col_f[:-1].long() | (seg_f << 24)).int(),
                               pad_i])
        self.pk_b = torch.cat([(self.col_b[:-1].long() | (seg_b << 24)).int(),
                               pad_i])
        self.ptr = ptr.int().contiguous()
        self.split_f = (ptr[:-1] + deg_in).int().contiguous()
        self.split_b = (ptr[:-1] + deg_out).int().contiguous()
        self.hub = (deg > hub_threshold).to(torch.uint8).contiguous()
        self.n_tiles = (N + ROWS - 1) // ROWS

    def fwd_args(self):
        return (self.ptr, self.pk_f, self.split_f, self.hub)

    def bwd_args(self):
        return (self.ptr, self.pk_b, self.w_b, self.split_b, self.hub)


def rel_plan(edge_index, N):
    """Cached :class:`RelPlan` of ``edge_index`` (tensor identity); None
    while a graph is being captured before the plan exists."""
    params = ('relfused', int(N), HUB_THRESHOLD)
    plan = _CACHE.get((edge_index, ), params)
    if plan is None:
        if edge_index.is_cuda and torch.cuda.is_current_stream_capturing():
            return None
        plan = _CACHE.put((edge_index, ), params, RelPlan(edge_index, N))
    return plan


def supported(psi_2, final, mlp0):
    """psi_2 = RelCNN(32, 32, 3, cat=True, lin=True) without BatchNorm or
    active dropout, fp32 on the GPU, consensus MLP width 32."""
    from ..models.rel import RelCNN
    if not isinstance(psi_2, RelCNN) or not _backend.hip_available():
        return False
    if psi_2.batch_norm or not psi_2.cat or not psi_2.lin:
        return False
    if psi_2.training and psi_2.dropout > 0:
        return False
    if psi_2.num_layers != 3 or psi_2.in_channels != 32:
        return False
    ok = all(c.in_channels == 32 and c.out_channels == 32 and
             c.lin1.weight.is_cuda and c.lin1.weight.dtype == torch.float32
             for c in psi_2.convs)
    return bool(ok and tuple(final.weight.shape) == (32, 128) and
                tuple(mlp0.weight.shape) == (32, 32) and
                final.weight.dtype == torch.float32)


def _layer_params(psi_2):
    out = []
    for c in psi_2.convs:
        out += [c.lin1.weight, c.lin2.weight, c.root.weight, c.root.bias]
    return out


class _RelPsi2Fold(torch.autograd.Function):
    """``PQ = [r | h1 | h2 | h3] (W1_mlp W_f)^T`` for one consensus step
    (``r = [r_s; r_t]``, ``h_l = relu(RelConv_l(h_{l-1}))``)."""

    @staticmethod
    def forward(ctx, r_t, r_s, plan, loop, w_mlp, w_final, *params):
        ops = _backend.ops()
        N, n_s = plan.N, r_s.size(0)
        dev = r_t.device
        from ..runtime.cache import cached
        # (one fold per forward: the num_steps uses share the weights)
        fold = cached(('rel_fold', id(w_mlp), id(w_final)),
                      lambda: (w_mlp, w_final, ops.fold_weights(
                          w_mlp.contiguous(), w_final.contiguous())[0]))[2]
        feat = torch.empty((N, 128), dtype=torch.float32, device=dev)
        pq = torch.empty((N, 32), dtype=torch.float32, device=dev)
        pa = plan.fwd_args()
        W = [p.contiguous() for p in params]
        for l in range(3):
            w1, w2, wr, b = W[4 * l:4 * l + 4]
            last = l == 2
            if l == 0:
                xa, xb, xcopy = r_s, r_t, feat[:, 0:32]
            else:
                xa, xb, xcopy = feat[:, 32 * l:32 * l + 32], None, None
            ops.relconv_fwd(*pa, xa, xb, w1, w2, wr, b, True,
                            feat[:, 32 * (l + 1):32 * (l + 2)], xcopy,
                            feat[:, 0:96] if last else None,
                            fold if last else None, pq if last else None)
        ctx.plan, ctx.loop, ctx.n_s = plan, loop, n_s
        ctx.idx = loop.register() if loop is not None else None
        ctx.save_for_backward(feat, fold, w_mlp, w_final, *W)
        return pq

    @staticmethod
    def backward(ctx, dpq):
        ops = _backend.ops()
        feat, fold, w_mlp, w_final = ctx.saved_tensors[:4]
        W = ctx.saved_tensors[4:]
        plan, loop, n_s = ctx.plan, ctx.loop, ctx.n_s
        N, dev = plan.N, feat.device
        dpq = dpq.contiguous().float()
        pa = plan.bwd_args()
        shapes = [('f', (plan.n_tiles, 32 * 128))] + [
            ('l%d' % l, (plan.n_tiles, PART)) for l in range(3)]
        bufs = {}
        for name, shape in shapes:
            if loop is not None:
                bufs[name] = loop.acc(name, shape, dev)
            else:
                bufs[name] = (torch.empty(shape, dtype=torch.float32,
                                          device=dev), False)
        dfeat = torch.empty((N, 128), dtype=torch.float32, device=dev)
        ops.rel_proj_bwd(dpq, feat, fold, dfeat, *bufs['f'])
        drt = torch.empty((N - n_s, 32), dtype=torch.float32, device=dev)
        for l in (2, 1, 0):
            w1, w2, wr = W[4 * l:4 * l + 3]
            g = dfeat[:, 32 * (l + 1):32 * (l + 2)]
            x = feat[:, 32 * l:32 * l + 32]
            prev = dfeat[:, 32 * l:32 * l + 32]
            if l > 0:
                # (dadd + dx) * relu'(h_l) = g' of layer l - 1, in place
                ops.relconv_bwd(*pa, g, x, None, w1, w2, wr, prev, prev, 0,
                                True, *bufs['l%d' % l])
            else:
                # d r_t = dfeat[n_s:, 0:32] + dx (r_s carries no gradient)
                ops.relconv_bwd(*pa, g, x, None, w1, w2, wr, prev, drt, n_s,
                                False, *bufs['l0'])
        n_params = len(W)
        grads = [None] * n_params
        gw_mlp = gw_final = None
        if loop is None or loop.arrive():
            red = {name: torch.empty(shape[1], dtype=torch.float32,
                                     device=dev) for name, shape in shapes}
            ops.rel_fold([bufs[name][0] for name, _ in shapes],
                         [red[name] for name, _ in shapes])
            for l in range(3):
                v = red['l%d' % l]
                grads[4 * l + 0] = v[0:1024].view(32, 32)
                grads[4 * l + 1] = v[1024:2048].view(32, 32)
                grads[4 * l + 2] = v[2048:3072].view(32, 32)
                grads[4 * l + 3] = v[3072:3104]
            gw_mlp, gw_final = ops.fold_weights_bwd(
                w_mlp.contiguous(), w_final.contiguous(),
                red['f'].view(32, 128))
            if loop is not None:
                loop.release()
        return (drt, None, None, None, gw_mlp, gw_final) + tuple(grads)


def psi2_fold(psi_2, mlp0_weight, plan, r_s, r_t, loop_key):
    """``[P; Q]`` (``[N, 32]``) of one consensus step; ``r_s [N_s, 32]`` is
    the random indicator (no gradient), ``r_t [N_t, 32]`` its transport."""
    from ..runtime import loopgrad
    loop = loopgrad.group(('relpsi2', ) + tuple(loop_key))
    return _RelPsi2Fold.apply(r_t.float().contiguous(),
                              r_s.detach().float().contiguous(), plan, loop,
                              mlp0_weight, psi_2.final.weight,
                              *_layer_params(psi_2))


def reference_psi2_fold(psi_2, mlp0_weight, edge_index, r_s, r_t):
    """The same quantity through the reference expression (fp64-capable
    oracle for tests): psi_2 features, then the folded projection."""
    x = torch.cat([r_s, r_t], 0)
    xs = [x]
    for conv in psi_2.convs:
        src, dst = edge_index[0], edge_index[1]
        N = x.size(0)

        def mean(msg, index):
            out = torch.zeros(N, msg.size(1), dtype=msg.dtype,
                              device=msg.device)
            out.index_add_(0, index, msg)
            cnt = torch.bincount(index, minlength=N).clamp(min=1)
            return out / cnt.to(msg.dtype).view(-1, 1)

        h = xs[-1]
        out = (mean(h[src] @ conv.lin1.weight.t().to(h.dtype), dst) +
               mean(h[dst] @ conv.lin2.weight.t().to(h.dtype), src) +
               h @ conv.root.weight.t().to(h.dtype) +
               conv.root.bias.to(h.dtype))
        xs.append(torch.relu(out))
    feat = torch.cat(xs, -1)
    fold = mlp0_weight.to(feat.dtype) @ psi_2.final.weight.to(feat.dtype)
    return feat @ fold.t()
