"""Fused slot convolution on graph-closed tiles (csrc/hip/slot_conv.hip).

Oracle: the unfused fp32 expression ``A @ (x @ [W_0 | .. | W_{S-1}])`` of
SplineConv (``/root/reference/dgmc/models/spline.py:49``) on the same
bf16-rounded operands, forward and backward (dx, dY = A^T g, dW, dbias).
"""
import pytest
import torch

from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops import sparse as sparse_ops
from deep_graph_matching_consensus_amd.runtime import loopgrad
from deep_graph_matching_consensus_amd.ops.sparse import (
    SparseOperator, gemm_spmm, slot_conv_error, slot_conv_image,
    slot_tile_plan)

pytestmark = pytest.mark.gpu
DEV = 'cuda'
C = 128


@pytest.fixture(autouse=True)
def _require_hip():
    assert _backend.hip_available(), 'HIP extension must be built'
    torch.manual_seed(0)
    slot_conv_error(DEV).zero_()


def _graph_batch(sizes, S, deg=4, seed=0):
    """Disjoint union of random graphs with slot-structured entries (unique
    (row, col) per slot, root slot S-1 on the diagonal) + graph-start
    flags."""
    g = torch.Generator().manual_seed(seed)
    rows, cols, vals, flag = [], [], [], []
    off = 0
    for n in sizes:
        flag += [1] + [0] * (n - 1)
        E = n * deg
        i = torch.randint(n, (E, ), generator=g)
        j = torch.randint(n, (E, ), generator=g)
        k = torch.randint(S - 1, (E, ), generator=g)
        key = torch.unique((i * n + j) * S + k)
        i, j, k = key // S // n, key // S % n, key % S
        rows += [i + off]
        cols += [(j + off) * S + k]
        vals += [torch.rand(key.numel(), generator=g) / deg]
        ar = torch.arange(n) + off
        rows += [ar]
        cols += [ar * S + S - 1]
        vals += [torch.ones(n)]
        off += n
    N = off
    op = SparseOperator.from_coo(torch.cat(rows).to(DEV),
                                 torch.cat(cols).to(DEV),
                                 torch.cat(vals).to(DEV), N, N * S)
    flag = torch.tensor(flag, dtype=torch.uint8, device=DEV)
    return op, flag


def _sizes(total_graphs, n_max, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(1, n_max + 1, (total_graphs, ), generator=g).tolist()


def _close(a, b, tol):
    a, b = a.detach(), b.detach()
    return float((a.float() - b).abs().max()) <= tol * float(b.abs().max()) \
        + 1e-3


@pytest.mark.parametrize('n_max,graphs,S', [(19, 300, 26), (8, 77, 5),
                                            (33, 40, 26), (1, 50, 3)])
def test_slot_conv_kernel_forward_backward(n_max, graphs, S):
    ops = _backend.ops()
    op, flag = _graph_batch(_sizes(graphs, n_max), S)
    N = op.num_rows
    window = 65 - n_max
    x = torch.randn(N, C, device=DEV).bfloat16()
    w_lp = (torch.randn(C, S * C, device=DEV) / C ** 0.5).bfloat16()
    bias = torch.randn(C, device=DEV)
    err = slot_conv_error(DEV)
    op.tile_flag, op.tile_window = flag, window
    plan = slot_tile_plan(op, S)
    out = ops.slot_conv(x, *plan, S, slot_conv_image(w_lp, C, False), False,
                        bias, True, torch.float32, None)
    A = op.to_dense()
    # The kernel rounds the operator's values to bf16 (MFMA operand).
    A_lp = A.bfloat16().float()
    y = (x.float() @ w_lp.float()).view(-1, C)
    ref = (A_lp @ y + bias).relu()
    assert int(err) == 0
    assert _close(out, ref, 2e-2)

    g = torch.randn(N, C, device=DEV).bfloat16()
    dy = torch.empty(N * S, C, dtype=torch.bfloat16, device=DEV)
    gx = ops.slot_conv(g, *plan, S, slot_conv_image(w_lp, C, True), True,
                       None, False, torch.float32, dy)
    dy_ref = A_lp.t() @ g.float()
    gx_ref = dy_ref.view(N, -1) @ w_lp.float().t()
    assert int(err) == 0
    assert _close(dy, dy_ref, 1e-2)
    assert _close(gx, gx_ref, 2e-2)


def test_slot_conv_fused_addend():
    """The transposed conv adds a strided bf16 gradient (a slice of the
    concatenation's gradient) in its epilogue."""
    ops = _backend.ops()
    S = 26
    op, flag = _graph_batch(_sizes(120, 19), S)
    N = op.num_rows
    op.tile_flag, op.tile_window = flag, 65 - 19
    plan = slot_tile_plan(op, S)
    w_lp = (torch.randn(C, S * C, device=DEV) / C ** 0.5).bfloat16()
    img = slot_conv_image(w_lp, C, True)
    g = torch.randn(N, C, device=DEV).bfloat16()
    wide = torch.randn(N, 3 * C, device=DEV).bfloat16()
    add = wide[:, C:2 * C]
    base = ops.slot_conv(g, *plan, S, img, True, None, False, torch.float32,
                         None)
    fused = ops.slot_conv(g, *plan, S, img, True, None, False, torch.float32,
                          None, add)
    assert int(slot_conv_error(DEV)) == 0
    torch.testing.assert_close(fused, base + add.float(), atol=1e-5,
                               rtol=1e-5)


def test_spline_cnn_passthrough_gradient_matches_autograd_add(monkeypatch):
    """SplineCNN(cat=True) routes the concatenation's use of each layer input
    through the conv (passthrough alias); gradients equal plain autograd."""
    from deep_graph_matching_consensus_amd.models.spline import SplineCNN
    from deep_graph_matching_consensus_amd.nn import conv as conv_mod
    torch.manual_seed(3)
    model = SplineCNN(C, C, dim=2, num_layers=2, cat=True, lin=False).to(DEV)
    N, E = 400, 2400
    ei = torch.randint(N, (2, E), device=DEV)
    attr = torch.rand(E, 2, device=DEV)

    def run(passthrough):
        if not passthrough:
            orig = conv_mod.SplineConv.forward
            monkeypatch.setattr(
                conv_mod.SplineConv, 'forward',
                lambda self, *a, passthrough=False, **k: (
                    orig(self, *a, **k), a[0]) if passthrough
                else orig(self, *a, **k))
        x = torch.randn(N, C, device=DEV, generator=torch.Generator(
            DEV).manual_seed(0)).requires_grad_()
        model.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = model(x, ei, attr)
        out.float().square().sum().backward()
        monkeypatch.undo()
        return x.grad.clone(), [p.grad.clone() for p in model.parameters()]

    gx1, gp1 = run(True)
    gx0, gp0 = run(False)
    torch.testing.assert_close(gx1, gx0, atol=2e-2, rtol=2e-2)
    for a, b in zip(gp1, gp0):
        torch.testing.assert_close(a, b, atol=2e-2, rtol=2e-2)


def test_slot_conv_flags_oversized_tiles():
    ops = _backend.ops()
    S = 4
    op, flag = _graph_batch([30] * 10, S)
    N = op.num_rows
    w_lp = torch.randn(C, S * C, device=DEV).bfloat16()
    err = slot_conv_error(DEV)
    x = torch.randn(N, C, device=DEV).bfloat16()
    # window 64 with 30-node graphs: a tile can reach 64 + 29 rows.
    ops.slot_tile_plan(flag, op.rowptr, op.col, op.val, 64, S, err)
    assert int(err) & 1
    err.zero_()
    # Flags that split a graph: entries leave their tile.
    bad = torch.ones_like(flag)
    ops.slot_tile_plan(bad, op.rowptr, op.col, op.val, 1, S, err)
    assert int(err) & 2
    err.zero_()


def test_gemm_spmm_uses_slot_conv_forward():
    """Outside a consensus loop: fused slot conv forward, GEMM + SpMM
    backward."""
    S = 26
    op, flag = _graph_batch(_sizes(120, 19, seed=3), S, seed=3)
    op.tile_flag, op.tile_window = flag, 65 - 19
    N = op.num_rows
    x = torch.randn(N, C, device=DEV).bfloat16().requires_grad_()
    w = (torch.randn(C, S * C, device=DEV) / C ** 0.5).requires_grad_()
    bias = torch.randn(C, device=DEV, requires_grad=True)
    w_lp = w.detach().bfloat16()
    calls = []
    real = _backend.ops().slot_conv

    class _Spy(object):
        def __getattr__(self, name):
            if name == 'slot_conv':
                def f(*a):
                    calls.append(a[7])
                    return real(*a)
                return f
            return getattr(torch.ops.dgmc_amd, name)
    orig = _backend.ops
    _backend.ops = lambda: _Spy()
    try:
        out = gemm_spmm(op, x, w, w_lp, C, bias=bias, relu=True)
        g = torch.randn(N, C, device=DEV).bfloat16().float()
        gx, gw, gb = torch.autograd.grad(out, (x, w, bias), g.bfloat16())
    finally:
        _backend.ops = orig
    assert calls == [False]
    assert int(slot_conv_error(DEV)) == 0
    A = op.to_dense().bfloat16().float()
    xf = x.detach().float().requires_grad_()
    wf = w_lp.float().requires_grad_()
    bf = bias.detach().clone().requires_grad_()
    pre = A @ (xf @ wf).view(-1, C) + bf
    assert _close(out, pre.relu(), 3e-2)
    mask = (out.detach().float() > 0).float()
    rx, rw, rb = torch.autograd.grad(pre, (xf, wf, bf), g * mask)
    assert _close(gx, rx, 3e-2)
    assert _close(gw, rw, 3e-2)
    assert _close(gb, rb, 1e-2)


def test_static_training_step_slot_conv_matches_unfused(monkeypatch):
    """PascalVOC-shaped static batch (psi_2 = SplineCNN(128, 128)): one
    forward/backward with the fused slot conv vs the GEMM + SpMM path."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets.static_batch import \
        StaticPairBatcher
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.ops import plans

    groups = make_keypoint_datasets(graphs=16, feature_dim=64, seed=2)
    store = GraphStore(groups, torch.device(DEV))
    batcher = StaticPairBatcher(store, 64, seed=0)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(64, 64, 2, 2, cat=False),
                 SplineCNN(128, 128, 2, 2, cat=True), num_steps=3).to(DEV)
    model.eval()   # no dropout: both runs see identical random draws
    assert batcher.load()

    def run(enabled):
        monkeypatch.setattr(sparse_ops, 'SLOT_CONV', enabled)
        plans.clear_plan_cache()
        batch = batcher.materialize()
        rows = torch.arange(batcher.cap_s, device=DEV)
        torch.manual_seed(1)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            S_0, S_L = model(batch.x_s, batch.edge_index_s,
                             batch.edge_attr_s, batch.x_s_batch, batch.x_t,
                             batch.edge_index_t, batch.edge_attr_t,
                             batch.x_t_batch)
        y = torch.stack([rows, batch.y])
        loss = model.loss(S_L, y, mask=batch.y_mask)
        grads = torch.autograd.grad(loss, list(model.psi_2.parameters()))
        return S_L.detach(), loss.detach(), grads

    S_a, l_a, g_a = run(True)
    S_b, l_b, g_b = run(False)
    assert int(slot_conv_error(DEV)) == 0
    assert torch.allclose(l_a, l_b, rtol=2e-2, atol=2e-2)
    assert (S_a - S_b).abs().max() < 0.05
    for a, b in zip(g_a, g_b):
        assert _close(a, b.float(), 0.1)


@pytest.mark.parametrize('uses,S,n_max',
                         [(3, 26, 19), (1, 5, 8), (10, 26, 12),
                          (17, 26, 12), (33, 5, 8)])
def test_slot_weight_grad_matches_dense(uses, S, n_max):
    from deep_graph_matching_consensus_amd.ops.sparse import slot_weight_grad
    op, flag = _graph_batch(_sizes(90, n_max, seed=5), S, seed=5)
    N = op.num_rows
    X = torch.randn(uses * N, C, device=DEV).bfloat16()
    G = torch.randn(uses * N, C, device=DEV).bfloat16()
    dW = slot_weight_grad(X, G, op, S, uses, nsplit=3)
    A = op.to_dense()                                   # [N, N*S]
    ref = torch.zeros(S, C, C, device=DEV)
    for u in range(uses):
        Xu, Gu = X[u * N:(u + 1) * N].float(), G[u * N:(u + 1) * N].float()
        dY = (A.t() @ Gu).view(N, S, C)                 # dY[j, k, :]
        ref += torch.einsum('jc,jko->kco', Xu, dY)
    # The kernel rounds a_e * X to bf16 (MFMA operand).
    assert _close(dW, ref, 2e-2)
    # Per-use tensors read in place through the pointer table: identical
    # summation order, hence bit-identical to the stacked form.
    Xs = [X[u * N:(u + 1) * N].clone() for u in range(uses)]
    Gs = [G[u * N:(u + 1) * N].clone() for u in range(uses)]
    assert torch.equal(slot_weight_grad(Xs, Gs, op, S, uses, nsplit=3), dW)


@pytest.mark.parametrize('num_steps', [4, 17])
def test_loop_training_step_slot_wgrad_matches_stacked_gemm(monkeypatch,
                                                            num_steps):
    """Consensus loop on a static batch: psi_2 weight gradients from the
    slot wgrad kernel vs the dY stack + GEMM path (17 steps: more uses than
    the kernel's pointer table, chunked)."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets.static_batch import \
        StaticPairBatcher
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.ops import plans

    groups = make_keypoint_datasets(graphs=16, feature_dim=64, seed=3)
    store = GraphStore(groups, torch.device(DEV))
    batcher = StaticPairBatcher(store, 64, seed=1)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(64, 64, 2, 2, cat=False),
                 SplineCNN(128, 128, 2, 2, cat=True),
                 num_steps=num_steps).to(DEV)
    model.eval()
    assert batcher.load()

    def run(enabled):
        # enabled: loop-folded slot weight gradient (one slot_wgrad launch
        # over the kept (x, g') pairs); disabled: per-use autograd through
        # the unfused backward (dY stack + GEMM).
        monkeypatch.setattr(loopgrad, 'ENABLED', enabled)
        plans.clear_plan_cache()
        batch = batcher.materialize()
        rows = torch.arange(batcher.cap_s, device=DEV)
        torch.manual_seed(1)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            S_0, S_L = model(batch.x_s, batch.edge_index_s,
                             batch.edge_attr_s, batch.x_s_batch, batch.x_t,
                             batch.edge_index_t, batch.edge_attr_t,
                             batch.x_t_batch)
        y = torch.stack([rows, batch.y])
        loss = model.loss(S_L, y, mask=batch.y_mask)
        return torch.autograd.grad(loss, list(model.parameters()))

    g_a = run(True)
    g_b = run(False)
    assert int(slot_conv_error(DEV)) == 0
    for a, b in zip(g_a, g_b):
        assert torch.isfinite(a).all()
        assert _close(a, b.float(), 0.1)


def test_slot_pair_lists_stable_counting_sort():
    from deep_graph_matching_consensus_amd.ops.sparse import slot_pair_lists
    S = 26
    op, _ = _graph_batch(_sizes(400, 19, seed=7), S, seed=7)
    esrc, edst, evals, soff = slot_pair_lists(op, S)
    col = op.col.long()
    k = col % S
    perm = torch.argsort(k, stable=True)
    assert torch.equal(esrc.long(), (col // S)[perm])
    assert torch.equal(edst.long(), op.row[perm])
    assert torch.equal(evals, op.val[perm])
    cnt = torch.bincount(k, minlength=S)
    assert torch.equal(soff[1:].long(), torch.cumsum(cnt, 0))


def _dense_case(seed=11):
    """Dense 32-node graphs: two per 64-row tile with > 4096 entries per
    tile, so the kernels read entries from global memory (unstaged path,
    E > kScECap in csrc/hip/slot_conv.hip)."""
    S = 26
    op, flag = _graph_batch([32] * 24 + [17, 9, 30], S, deg=100, seed=seed)
    op.tile_flag, op.tile_window = flag, 65 - 32
    N = op.num_rows
    g = torch.Generator(DEV).manual_seed(seed)
    x = torch.randn(N, C, device=DEV, generator=g).bfloat16()
    gy = torch.randn(N, C, device=DEV, generator=g).bfloat16()
    w_lp = (torch.randn(C, S * C, device=DEV, generator=g) /
            C ** 0.5).bfloat16()
    bias = torch.randn(C, device=DEV, generator=g)
    return op, S, x, gy, w_lp, bias


def _dense_case_outputs():
    ops = _backend.ops()
    op, S, x, gy, w_lp, bias = _dense_case()
    plan = slot_tile_plan(op, S)
    out = ops.slot_conv(x, *plan, S, slot_conv_image(w_lp, C, False), False,
                        bias, True, torch.float32, None)
    gx = ops.slot_conv(gy, *plan, S, slot_conv_image(w_lp, C, True), True,
                       None, False, torch.float32, None)
    return op, plan, out, gx


def test_slot_conv_unstaged_dense_tiles():
    _, S, x, gy, w_lp, bias = _dense_case()
    op, plan, out, gx = _dense_case_outputs()
    # tiles[t] = (r0, r1, e0, E | largest slot bucket << 16): at least one
    # tile holds more entries than the LDS staging capacity (4096)
    E_tile = plan[0].view(-1, 4)[:, 3] & 0xFFFF
    assert int(E_tile.max()) > 4096
    A = op.to_dense().bfloat16().float()
    y = (x.float() @ w_lp.float()).view(-1, C)
    assert int(slot_conv_error(DEV)) == 0
    assert _close(out, (A @ y + bias).relu(), 2e-2)
    gx_ref = (A.t() @ gy.float()).view(op.num_rows, -1) @ w_lp.float().t()
    assert _close(gx, gx_ref, 2e-2)


def test_slot_conv_relu_bwd_fused_prologue():
    """Transposed slot conv with the fused ReLU/bias backward == ReLU mask +
    column sums + plain transposed conv (strided G, addend)."""
    ops = _backend.ops()
    S = 26
    op, flag = _graph_batch(_sizes(150, 19, seed=9), S, seed=9)
    N = op.num_rows
    op.tile_flag, op.tile_window = flag, 65 - 19
    plan = slot_tile_plan(op, S)
    w_lp = (torch.randn(C, S * C, device=DEV) / C ** 0.5).bfloat16()
    img = slot_conv_image(w_lp, C, True)
    wide = torch.randn(N, 3 * C, device=DEV).bfloat16()
    G = wide[:, C:2 * C]                         # row stride 384
    relu_out = torch.randn(N, C, device=DEV).relu().bfloat16()
    add = torch.randn(N, 2 * C, device=DEV).bfloat16()[:, :C]
    g_out = torch.empty(N, C, dtype=torch.bfloat16, device=DEV)
    T = plan[0].size(0)
    part = torch.full((T, C), float('nan'), device=DEV)
    gx = ops.slot_conv_relu_bwd(G, relu_out, *plan, S, img, torch.float32,
                                add, g_out, part)
    g_ref = torch.where(relu_out > 0, G, torch.zeros_like(G))
    assert torch.equal(g_out, g_ref)
    torch.testing.assert_close(part.sum(0), g_ref.float().sum(0), atol=1e-3,
                               rtol=1e-4)
    base = ops.slot_conv(g_ref.contiguous(), *plan, S, img, True, None, False,
                         torch.float32, None, add)
    assert int(slot_conv_error(DEV)) == 0
    torch.testing.assert_close(gx, base, atol=0, rtol=0)
