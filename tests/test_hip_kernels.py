"""HIP kernel numerics vs the fp32 PyTorch oracles (run on an MI355X).

Every native op is compared against ``ops/reference.py`` (plain PyTorch,
fp32) forward AND backward.  These tests must exercise the HIP path: they
assert the extension is loaded (no silent fallback).
"""
import pytest
import torch

from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops import dense as dense_ops
from deep_graph_matching_consensus_amd.ops import reference as ref
from deep_graph_matching_consensus_amd.ops import sparse_corr
from deep_graph_matching_consensus_amd.ops.plans import (
    compute_spline_basis, clear_plan_cache)
from deep_graph_matching_consensus_amd.ops.sparse import (SparseOperator,
                                                          spmm)
from deep_graph_matching_consensus_amd.runtime import reference_mode

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(autouse=True)
def _require_hip():
    assert _backend.hip_available(), 'HIP extension must be built'
    torch.manual_seed(0)


def _random_op(R, C, nnz, device):
    row = torch.randint(R, (nnz, ), device=device)
    col = torch.randint(C, (nnz, ), device=device)
    val = torch.randn(nnz, device=device)
    return SparseOperator.from_coo(row, col, val, R, C)


@pytest.mark.parametrize('C', [1, 7, 8, 16, 32, 128, 256, 300])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_spmm_forward_backward(C, dtype):
    R, X, nnz = 97, 131, 900
    op = _random_op(R, X, nnz, DEV)
    x = torch.randn(X, C, device=DEV).to(dtype).requires_grad_()
    bias = torch.randn(C, device=DEV, requires_grad=True)
    out = spmm(op, x, bias=bias, relu=True)
    with reference_mode():
        x2 = x.detach().clone().requires_grad_()
        b2 = bias.detach().clone().requires_grad_()
        out2 = spmm(op, x2, bias=b2, relu=True)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert torch.allclose(out, out2, atol=tol, rtol=tol)
    g = torch.randn_like(out)
    gx, gb = torch.autograd.grad(out, (x, bias), g)
    gx2, gb2 = torch.autograd.grad(out2, (x2, b2), g)
    assert torch.allclose(gx.float(), gx2.float(), atol=tol * 4, rtol=tol)
    assert torch.allclose(gb, gb2, atol=1e-4, rtol=1e-4)


def _skewed_op(R, X, device, hub=1500):
    """Random CSR with a hub row of ``hub`` entries, rows of 60-70 entries
    (one or two pieces) and empty rows."""
    g = torch.Generator().manual_seed(3)
    deg = torch.randint(0, 12, (R, ), generator=g)
    deg[0] = hub
    deg[5] = 64
    deg[6] = 65
    deg[7:12] = 0
    row = torch.repeat_interleave(torch.arange(R), deg)
    col = torch.randint(X, (row.numel(), ), generator=g)
    val = torch.randn(row.numel(), generator=g)
    op = SparseOperator.from_coo(row.to(device), col.to(device),
                                 val.to(device), R, X)
    op.balanced = True
    return op


@pytest.mark.parametrize('C,dtype', [(4, torch.float32), (32, torch.float32),
                                     (96, torch.float32), (256, torch.float32),
                                     (300, torch.float32), (7, torch.float32),
                                     (32, torch.bfloat16),
                                     (128, torch.bfloat16)])
def test_spmm_pieces_skewed_rows(C, dtype):
    """Piece-balanced SpMM (hub rows split, partials folded in order) ==
    fp32 oracle, forward (bias + ReLU) and backward (transposed operator,
    also balanced), and bitwise reproducible."""
    R, X = 300, 257
    op = _skewed_op(R, X, DEV)
    x = torch.randn(X, C, device=DEV).to(dtype).requires_grad_()
    bias = torch.randn(C, device=DEV, requires_grad=True)
    out = spmm(op, x, bias=bias, relu=True)
    again = spmm(op, x, bias=bias, relu=True)
    assert torch.equal(out, again)
    with reference_mode():
        x2 = x.detach().clone().requires_grad_()
        b2 = bias.detach().clone().requires_grad_()
        out2 = spmm(op, x2, bias=b2, relu=True)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert torch.allclose(out.float(), out2.float(), atol=tol * 10, rtol=tol)
    g = torch.randn_like(out)
    gx, gb = torch.autograd.grad(out, (x, bias), g)
    gx2, gb2 = torch.autograd.grad(out2, (x2, b2), g)
    assert torch.allclose(gx.float(), gx2.float(), atol=tol * 10, rtol=tol)
    assert torch.allclose(gb, gb2, atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize('C,dtype', [(32, torch.float32),
                                     (64, torch.float32),
                                     (8, torch.float32),
                                     (128, torch.bfloat16)])
def test_spmm_split_static_operator(C, dtype):
    """Static skewed operators (KG relational plans): the one-launch short /
    long row split == the piece-balanced path == fp32 oracle, forward (self
    term, bias, ReLU) and backward (transposed operator), bitwise
    reproducible."""
    R, X = 300, 257
    op = _skewed_op(R, X, DEV, hub=700)
    op.static = True
    assert op.split_rows()[1].numel() > 0        # long rows exist
    x = torch.randn(X, C, device=DEV).to(dtype).requires_grad_()
    bias = torch.randn(C, device=DEV, requires_grad=True)
    out = spmm(op, x, bias=bias, relu=True)
    assert torch.equal(out, spmm(op, x, bias=bias, relu=True))
    op.static = False
    op.t().static = False
    pieces = spmm(op, x, bias=bias, relu=True)
    op.static = True
    op.t().static = True
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert torch.allclose(out.float(), pieces.float(), atol=tol * 10,
                          rtol=tol)
    with reference_mode():
        x2 = x.detach().clone().requires_grad_()
        b2 = bias.detach().clone().requires_grad_()
        out2 = spmm(op, x2, bias=b2, relu=True)
    assert torch.allclose(out.float(), out2.float(), atol=tol * 10, rtol=tol)
    g = torch.randn_like(out)
    gx, gb = torch.autograd.grad(out, (x, bias), g)
    gx2, gb2 = torch.autograd.grad(out2, (x2, b2), g)
    assert torch.allclose(gx.float(), gx2.float(), atol=tol * 10, rtol=tol)
    assert torch.allclose(gb, gb2, atol=1e-3, rtol=1e-4)
    # Self term (GIN-like (1 + eps) x) through spmm_split_out directly.
    sx = torch.randn(R, C, device=DEV).to(dtype)
    scale = torch.tensor([1.5], device=DEV)
    o3 = torch.empty(R, C, device=DEV, dtype=dtype)
    sr, lr = op.split_rows()
    _backend.ops().spmm_split_out(op.rowptr, op.col, op.val, sr, lr,
                                  x.detach().contiguous(), sx, scale, None,
                                  False, o3)
    ref3 = op.to_dense() @ x.detach().float() + 1.5 * sx.float()
    assert torch.allclose(o3.float(), ref3, atol=tol * 10, rtol=tol)


def test_piece_plan_hip_matches_torch():
    from deep_graph_matching_consensus_amd.ops.sparse import piece_plan
    # (20011 rows: several rows per scan thread, a partial last thread)
    for op in (_skewed_op(300, 257, DEV), _skewed_op(20011, 257, DEV)):
        for T in (1, 16, 64):
            a = piece_plan(op.rowptr, op.nnz, T)
            b = piece_plan(op.rowptr.cpu(), op.nnz, T)
            for x, y in zip(a, b):
                assert torch.equal(x.cpu(), y)


def test_spmm_pieces_self_term_and_perm():
    """Self term (GIN form) and values read through a permutation."""
    R, X, C = 200, 200, 32
    op = _skewed_op(R, X, DEV, hub=700)
    x = torch.randn(X, C, device=DEV)
    sx = torch.randn(R, C, device=DEV)
    scale = torch.tensor([1.5], device=DEV)
    perm = torch.randperm(op.nnz, device=DEV)
    shuffled = torch.empty_like(op.val)
    shuffled[perm] = op.val            # shuffled[perm[e]] == val[e]
    out = torch.empty(R, C, device=DEV)
    _backend.ops().spmm_pieces_out(op.rowptr, op.col, shuffled,
                                   perm.to(torch.int32), *op.pieces(),
                                   x, sx, scale, None, False, out)
    dense = op.to_dense()
    assert torch.allclose(out, dense @ x + 1.5 * sx, atol=1e-4, rtol=1e-4)


def test_spmm_self_term_gin():
    N, C = 50, 24
    op = _random_op(N, N, 300, DEV)
    x = torch.randn(N, C, device=DEV, requires_grad=True)
    eps = torch.tensor([0.3], device=DEV, requires_grad=True)
    out = spmm(op, x, self_x=x, self_scale=1 + eps)
    with reference_mode():
        x2 = x.detach().clone().requires_grad_()
        e2 = eps.detach().clone().requires_grad_()
        out2 = spmm(op, x2, self_x=x2, self_scale=1 + e2)
    assert torch.allclose(out, out2, atol=1e-5)
    g = torch.randn_like(out)
    ga = torch.autograd.grad(out, (x, eps), g)
    gb = torch.autograd.grad(out2, (x2, e2), g)
    assert torch.allclose(ga[0], gb[0], atol=1e-4)
    assert torch.allclose(ga[1], gb[1], atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize('degree', [1, 2, 3])
@pytest.mark.parametrize('dim', [1, 2, 3])
def test_spline_basis(degree, dim):
    pseudo = torch.rand(500, dim, device=DEV)
    ks, op = [5] * dim, [1] * dim
    b1, w1 = compute_spline_basis(pseudo, ks, op, degree)
    b2, w2 = ref.spline_basis(pseudo, ks, op, degree)
    assert torch.allclose(b1, b2, atol=1e-6)
    assert torch.equal(w1, w2)


def test_spline_conv_matches_cpu():
    from deep_graph_matching_consensus_amd.nn import SplineConv
    torch.manual_seed(1)
    conv = SplineConv(16, 32, 2, kernel_size=5)
    x = torch.randn(60, 16)
    ei = torch.randint(60, (2, 240))
    pseudo = torch.rand(240, 2)
    out_cpu = conv(x, ei, pseudo, act='relu')
    clear_plan_cache()
    conv_gpu = conv.to(DEV)
    out_gpu = conv_gpu(x.to(DEV), ei.to(DEV), pseudo.to(DEV), act='relu')
    assert torch.allclose(out_cpu, out_gpu.cpu(), atol=1e-4)


def _layouts(B, Ns, Nt):
    from deep_graph_matching_consensus_amd.graph.dense import DenseLayout
    from deep_graph_matching_consensus_amd.graph.meta import BatchInfo
    c_s = torch.randint(1, Ns + 1, (B, ))
    c_t = torch.randint(1, Nt + 1, (B, ))
    c_s[0], c_t[0] = Ns, Nt
    return (DenseLayout(BatchInfo(c_s), torch.device(DEV)),
            DenseLayout(BatchInfo(c_t), torch.device(DEV)))


def _mask(lay_s, lay_t):
    return ref.count_mask(lay_s.counts, lay_t.counts, lay_s.N, lay_t.N)


@pytest.mark.parametrize('shape', [(7, 13, 17), (3, 64, 64), (5, 1, 9)])
def test_dense_masked_softmax(shape):
    lay_s, lay_t = _layouts(*shape)
    S_hat = torch.randn(shape, device=DEV, requires_grad=True)
    out = dense_ops.masked_softmax(S_hat, lay_s, lay_t)
    S2 = S_hat.detach().clone().requires_grad_()
    out2 = ref.masked_softmax(S2, _mask(lay_s, lay_t))
    assert torch.allclose(out, out2, atol=1e-6)
    g = torch.randn_like(out)
    assert torch.allclose(torch.autograd.grad(out, S_hat, g)[0],
                          torch.autograd.grad(out2, S2, g)[0], atol=1e-5)


@pytest.mark.parametrize('R,dtype', [(8, torch.float32), (64, torch.float32),
                                     (100, torch.float32),
                                     (128, torch.float32),
                                     (128, torch.bfloat16),
                                     (300, torch.float32)])
def test_dense_softmax_transport(R, dtype):
    B, Ns, Nt = 6, 19, 23
    lay_s, lay_t = _layouts(B, Ns, Nt)
    S_hat = torch.randn(B, Ns, Nt, device=DEV, requires_grad=True)
    r_s = torch.randn(lay_s.num_nodes, R, device=DEV).to(dtype)
    if dtype != torch.float32:
        r_t = dense_ops.softmax_transport(S_hat, r_s, lay_s, lay_t)
        S2 = S_hat.detach().clone().requires_grad_()
        r_t2 = lay_t.to_sparse(ref.masked_softmax(
            S2, _mask(lay_s, lay_t)).transpose(-1, -2) @
            lay_s.to_dense(r_s.float()))
        assert r_t.dtype == dtype
        assert torch.allclose(r_t.float(), r_t2, atol=2e-2, rtol=2e-2)
        g = torch.randn_like(r_t2)
        ga = torch.autograd.grad(r_t, S_hat, g.to(dtype))[0]
        gb = torch.autograd.grad(r_t2, S2, g.to(dtype).float())[0]
        assert torch.allclose(ga, gb, atol=1e-3, rtol=1e-3)
        return
    r_t = dense_ops.softmax_transport(S_hat, r_s, lay_s, lay_t)
    assert r_t.shape == (lay_t.num_nodes, R)
    S2 = S_hat.detach().clone().requires_grad_()
    r_t2 = ref.masked_softmax(S2, _mask(lay_s, lay_t)).transpose(-1, -2) \
        @ lay_s.to_dense(r_s)
    r_t2 = lay_t.to_sparse(r_t2)
    assert torch.allclose(r_t, r_t2, atol=1e-5)
    g = torch.randn_like(r_t)
    g_ref = torch.autograd.grad(r_t2, S2, g)[0]
    assert torch.allclose(torch.autograd.grad(r_t, S_hat, g)[0], g_ref,
                          atol=1e-4)
    # Joint [r_s; r_t] output (psi_2's fused input, no cat kernel).
    joint = dense_ops.softmax_transport_joint(S_hat, r_s, lay_s, lay_t)
    assert torch.equal(joint[:lay_s.num_nodes], r_s)
    assert torch.allclose(joint[lay_s.num_nodes:], r_t2, atol=1e-5)
    gj = torch.cat([torch.randn_like(r_s), g])
    assert torch.allclose(torch.autograd.grad(joint, S_hat, gj)[0], g_ref,
                          atol=1e-4)


@pytest.mark.parametrize('R', [8, 32, 100, 128, 300])
@pytest.mark.parametrize('joint', [False, True])
def test_dense_consensus_update(R, joint):
    B, Ns, Nt = 5, 21, 18
    lay_s, lay_t = _layouts(B, Ns, Nt)
    S_hat = torch.randn(B, Ns, Nt, device=DEV, requires_grad=True)
    mlp = torch.nn.Sequential(torch.nn.Linear(R, R), torch.nn.ReLU(),
                              torch.nn.Linear(R, 1)).to(DEV)
    o = torch.randn(lay_s.num_nodes + lay_t.num_nodes, R, device=DEV,
                    requires_grad=True)
    o_s, o_t = o[:lay_s.num_nodes], o[lay_s.num_nodes:]
    out = dense_ops.consensus_update(S_hat, o_s, o_t, mlp, lay_s, lay_t,
                                     o_joint=o if joint else None)
    with reference_mode():
        out2 = dense_ops.consensus_update(S_hat, o_s, o_t, mlp, lay_s, lay_t)
    assert torch.allclose(out, out2, atol=1e-4)
    g = torch.randn_like(out)
    inputs = (S_hat, o) + tuple(mlp.parameters())
    ga = torch.autograd.grad(out, inputs, g)
    gb = torch.autograd.grad(out2, inputs, g)
    for a, b in zip(ga, gb):
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize('shape', [(1, 300, 700, 256), (3, 50, 64, 32),
                                   (2, 130, 129, 100)])
@pytest.mark.parametrize('k', [1, 10, 20, 40])
@pytest.mark.parametrize('exact', [True, False])
def test_topk_dot(shape, k, exact):
    B, Ns, Nt, C = shape
    h_s = torch.randn(B, Ns, C, device=DEV)
    h_t = torch.randn(B, Nt, C, device=DEV)
    idx = sparse_corr.top_k(h_s, h_t, k, exact=exact)
    scores = h_s @ h_t.transpose(-1, -2)
    ref_val, ref_idx = scores.topk(k, dim=-1)
    got_val = torch.gather(scores, -1, idx)
    # split-bf16 scores: |error| <~ 2^-16 * sum|a||b| (~3e-3 at C=256)
    tol = 1e-4 if exact else 4e-3
    assert torch.allclose(got_val, ref_val, atol=tol)
    assert (got_val[..., :-1] >= got_val[..., 1:] - tol).all()
    assert (idx >= 0).all() and (idx < Nt).all()
    # the candidate sets agree except at near-ties
    same = (idx.sort(-1)[0] == ref_idx.sort(-1)[0]).float().mean().item()
    assert same > (0.999 if exact else 0.98)


def _hub_case(B, Ns, Nt, C, seed):
    """Hub-heavy scores with near-ties: low-rank sources, a few large-norm
    hub targets that rank first for most rows, exact duplicates and
    near-duplicates (differences at the last fp32 bits)."""
    g = torch.Generator().manual_seed(seed)
    basis = torch.randn(B, 4, C, generator=g)
    h_s = torch.randn(B, Ns, 4, generator=g) @ basis + \
        1e-3 * torch.randn(B, Ns, C, generator=g)
    h_t = torch.randn(B, Nt, C, generator=g)
    h_t[:, :8] *= 6.0                                   # hubs
    h_t[:, Nt - 40:Nt - 20] = h_t[:, 100:120]          # exact ties
    h_t[:, Nt - 20:] = h_t[:, 200:220] * (1 + 2e-7)     # near-ties
    return h_s.to(DEV), h_t.to(DEV)


@pytest.mark.parametrize('case', ['random', 'hub', 'clustered'])
@pytest.mark.parametrize('k', [1, 10, 16])
def test_topk_exact_refined_equals_brute_force(case, k):
    """The default exact selection (split-bf16 filter + exact fp32
    re-score, exhaustive fallback) returns exactly the brute-force exact-f32
    MFMA kernel's indices (order included: score desc, index asc)."""
    from deep_graph_matching_consensus_amd.ops import _backend
    if case == 'random':
        torch.manual_seed(1)
        h_s = torch.randn(2, 700, 256, device=DEV)
        h_t = torch.randn(2, 1500, 256, device=DEV)
    elif case == 'hub':
        h_s, h_t = _hub_case(1, 2000, 3000, 256, seed=3)
    else:   # every target a near-copy of one of 5 centres: many near-ties
        g = torch.Generator().manual_seed(5)
        cent = torch.randn(5, 64, generator=g)
        h_t = (cent[torch.randint(0, 5, (2500, ), generator=g)] +
               1e-6 * torch.randn(2500, 64, generator=g))[None].to(DEV)
        h_s = torch.randn(1, 900, 64, generator=g).to(DEV)
    want = sparse_corr.top_k(h_s, h_t, k, brute_force=True)
    got, n_over = _backend.ops().topk_dot_refined_stats(
        h_s.contiguous(), h_t.contiguous(), k)
    assert torch.equal(got, want)
    assert torch.equal(sparse_corr.top_k(h_s, h_t, k), want)  # the default
    if case == 'random':
        assert int(n_over) == 0      # the margin covers random inputs


@pytest.mark.parametrize('case', ['random', 'hub', 'clustered'])
def test_topk_warm_start_same_output(case):
    """The filter's warm start (a persistent candidate state re-scored into
    per-row lower bounds of the threshold, ``topk_warm_kernel``) never
    changes the selection: cold state, the previous call's state on the
    same or on perturbed embeddings (training steps), the WORST targets as
    the state (weak bounds), and garbage states (duplicates, out-of-range
    indices) all give the brute-force exact indices."""
    if case == 'random':
        torch.manual_seed(1)
        h_s = torch.randn(2, 700, 256, device=DEV)
        h_t = torch.randn(2, 1500, 256, device=DEV)
    elif case == 'hub':
        h_s, h_t = _hub_case(1, 2000, 3000, 256, seed=3)
    else:
        g = torch.Generator().manual_seed(5)
        cent = torch.randn(5, 64, generator=g)
        h_t = (cent[torch.randint(0, 5, (2500, ), generator=g)] +
               1e-6 * torch.randn(2500, 64, generator=g))[None].to(DEV)
        h_s = torch.randn(1, 900, 64, generator=g).to(DEV)
    B, Ns, _ = h_s.shape
    Nt = h_t.size(1)
    state = torch.full((B, Ns, 32), -1, dtype=torch.long, device=DEV)
    want = sparse_corr.top_k(h_s, h_t, 10, brute_force=True)
    assert torch.equal(sparse_corr.top_k(h_s, h_t, 10, warm=state), want)
    assert bool((state[..., :16] >= 0).all())         # kept for next call
    assert torch.equal(sparse_corr.top_k(h_s, h_t, 10, warm=state), want)
    # a "training step": perturbed embeddings, previous state
    g = torch.Generator(device=DEV).manual_seed(9)
    h_s2 = h_s + 0.05 * torch.randn(h_s.shape, device=DEV, generator=g)
    h_t2 = h_t + 0.05 * torch.randn(h_t.shape, device=DEV, generator=g)
    want2 = sparse_corr.top_k(h_s2, h_t2, 10, brute_force=True)
    assert torch.equal(sparse_corr.top_k(h_s2, h_t2, 10, warm=state), want2)
    # weak bounds: the 16 worst targets of every row
    worst = sparse_corr.top_k(-h_s2, h_t2, 16, brute_force=True)
    state[..., :16] = worst
    assert torch.equal(sparse_corr.top_k(h_s2, h_t2, 10, warm=state), want2)
    # garbage: duplicates, negative and out-of-range indices
    bad = torch.randint(0, 4, (B, Ns, 32), device=DEV)
    bad[:, ::3, 5] = Nt + 7
    bad[:, 1::3, 2] = -5
    state.copy_(bad)
    assert torch.equal(sparse_corr.top_k(h_s2, h_t2, 10, warm=state), want2)


@pytest.mark.parametrize('exact', [True, False])
def test_topk_nonfinite_rows_give_valid_indices(exact):
    """Rows (or targets) holding NaN / Inf still produce k in-range indices
    (the consumers gather with them); finite rows are unaffected."""
    torch.manual_seed(2)
    h_s = torch.randn(1, 300, 64, device=DEV)
    h_t = torch.randn(1, 900, 64, device=DEV)
    want = sparse_corr.top_k(h_s, h_t, 10, brute_force=True)
    h_s[0, 5, 0] = float('nan')
    h_s[0, 6, :] = float('nan')
    h_s[0, 7, 3] = float('inf')
    idx = sparse_corr.top_k(h_s, h_t, 10, exact=exact)
    torch.cuda.synchronize()
    assert (idx >= 0).all() and (idx < 900).all()
    ok = torch.ones(300, dtype=torch.bool)
    ok[5:8] = False
    if exact:
        assert torch.equal(idx[0, ok], want[0, ok])
    h_t[0, 11, 0] = float('nan')
    idx = sparse_corr.top_k(h_s, h_t, 10, exact=exact)
    torch.cuda.synchronize()
    assert (idx >= 0).all() and (idx < 900).all()


@pytest.mark.parametrize('Ns,Nt', [(4000, 3000), (200, 5000)])
def test_topk_dot_split_merge(Ns, Nt):
    """Few source rows -> the target range is split over blocks and the
    per-split lists are merged (bf16x3 path); compare with exact-f32."""
    torch.manual_seed(0)
    h_s = torch.randn(1, Ns, 64, device=DEV)
    h_t = torch.randn(1, Nt, 64, device=DEV)
    # duplicated targets -> exact ties must resolve to the lower index
    h_t[0, Nt // 2:Nt // 2 + 7] = h_t[0, 3:10]
    a = sparse_corr.top_k(h_s, h_t, 10, exact=False)
    b = sparse_corr.top_k(h_s, h_t, 10, brute_force=True)
    assert torch.equal(sparse_corr.top_k(h_s, h_t, 10, exact=True), b)
    scores = h_s @ h_t.transpose(-1, -2)
    va, vb = torch.gather(scores, -1, a), torch.gather(scores, -1, b)
    assert torch.allclose(va, vb, atol=1e-3)
    assert (a == b).float().mean().item() > 0.99


@pytest.mark.parametrize('B,Ns,Nt,C', [(1, 3000, 9000, 256),
                                        (2, 1000, 4000, 128),
                                        (1, 4900, 6001, 256),
                                        (3, 300, 2000, 64)])
def test_topk_split_shapes(B, Ns, Nt, C):
    """The filter on split target ranges of several shapes (batches, C =
    64 / 128 / 256, row blocks that do not fill the chip): exact selection
    == brute force, the split-bf16 one within its score tolerance."""
    torch.manual_seed(B + Ns)
    h_s = torch.randn(B, Ns, C, device=DEV)
    h_t = torch.randn(B, Nt, C, device=DEV)
    want = sparse_corr.top_k(h_s, h_t, 10, brute_force=True)
    assert torch.equal(sparse_corr.top_k(h_s, h_t, 10), want)
    got = sparse_corr.top_k(h_s, h_t, 10, exact=False)
    assert (got >= 0).all() and (got < Nt).all()
    scores = h_s @ h_t.transpose(-1, -2)
    torch.testing.assert_close(torch.gather(scores, -1, got),
                               torch.gather(scores, -1, want), atol=4e-3,
                               rtol=0)


def test_dgmc_dense_hip_vs_reference_mode():
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, DevicePairLoader, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    groups = make_keypoint_datasets(graphs=8, feature_dim=32, seed=0)
    store = GraphStore(groups, DEV)
    batch = next(iter(DevicePairLoader(store, batch_size=24, seed=0)))
    torch.manual_seed(3)
    model = DGMC(SplineCNN(32, 32, 2, 2, cat=False),
                 SplineCNN(16, 16, 2, 2, cat=True), num_steps=3).to(DEV)
    args = (batch.x_s, batch.edge_index_s, batch.edge_attr_s,
            batch.x_s_batch, batch.x_t, batch.edge_index_t,
            batch.edge_attr_t, batch.x_t_batch)
    y = torch.stack([torch.arange(batch.y.numel(), device=DEV), batch.y])

    torch.manual_seed(5)
    S_0, S_L = model(*args)
    loss = model.loss(S_0, y) + model.loss(S_L, y)
    grads = torch.autograd.grad(loss, list(model.parameters()))
    with reference_mode():
        torch.manual_seed(5)
        R_0, R_L = model(*args)
        loss2 = model.loss(R_0, y) + model.loss(R_L, y)
        grads2 = torch.autograd.grad(loss2, list(model.parameters()))
    assert torch.allclose(S_0, R_0, atol=1e-4)
    assert torch.allclose(S_L, R_L, atol=1e-4)
    assert torch.allclose(loss, loss2, atol=1e-4)
    for a, b in zip(grads, grads2):
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-2)


def test_dgmc_folded_projection_matches_unfolded(monkeypatch):
    """psi_2's final Linear folded into the consensus MLP's first layer
    (one GEMM on the pre-projection features) gives the same outputs and
    gradients as the two-GEMM form (the final bias' gradient is exactly 0)."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, DevicePairLoader, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.models import dgmc as dgmc_mod
    groups = make_keypoint_datasets(graphs=8, feature_dim=32, seed=0)
    store = GraphStore(groups, DEV)
    batch = next(iter(DevicePairLoader(store, batch_size=24, seed=0)))
    torch.manual_seed(3)
    model = DGMC(SplineCNN(32, 32, 2, 2, cat=False),
                 SplineCNN(16, 16, 2, 2, cat=True), num_steps=3).to(DEV)
    args = (batch.x_s, batch.edge_index_s, batch.edge_attr_s,
            batch.x_s_batch, batch.x_t, batch.edge_index_t,
            batch.edge_attr_t, batch.x_t_batch)
    y = torch.stack([torch.arange(batch.y.numel(), device=DEV), batch.y])

    def run(fold):
        monkeypatch.setattr(dgmc_mod, 'FOLD_PROJECTION', fold)
        torch.manual_seed(5)
        S_0, S_L = model(*args)
        loss = model.loss(S_0, y) + model.loss(S_L, y)
        return S_L, torch.autograd.grad(loss, list(model.parameters()))

    S1, g1 = run(True)
    S0, g0 = run(False)
    assert torch.allclose(S1, S0, atol=1e-4)
    names = [n for n, _ in model.named_parameters()]
    for n, a, b in zip(names, g1, g0):
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-2), n
    assert float(g1[names.index('psi_2.final.bias')].abs().max()) == 0.0


def test_dgmc_sparse_folded_projection_matches_unfolded(monkeypatch):
    """Sparse (top-k) path: psi_2's final Linear folded into the consensus
    MLP (one node GEMM on psi_2's joint features) == the unfolded form,
    outputs and parameter gradients (the final bias' gradient is 0)."""
    from deep_graph_matching_consensus_amd.models import DGMC, RelCNN
    from deep_graph_matching_consensus_amd.models import dgmc as dgmc_mod
    torch.manual_seed(0)
    N, E = 400, 2000
    x1 = torch.randn(N, 24, device=DEV)
    x2 = x1[torch.randperm(N, device=DEV)] + 0.1 * torch.randn(N, 24,
                                                             device=DEV)
    e1 = torch.randint(N, (2, E), device=DEV)
    e2 = torch.randint(N, (2, E), device=DEV)
    model = DGMC(RelCNN(24, 32, 2), RelCNN(8, 8, 2), num_steps=3,
                 k=5).to(DEV)
    y = torch.stack([torch.arange(60, device=DEV),
                     torch.randint(N, (60, ), device=DEV)])

    def run(fold):
        monkeypatch.setattr(dgmc_mod, 'FOLD_PROJECTION', fold)
        torch.manual_seed(7)
        _, S_L = model(x1, e1, None, None, x2, e2, None, None, y)
        loss = model.loss(S_L, y)
        grads = torch.autograd.grad(loss, list(model.parameters()),
                                    allow_unused=True)
        return S_L, grads

    S1, g1 = run(True)
    S0, g0 = run(False)
    assert torch.equal(S1.__idx__, S0.__idx__)
    assert torch.allclose(S1.__val__, S0.__val__, atol=1e-5)
    names = [n for n, _ in model.named_parameters()]
    for n, a, b in zip(names, g1, g0):
        if n == 'psi_2.final.bias':
            assert a is None or float(a.abs().max()) == 0.0
            continue
        if a is None or b is None:      # unused modules (e.g. BN, off)
            assert a is None and b is None, n
            continue
        assert torch.allclose(a, b, atol=1e-4, rtol=1e-3), n


def test_dgmc_sparse_gpu_matches_dense():
    from deep_graph_matching_consensus_amd.models import DGMC, GIN
    torch.manual_seed(0)
    x = torch.randn(30, 16, device=DEV)
    ei = torch.randint(30, (2, 90), device=DEV)
    model = DGMC(GIN(16, 16, 2), GIN(8, 8, 2), num_steps=2).to(DEV)
    torch.manual_seed(1)
    S1_0, S1_L = model(x, ei, None, None, x, ei, None, None)
    model.k = 30
    torch.manual_seed(1)
    S2_0, S2_L = model(x, ei, None, None, x, ei, None, None)
    assert torch.allclose(S1_0, S2_0.to_dense(), atol=1e-5)
    assert torch.allclose(S1_L, S2_L.to_dense(), atol=1e-4)


def test_graph_captured_step_matches_eager():
    """hipGraph replay of a static-shape step == eager on the same batch."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets.static_batch import \
        StaticPairBatcher
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.runtime import GraphedStep
    groups = make_keypoint_datasets(graphs=8, feature_dim=32, seed=0)
    store = GraphStore(groups, DEV)
    batcher = StaticPairBatcher(store, 24, seed=0)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(32, 32, 2, 2, cat=False),
                 SplineCNN(16, 16, 2, 2, cat=True), num_steps=0).to(DEV)
    rows = torch.arange(batcher.cap_s, device=DEV)
    out = {}

    def body():
        for p in model.parameters():
            p.grad = None
        b = batcher.materialize()
        with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
            S_0, _ = model(b.x_s, b.edge_index_s, b.edge_attr_s, b.x_s_batch,
                           b.x_t, b.edge_index_t, b.edge_attr_t, b.x_t_batch)
        y = torch.stack([rows, b.y])
        loss = model.loss(S_0, y, mask=b.y_mask)
        out['loss'] = loss.detach()
        out['g'] = torch.autograd.grad(loss, model.psi_1.convs[0].weight)[0]

    ids = [batcher.next_ids() for _ in range(3)]
    assert batcher.load(*ids[0])
    step = GraphedStep(body, warmup=2).capture()
    graph_out = dict(out)   # tensors owned by the captured graph
    results = []
    for s, t in ids[1:]:
        assert batcher.load(s, t)
        step()
        torch.cuda.synchronize()
        replay = (graph_out['loss'].clone(), graph_out['g'].clone())
        body()   # eager on the same static inputs
        torch.cuda.synchronize()
        results.append((replay, (out['loss'], out['g'])))
    for (la, ga), (lb, gb) in results:
        assert torch.isfinite(la)
        assert torch.allclose(la, lb, atol=1e-5)
        assert torch.allclose(ga, gb, atol=1e-5, rtol=1e-4)
    assert not torch.allclose(results[0][0][0], results[1][0][0])


def _cand_inputs(B=3, Ns=37, Nt=41, k=7, C=48, hub=False):
    S_idx = torch.randint(Nt, (B, Ns, k), device=DEV)
    if hub:
        # Hub targets (the hubness of random embeddings): target 0 of every
        # batch element in most rows, target 3 in a third of them - columns
        # of hundreds of entries, walked in several pieces.
        S_idx[:, : Ns * 9 // 10, 0] = 0
        S_idx[:, ::3, 1] = 3
    return S_idx, sparse_corr.CandidateGraph(S_idx, Nt)


@pytest.mark.parametrize('C,hub', [(16, False), (100, False), (256, False),
                                   (32, True), (256, True), (100, True)])
def test_sparse_gather_dot(C, hub):
    B, Ns, Nt, k = 3, 37, 41, 7
    if hub:
        Ns = 700
    S_idx, cand = _cand_inputs(B, Ns, Nt, k, hub=hub)
    h_s = torch.randn(B, Ns, C, device=DEV, requires_grad=True)
    h_t = torch.randn(B, Nt, C, device=DEV, requires_grad=True)
    out = sparse_corr.gather_dot(h_s, h_t, S_idx, cand)
    out2 = sparse_corr.gather_dot(h_s, h_t, S_idx, None)
    assert torch.allclose(out, out2, atol=1e-4)
    g = torch.randn_like(out)
    ga = torch.autograd.grad(out, (h_s, h_t), g)
    gb = torch.autograd.grad(out2, (h_s, h_t), g)
    for a, b in zip(ga, gb):
        assert torch.allclose(a, b, atol=1e-4)


@pytest.mark.parametrize('R,hub', [(8, False), (32, False), (130, False),
                                   (32, True), (4, True), (256, True)])
def test_sparse_transport(R, hub):
    B, Ns, Nt, k = 2, 29, 31, 6
    if hub:
        Ns = 900
    S_idx, cand = _cand_inputs(B, Ns, Nt, k, hub=hub)
    S = torch.rand(B, Ns, k, device=DEV, requires_grad=True)
    r_s = torch.randn(B, Ns, R, device=DEV)
    out = sparse_corr.sparse_transport(S, r_s, S_idx, Nt, cand)
    out2 = sparse_corr.sparse_transport(S, r_s, S_idx, Nt, None)
    # hub columns sum hundreds of terms (in a different order than the
    # scatter_add oracle): relative tolerance
    tol = 1e-3 if hub else 1e-5
    assert torch.allclose(out, out2, atol=tol, rtol=1e-5)
    g = torch.randn_like(out)
    assert torch.allclose(torch.autograd.grad(out, S, g)[0],
                          torch.autograd.grad(out2, S, g)[0], atol=1e-4)


@pytest.mark.parametrize('R,hub', [(8, False), (32, False), (70, False),
                                   (32, True), (64, True), (70, True)])
def test_sparse_consensus(R, hub):
    B, Ns, Nt, k = 2, 23, 27, 5
    if hub:
        Ns = 800
    S_idx, cand = _cand_inputs(B, Ns, Nt, k, hub=hub)
    mlp = torch.nn.Sequential(torch.nn.Linear(R, R), torch.nn.ReLU(),
                              torch.nn.Linear(R, 1)).to(DEV)
    S_hat = torch.randn(B, Ns, k, device=DEV, requires_grad=True)
    o_s = torch.randn(B, Ns, R, device=DEV, requires_grad=True)
    o_t = torch.randn(B, Nt, R, device=DEV, requires_grad=True)
    out = sparse_corr.consensus_update(S_hat, o_s, o_t, S_idx, mlp, cand)
    out2 = sparse_corr.consensus_update(S_hat, o_s, o_t, S_idx, mlp, None)
    assert torch.allclose(out, out2, atol=1e-4)
    g = torch.randn_like(out)
    inputs = (S_hat, o_s, o_t) + tuple(mlp.parameters())
    ga = torch.autograd.grad(out, inputs, g)
    gb = torch.autograd.grad(out2, inputs, g)
    for a, b in zip(ga, gb):
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-3)


def test_dgmc_sparse_training_hip_vs_reference(monkeypatch):
    """RelCNN + top-k (DBP15K-style) forward/backward: HIP == oracle.  The
    native path draws its random negatives in the candidate kernel (Philox,
    csrc/hip/candidates.hip), the oracle with ``torch.randint``: the oracle
    run is handed the native negatives, so both see one candidate set."""
    from deep_graph_matching_consensus_amd.models import DGMC, RelCNN
    torch.manual_seed(0)
    N, E = 300, 1500
    x1 = torch.randn(N, 24, device=DEV)
    x2 = x1[torch.randperm(N, device=DEV)] + 0.1 * torch.randn(N, 24,
                                                             device=DEV)
    e1 = torch.randint(N, (2, E), device=DEV)
    e2 = torch.randint(N, (2, E), device=DEV)
    model = DGMC(RelCNN(24, 32, 2), RelCNN(8, 8, 2), num_steps=2,
                 k=5).to(DEV)
    y = torch.stack([torch.arange(50, device=DEV),
                     torch.randint(N, (50, ), device=DEV)])
    torch.manual_seed(1)
    _, S_L = model(x1, e1, None, None, x2, e2, None, None, y)
    loss = model.loss(S_L, y)
    grads = torch.autograd.grad(loss, list(model.parameters()),
                                allow_unused=True)
    negs = S_L.__idx__[:, 5:].contiguous()
    randint = torch.randint

    def native_negatives(high, size, **kw):
        if tuple(size) == (1, N, negs.size(1)):
            return negs.view(size).clone()
        return randint(high, size, **kw)
    monkeypatch.setattr(torch, 'randint', native_negatives)
    with reference_mode():
        torch.manual_seed(1)
        _, R_L = model(x1, e1, None, None, x2, e2, None, None, y)
        loss2 = model.loss(R_L, y)
        grads2 = torch.autograd.grad(loss2, list(model.parameters()),
                                     allow_unused=True)
    assert torch.equal(S_L.__idx__, R_L.__idx__)
    assert torch.allclose(S_L.__val__, R_L.__val__, atol=1e-4)
    assert torch.allclose(loss, loss2, atol=1e-4)
    for a, b in zip(grads, grads2):
        if a is None or b is None:
            assert a is None and b is None
        else:
            assert torch.allclose(a, b, atol=1e-3, rtol=1e-2)


@pytest.mark.parametrize('rows', [1, 63, 1000, 20000])
@pytest.mark.parametrize('C', [1, 5, 128, 300])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_col_sum_and_relu_bias_accumulate(rows, C, dtype):
    ops = _backend.ops()
    src = torch.randn(rows, C, device=DEV).to(dtype)
    ref_sum = src.float().sum(0)
    out = ops.col_sum(src)
    assert torch.allclose(out, ref_sum, atol=1e-3, rtol=1e-4)
    # Accumulate into an existing buffer (loop-shared gradients).
    acc = torch.ones(C, device=DEV)
    ops.col_sum(src, acc, True)
    assert torch.allclose(acc, ref_sum + 1, atol=1e-3, rtol=1e-4)
    # relu_bias_bwd: g' = grad * (out > 0); dbias = sum g'.
    grad = torch.randn(rows, C, device=DEV).to(dtype)
    o = torch.randn(rows, C, device=DEV).to(dtype)
    g, db = ops.relu_bias_bwd(grad, o, True, dtype)
    gm = grad.float() * (o.float() > 0)
    assert torch.allclose(g.float(), gm, atol=1e-2, rtol=1e-2)
    assert torch.allclose(db, gm.sum(0), atol=1e-3, rtol=1e-4)
    buf = torch.full((C, ), 2.0, device=DEV)
    g2, db2 = ops.relu_bias_bwd(grad, o, True, dtype, buf, True)
    assert torch.allclose(buf, gm.sum(0) + 2, atol=1e-3, rtol=1e-4)
    # Partials-only mode (loop-gradient stacks): the caller folds.
    from deep_graph_matching_consensus_amd.ops.gemm import col_partial_rows
    part = torch.empty(col_partial_rows(rows), C, device=DEV)
    ops.col_sum(src, None, False, part)
    assert torch.allclose(part.sum(0), ref_sum, atol=1e-3, rtol=1e-4)
    part2 = torch.empty_like(part)
    g3, _ = ops.relu_bias_bwd(grad, o, True, dtype, None, False, part2)
    assert torch.allclose(part2.sum(0), gm.sum(0), atol=1e-3, rtol=1e-4)
    # Column slice of a wider gradient (one block of a concatenation).
    wide = torch.randn(rows, 3 * C + 8, device=DEV).to(dtype)
    gs = wide[:, C + 8:2 * C + 8]
    g4, db4 = ops.relu_bias_bwd(gs, o, True, dtype)
    gsm = gs.float() * (o.float() > 0)
    assert torch.equal(g4, ops.relu_bias_bwd(gs.contiguous(), o, True,
                                             dtype)[0])
    assert torch.allclose(db4, gsm.sum(0), atol=1e-3, rtol=1e-4)
    g5, db5 = ops.relu_bias_bwd(gs, gs, False, dtype)
    assert torch.equal(g5.float(), gs.float())
    assert torch.allclose(db5, gs.float().sum(0), atol=1e-3, rtol=1e-4)
    # Deterministic: repeated calls are bit-identical.
    assert torch.equal(ops.col_sum(src), ops.col_sum(src))


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_consensus_update_bf16_node_operands(dtype):
    # The training path feeds bf16 P/Q (encoder GEMM dtype): compare the HIP
    # kernels against the fp32 oracle on the same rounded operands.
    B, Ns, Nt, R = 7, 19, 17, 128
    lay_s, lay_t = _layouts(B, Ns, Nt)
    S_hat = torch.randn(B, Ns, Nt, device=DEV, requires_grad=True)
    mlp = torch.nn.Sequential(torch.nn.Linear(R, R), torch.nn.ReLU(),
                              torch.nn.Linear(R, 1)).to(DEV)
    o = torch.randn(lay_s.num_nodes + lay_t.num_nodes, R, device=DEV)
    o = o.to(dtype).requires_grad_()
    o_s, o_t = o[:lay_s.num_nodes], o[lay_s.num_nodes:]
    with torch.autocast('cuda', dtype=torch.bfloat16,
                        enabled=dtype != torch.float32):
        out = dense_ops.consensus_update(S_hat, o_s, o_t, mlp, lay_s, lay_t,
                                         o_joint=o)
    with reference_mode():
        out2 = dense_ops.consensus_update(S_hat, o_s.float(), o_t.float(),
                                          mlp, lay_s, lay_t)
    tol = 1e-4 if dtype == torch.float32 else 0.1
    assert torch.allclose(out, out2, atol=tol, rtol=tol)
    g = torch.randn_like(out)
    ga = torch.autograd.grad(out, (S_hat, ) + tuple(mlp.parameters()), g)
    gb = torch.autograd.grad(out2, (S_hat, ) + tuple(mlp.parameters()), g)
    assert torch.equal(ga[0], gb[0])
    for a, b in zip(ga[1:], gb[1:]):
        rel = (a - b).norm() / b.norm().clamp(min=1e-6)
        assert rel < (1e-4 if dtype == torch.float32 else 5e-2), rel


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_cat_rows(dtype):
    parts = [torch.randn(n, 384, device=DEV).to(dtype) for n in
             (1, 7, 1000, 9216)]
    parts.append(torch.randn(500, 512, device=DEV).to(dtype)[:, 128:512])
    out = _backend.ops().cat_rows(parts)
    assert torch.equal(out, torch.cat(parts))
    buf = torch.empty_like(out)
    _backend.ops().cat_rows(parts, buf)
    assert torch.equal(buf, out)


def test_split_k_accumulate():
    from deep_graph_matching_consensus_amd.ops.gemm import matmul_tn_fp32
    a = torch.randn(9999, 128, device=DEV).bfloat16()
    b = torch.randn(9999, 384, device=DEV).bfloat16()
    ref_ = a.float().t() @ b.float()
    out = matmul_tn_fp32(a, b)
    assert torch.allclose(out, ref_, atol=0.05, rtol=1e-3)
    buf = torch.ones(128, 384, device=DEV)
    matmul_tn_fp32(a, b, out=buf, accumulate=True)
    assert torch.allclose(buf, ref_ + 1, atol=0.05, rtol=1e-3)


def _slot_op(N, S, E, device):
    """Random slot-structured operator [N, N*S] (SplineConv-like)."""
    row = torch.randint(N, (E, ), device=device)
    j = torch.randint(N, (E, ), device=device)
    k = torch.randint(S - 1, (E, ), device=device)
    val = torch.rand(E, device=device)
    ar = torch.arange(N, device=device)
    row = torch.cat([row, ar])
    col = torch.cat([j * S + k, ar * S + (S - 1)])
    val = torch.cat([val, torch.ones(N, device=device)])
    return SparseOperator.from_coo(row, col, val, N, N * S)


@pytest.mark.parametrize('N,K,M', [(300, 128, 3328), (257, 3328, 128),
                                   (64, 64, 96), (100, 32, 130)])
def test_gemm_abt(N, K, M):
    ops = _backend.ops()
    a = torch.randn(N, K, device=DEV).bfloat16()
    bt = torch.randn(M, K, device=DEV).bfloat16()
    ref_ = a.float() @ bt.float().t()
    out = ops.gemm_abt(a, bt)
    assert torch.allclose(out.float(), ref_, atol=0.1, rtol=1e-2)
    acc = torch.ones(N, M, device=DEV)
    ops.gemm_abt(a, bt, acc, True)
    assert torch.allclose(acc, ref_ + 1, atol=0.1, rtol=1e-2)


@pytest.mark.parametrize('shape', [(7, 13, 17), (3, 64, 64), (64, 19, 19)])
def test_masked_softmax_packed(shape):
    lay_s, lay_t = _layouts(*shape)
    S_hat = torch.randn(shape, device=DEV, requires_grad=True)
    out = dense_ops.masked_softmax_packed(S_hat, lay_s, lay_t)
    S2 = S_hat.detach().clone().requires_grad_()
    out2 = lay_s.to_sparse(ref.masked_softmax(S2, _mask(lay_s, lay_t)))
    assert out.shape == out2.shape
    assert torch.allclose(out, out2, atol=1e-6)
    g = torch.randn_like(out)
    assert torch.allclose(torch.autograd.grad(out, S_hat, g)[0],
                          torch.autograd.grad(out2, S2, g)[0], atol=1e-5)


@pytest.mark.parametrize('masked', [False, True])
@pytest.mark.parametrize('reduction', ['mean', 'sum'])
def test_fused_nll_and_hits(masked, reduction):
    from deep_graph_matching_consensus_amd.models import DGMC, MLP
    rows, Nt, G = 777, 23, 500
    S = torch.randn(rows, Nt, device=DEV).softmax(-1).requires_grad_()
    y = torch.stack([torch.randperm(rows, device=DEV)[:G],
                     torch.randint(0, Nt, (G, ), device=DEV)])
    mask = (torch.rand(G, device=DEV) > 0.3) if masked else None
    model = DGMC(MLP(4, 4, 1), MLP(4, 4, 1), num_steps=1)
    loss = model.loss(S, y, reduction=reduction, mask=mask)
    with reference_mode():
        loss2 = model.loss(S, y, reduction=reduction, mask=mask)
    assert torch.allclose(loss, loss2, rtol=1e-5, atol=1e-6)
    ga = torch.autograd.grad(loss, S)[0]
    gb = torch.autograd.grad(loss2, S)[0]
    assert torch.allclose(ga, gb, rtol=1e-5, atol=1e-6)
    l3, cnt, cor = model.loss_stats(S, y, mask)
    m = mask if masked else torch.ones(G, dtype=torch.bool, device=DEV)
    assert int(cnt) == int(m.sum())
    pred = S.detach()[y[0]].argmax(-1)
    assert int(cor) == int(((pred == y[1]) & m).sum())


def _sparse_S(val, idx, Nt):
    rows, k = val.shape
    row = torch.arange(rows, device=val.device).view(-1, 1).expand(-1, k)
    S = torch.sparse_coo_tensor(torch.stack([row.reshape(-1),
                                             idx.reshape(-1)]),
                                val.reshape(-1), (rows, Nt),
                                requires_grad=val.requires_grad)
    S.__idx__, S.__val__ = idx, val
    return S


@pytest.mark.parametrize('masked', [False, True])
@pytest.mark.parametrize('reduction', ['mean', 'sum'])
def test_fused_sparse_nll_and_hits(masked, reduction):
    """Native sparse NLL (loss.hip::sparse_nll_*) against the reference
    expression (dgmc.py:258-266): ground truths outside the candidates,
    duplicated ground truths (same row and target, same row other target),
    ties in the candidate values, and the ground-truth mask."""
    from deep_graph_matching_consensus_amd.models import DGMC, MLP
    g = torch.Generator(device='cpu').manual_seed(3)
    rows, Nt, k, G = 901, 4000, 12, 600
    idx = torch.stack([torch.randperm(Nt, generator=g)[:k]
                       for _ in range(rows)]).to(DEV)
    val = torch.randn(rows, k, generator=g).to(DEV).softmax(-1)
    val[5, 3] = val[5, 7] = val[5].max()        # tie: first slot wins
    val = val.requires_grad_()
    y0 = torch.randperm(rows, generator=g)[:G].to(DEV)
    slot = torch.randint(0, k, (G, ), generator=g).to(DEV)
    y1 = idx[y0, slot]
    y1[::7] = torch.randint(0, Nt, (y1[::7].numel(), ), generator=g).to(DEV)
    y0 = torch.cat([y0, y0[:20], y0[20:30]])     # duplicated ground truths
    y1 = torch.cat([y1, y1[:20], idx[y0[20:30], (slot[20:30] + 1) % k]])
    y0[-1] = 5
    y1[-1] = idx[5, 7]
    y = torch.stack([y0, y1])
    mask = (torch.rand(y.size(1), generator=g) > 0.3).to(DEV) \
        if masked else None
    model = DGMC(MLP(4, 4, 1), MLP(4, 4, 1), num_steps=1)
    S = _sparse_S(val, idx, Nt)
    assert model._fused_sparse_nll_ok(S, y, reduction, mask)
    loss = model.loss(S, y, reduction=reduction, mask=mask)
    with reference_mode():
        loss2 = model.loss(S, y, reduction=reduction, mask=mask)
    assert torch.allclose(loss, loss2, rtol=1e-5, atol=1e-6)
    ga = torch.autograd.grad(loss, val)[0]
    gb = torch.autograd.grad(loss2, val)[0]
    assert torch.allclose(ga, gb, rtol=1e-5, atol=1e-7)
    assert torch.equal(ga, torch.autograd.grad(
        model.loss(S, y, reduction=reduction, mask=mask), val)[0])
    l3, cnt, cor = model.loss_stats(S, y, mask)
    m = mask if masked else torch.ones(y.size(1), dtype=torch.bool,
                                       device=DEV)
    assert int(cnt) == int(m.sum())
    pred = idx[y[0], val.detach()[y[0]].argmax(-1)]
    assert int(cor) == int(((pred == y[1]) & m).sum())
    if reduction == 'mean':
        assert torch.allclose(l3, loss2, rtol=1e-5, atol=1e-6)


def test_nonfinite_flag():
    x = torch.randn(1000003, device=DEV)
    flag = torch.full((), 7.0, device=DEV)
    cnt = torch.zeros(1, dtype=torch.float64, device=DEV)
    _backend.ops().nonfinite_flag(x, flag, cnt)
    assert float(flag) == 0.0 and float(cnt) == 0.0
    x[123457] = float('nan')
    _backend.ops().nonfinite_flag(x, flag, cnt)
    assert float(flag) == 1.0 and float(cnt) == 1.0
    x[123457] = 0.0
    x[-1] = float('inf')
    _backend.ops().nonfinite_flag(x, flag, cnt)
    assert float(flag) == 1.0 and float(cnt) == 2.0


def test_hip_adam_matches_torch_adam():
    """Multi-tensor HIP Adam == torch.optim.Adam (same state schema), skips
    on found_inf, and survives a state_dict round trip."""
    from deep_graph_matching_consensus_amd.runtime import optim as hip_optim
    torch.manual_seed(0)
    shapes = [(37, 5), (1, ), (4096 * 3 + 12, ), (128, 128)]
    p_ref = [torch.randn(s, device=DEV) for s in shapes]
    p_hip = [p.clone() for p in p_ref]
    flat = torch.zeros(sum((p.numel() + 3) // 4 * 4 for p in p_hip),
                       device=DEV)
    off = 0
    for p in p_hip:                      # grads as aligned flat-buffer views
        p.grad = flat[off:off + p.numel()].view_as(p)
        off += (p.numel() + 3) // 4 * 4
    ref = torch.optim.Adam([torch.nn.Parameter(p) for p in p_ref], lr=1e-2,
                           weight_decay=1e-3)
    hip_params = [torch.nn.Parameter(p) for p in p_hip]
    for p, q in zip(hip_params, p_hip):
        p.grad = q.grad
    opt = torch.optim.Adam(hip_params, lr=1e-2, weight_decay=1e-3)
    assert hip_optim.supported(opt)
    found = torch.zeros((), device=DEV)
    for it in range(4):
        grads = [torch.randn(s, device=DEV) for s in shapes]
        for p, g in zip(ref.param_groups[0]['params'], grads):
            p.grad = g.clone()
        for p, g in zip(hip_params, grads):
            p.grad.copy_(g)
        if it == 2:                      # non-finite step: skipped
            found.fill_(1.0)
            hip_optim.hip_adam_step(opt, found)
            found.zero_()
            continue
        ref.step()
        hip_optim.hip_adam_step(opt, found)
    for a, b in zip(ref.param_groups[0]['params'], hip_params):
        torch.testing.assert_close(b, a, atol=1e-6, rtol=1e-5)
    sd = opt.state_dict()
    assert float(sd['state'][0]['step']) == 3.0
    opt2 = torch.optim.Adam(hip_params, lr=1e-2, weight_decay=1e-3)
    opt2.load_state_dict(sd)
    hip_optim.hip_adam_step(opt2, None)
    assert float(opt2.state[hip_params[1]]['step']) == 4.0


def test_hip_adam_state_round_trip_through_torch_adam(tmp_path):
    """Per-parameter step counters: a HIP Adam state resumes under
    torch.optim.Adam (and back) along the same trajectory as torch Adam
    throughout, including a parameter whose first gradient arrives late."""
    from deep_graph_matching_consensus_amd.runtime import optim as hip_optim
    torch.manual_seed(1)
    shapes = [(33, 7), (128, ), (5, )]
    init = [torch.randn(s, device=DEV) for s in shapes]
    grads = [[torch.randn(s, device=DEV) for s in shapes] for _ in range(9)]

    def make():
        ps = [torch.nn.Parameter(p.clone()) for p in init]
        return ps, torch.optim.Adam(ps, lr=1e-2)

    def feed(ps, it):
        for j, (p, g) in enumerate(zip(ps, grads[it])):
            # parameter 2 gets no gradient in the first two steps
            p.grad = None if (j == 2 and it < 2) else g.clone()

    ref_ps, ref = make()
    for it in range(9):
        feed(ref_ps, it)
        ref.step()
    ps, opt = make()
    for it in range(3):                   # HIP
        feed(ps, it)
        hip_optim.hip_adam_step(opt)
    steps = [float(opt.state[p]['step']) for p in ps]
    assert steps == [3.0, 3.0, 1.0]
    path = str(tmp_path / 'opt.pt')
    torch.save(opt.state_dict(), path)
    opt_t = torch.optim.Adam(ps, lr=1e-2)
    opt_t.load_state_dict(torch.load(path, weights_only=True))
    for it in range(3, 6):                # torch
        feed(ps, it)
        opt_t.step()
    assert [float(opt_t.state[p]['step']) for p in ps] == [6.0, 6.0, 4.0]
    opt_h = torch.optim.Adam(ps, lr=1e-2)
    opt_h.load_state_dict(opt_t.state_dict())
    for it in range(6, 9):                # HIP again
        feed(ps, it)
        hip_optim.hip_adam_step(opt_h)
    assert [float(opt_h.state[p]['step']) for p in ps] == [9.0, 9.0, 7.0]
    ids = {opt_h.state[p]['step'].data_ptr() for p in ps}
    assert len(ids) == len(ps)            # never shared
    for a, b in zip(ref_ps, ps):
        torch.testing.assert_close(b, a, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize('K,cin,cout,root', [(25, 1024, 256, True),
                                             (25, 128, 128, True),
                                             (4, 3, 8, False)])
def test_spline_weight_pack_unpack(K, cin, cout, root):
    """Stacked SplineConv operand / gradient layouts vs torch permute+cat."""
    ops = _backend.ops()
    w = torch.randn(K, cin, cout, device=DEV)
    r = torch.randn(cin, cout, device=DEV) if root else None
    ref = w.permute(1, 0, 2).reshape(cin, K * cout)
    if root:
        ref = torch.cat([ref, r], dim=1)
    assert torch.equal(ops.spline_weight_pack(w, r, torch.float32), ref)
    assert torch.equal(ops.spline_weight_pack(w, r, torch.bfloat16),
                       ref.bfloat16())
    g = torch.randn_like(ref)
    gw, gr = ops.spline_weight_unpack(g, K, root)
    S = K + int(root)
    g3 = g.view(cin, S, cout)
    assert torch.equal(gw, g3[:, :K].permute(1, 0, 2))
    if root:
        assert torch.equal(gr, g3[:, K])


def test_spline_conv_packed_weight_gradients_match_stacked(monkeypatch):
    """SplineConv with the one-kernel packed operand == the permute + cat
    autograd path (forward and parameter gradients)."""
    from deep_graph_matching_consensus_amd.nn import conv as conv_mod
    torch.manual_seed(5)
    conv = conv_mod.SplineConv(64, 32, dim=2, kernel_size=5).to(DEV)
    N, E = 300, 1500
    ei = torch.randint(N, (2, E), device=DEV)
    attr = torch.rand(E, 2, device=DEV)
    x = torch.randn(N, 64, device=DEV)

    def run():
        conv.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = conv(x, ei, attr, act='relu')
        out.float().square().sum().backward()
        return out.detach().float(), [p.grad.clone() for p in
                                      (conv.weight, conv.root, conv.bias)]

    o1, g1 = run()
    orig = conv_mod.SplineConv.stacked_operands

    def stacked(self, dtype, like, plan=None):
        w = self.stacked_weight()
        return w, w.detach().to(dtype)
    monkeypatch.setattr(conv_mod.SplineConv, 'stacked_operands', stacked)
    o0, g0 = run()
    monkeypatch.setattr(conv_mod.SplineConv, 'stacked_operands', orig)
    torch.testing.assert_close(o1, o0, atol=0, rtol=0)
    for a, b in zip(g1, g0):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-6)


def test_pack_grads_multi_tensor():
    """pack_grads copies every gradient into its flat view (zeros for a
    missing one) in one launch."""
    ops = _backend.ops()
    sizes = [37 * 5, 4, 4096 * 3 + 12, 128 * 128, 8]
    pad = [(n + 3) // 4 * 4 for n in sizes]
    flat = torch.full((sum(pad), ), 7.0, device=DEV)
    views, grads, off = [], [], 0
    for i, (n, pn) in enumerate(zip(sizes, pad)):
        views.append(flat[off:off + n])
        grads.append(None if i == 1 else torch.randn(n, device=DEV))
        off += pn
    ops.pack_grads(grads, views)
    for g, v in zip(grads, views):
        if g is None:
            assert bool((v == 0).all())
        else:
            assert torch.equal(v, g)
    # Non-finite flags folded by the step-counter kernel: a finite step bumps
    # the counters, a step with an inf sets found_inf, counts a skip and
    # leaves the counters alone.
    steps = [torch.full((), 3.0, device=DEV) for _ in range(3)]
    found = torch.zeros((), device=DEV)
    skips = torch.zeros(1, dtype=torch.float64, device=DEV)
    flags = ops.pack_grads(grads, views, True)
    assert flags.dtype == torch.int32 and int(flags.sum()) == 0
    ops.adam_step_inc(steps, found, flags, skips)
    assert float(found) == 0 and float(skips) == 0
    assert all(float(t) == 4.0 for t in steps)
    grads[2][5000] = float('inf')
    flags = ops.pack_grads(grads, views, True)
    assert int(flags.sum()) == 1
    ops.adam_step_inc(steps, found, flags, skips)
    assert float(found) == 1 and float(skips) == 1
    assert all(float(t) == 4.0 for t in steps)


def test_spline_slot_images_match_permuted_pack():
    """Both slot-conv weight images from the parameters in one kernel ==
    slot_conv_image of the stacked bf16 operand."""
    from deep_graph_matching_consensus_amd.ops.sparse import (
        slot_conv_image, slot_k_order)
    ops = _backend.ops()
    w = torch.randn(25, 128, 128, device=DEV)
    r = torch.randn(128, 128, device=DEV)
    w_lp = ops.spline_weight_pack(w, r, torch.bfloat16)
    img_f, img_t = ops.spline_slot_images(w, r, slot_k_order(w.device))
    assert torch.equal(img_f, slot_conv_image(w_lp, 128, False))
    assert torch.equal(img_t, slot_conv_image(w_lp, 128, True))


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_pair_scores_matches_dense_bmm(dtype):
    """Per-pair S_hat = h_s h_t^T from the packed joint embedding (+ its
    backward into the joint rows, padding rows zero) vs to_dense + bmm."""
    torch.manual_seed(7)
    B, C = 37, 256
    n_s = torch.randint(1, 20, (B, ))
    n_t = torch.randint(1, 20, (B, ))
    pad_s, pad_t = 5, 3
    rows_s = int(n_s.sum()) + pad_s
    rows_t = int(n_t.sum()) + pad_t
    h = torch.randn(rows_s + rows_t, C, device=DEV).to(dtype) \
        .requires_grad_()
    ptr_s = torch.zeros(B + 1, dtype=torch.int32)
    ptr_t = torch.zeros(B + 1, dtype=torch.int32)
    ptr_s[1:] = torch.cumsum(n_s, 0)
    ptr_t[1:] = torch.cumsum(n_t, 0)
    Ns, Nt = int(n_s.max()), int(n_t.max())

    class Lay(object):
        pass
    lay_s, lay_t = Lay(), Lay()
    lay_s.ptr, lay_s.N = ptr_s.to(DEV), Ns
    lay_t.ptr, lay_t.N = ptr_t.to(DEV), Nt
    S = dense_ops.pair_scores(h, rows_s, lay_s, lay_t)
    hf = h.detach().float().requires_grad_()
    ref = torch.zeros(B, Ns, Nt, device=DEV)
    parts = []
    for b in range(B):
        a = hf[int(ptr_s[b]):int(ptr_s[b + 1])]
        t = hf[rows_s + int(ptr_t[b]):rows_s + int(ptr_t[b + 1])]
        parts.append((b, a, t))
    ref = torch.stack([torch.nn.functional.pad(
        a @ t.t(), (0, Nt - t.size(0), 0, Ns - a.size(0)))
        for b, a, t in parts])
    torch.testing.assert_close(S, ref, atol=1e-3, rtol=1e-4)
    g = torch.randn_like(ref)
    (dh, ) = torch.autograd.grad(S, h, g)
    (dref, ) = torch.autograd.grad(ref, hf, g)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(dh.float(), dref, atol=tol, rtol=tol)
    assert bool((dh[int(ptr_s[-1]):rows_s] == 0).all())
    assert bool((dh[rows_s + int(ptr_t[-1]):] == 0).all())


@pytest.mark.parametrize('num_steps', [0, 3])
def test_objective_fused_softmax_nll_matches_unfused(monkeypatch, num_steps):
    """DGMC.objective with the fused softmax + NLL kernels == forward +
    masked_softmax_packed + NLL (loss, count, Hits@1 count, gradients)."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets.static_batch import \
        StaticPairBatcher
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    groups = make_keypoint_datasets(graphs=16, feature_dim=32, seed=4)
    store = GraphStore(groups, torch.device(DEV))
    batcher = StaticPairBatcher(store, 48, seed=2)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(32, 64, 2, 2, cat=False),
                 SplineCNN(16, 16, 2, 2, cat=True),
                 num_steps=num_steps).to(DEV)
    model.eval()
    assert batcher.load()
    batch = batcher.materialize()

    def run():
        torch.manual_seed(1)
        loss, count, correct = model.objective(
            batch.x_s, batch.edge_index_s, batch.edge_attr_s, batch.x_s_batch,
            batch.x_t, batch.edge_index_t, batch.edge_attr_t,
            batch.x_t_batch, batch.y, batch.y_mask)
        grads = torch.autograd.grad(loss, list(model.parameters()),
                                    allow_unused=True)
        return loss.detach(), count, correct, grads

    fused = run()
    monkeypatch.setattr(dense_ops, 'softmax_nll_supported',
                        lambda *a: False)
    plain = run()
    torch.testing.assert_close(fused[0], plain[0], atol=1e-5, rtol=1e-5)
    assert float(fused[1]) == float(plain[1]) == float(batch.y_mask.sum())
    assert float(fused[2]) == float(plain[2])
    for a, b in zip(fused[3], plain[3]):
        if a is None or b is None:
            assert a is None or b is None or float(a.abs().max()) == 0 or \
                float(b.abs().max()) == 0
            continue
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize('widths,M', [((128, 128, 128), 10307),
                                      ((128, ), 77), ((256, 128), 300)])
def test_cat_gemm_matches_cat_matmul(widths, M):
    """cat_gemm: [X_0 | X_1 | ...] @ W^T from strided inputs, plus the
    concatenation side output."""
    ops = _backend.ops()
    torch.manual_seed(3)
    wide = torch.randn(M, sum(widths) + 64, device=DEV).bfloat16()
    parts, off = [], 0
    for w in widths:
        parts.append(wide[:, off:off + w])      # strided column slices
        off += w
    K = sum(widths)
    W = (torch.randn(128, K, device=DEV) / K ** 0.5).bfloat16()
    ocat = torch.empty(M, K, dtype=torch.bfloat16, device=DEV)
    out = ops.cat_gemm(parts, W, ocat)
    cat = torch.cat(parts, dim=1)
    assert torch.equal(ocat, cat)
    ref = cat.float() @ W.float().t()
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    # transposed use (backward): [M, 128] @ [128, K] with W^T staged
    g = torch.randn(M, 128, device=DEV).bfloat16()
    gx = ops.cat_gemm([g], W.t().contiguous(), None)
    torch.testing.assert_close(gx.float(), g.float() @ W.float(), atol=2e-2,
                               rtol=2e-2)


def test_consensus_cat_matmul_matches_formed_concatenation(monkeypatch):
    """Static-batch consensus loop: the unformed psi_2 concatenation read by
    cat_gemm == torch.cat + GEMM (forward S_L and every gradient)."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets.static_batch import \
        StaticPairBatcher
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    groups = make_keypoint_datasets(graphs=16, feature_dim=32, seed=5)
    store = GraphStore(groups, torch.device(DEV))
    batcher = StaticPairBatcher(store, 48, seed=3)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(32, 64, 2, 2, cat=False),
                 SplineCNN(128, 128, 2, 2, cat=True), num_steps=4).to(DEV)
    model.eval()
    assert batcher.load()
    batch = batcher.materialize()

    def run():
        torch.manual_seed(1)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss, count, correct = model.objective(
                batch.x_s, batch.edge_index_s, batch.edge_attr_s,
                batch.x_s_batch, batch.x_t, batch.edge_index_t,
                batch.edge_attr_t, batch.x_t_batch, batch.y, batch.y_mask)
        return loss.detach(), torch.autograd.grad(
            loss, list(model.parameters()), allow_unused=True)

    l1, g1 = run()
    monkeypatch.setattr(dense_ops, 'cat_matmul_supported', lambda *a: False)
    l0, g0 = run()
    torch.testing.assert_close(l1, l0, atol=1e-3, rtol=1e-3)
    for a, b in zip(g1, g0):
        if a is None or b is None:
            assert a is None and b is None
            continue
        torch.testing.assert_close(a, b, atol=2e-2, rtol=2e-2)


def test_fused_step_boundary_matches_separate_kernels(monkeypatch):
    """Consensus update + next softmax transport in one kernel (forward and
    backward) == the separate consensus / transport kernels."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets.static_batch import \
        StaticPairBatcher
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    groups = make_keypoint_datasets(graphs=16, feature_dim=32, seed=6)
    store = GraphStore(groups, torch.device(DEV))
    batcher = StaticPairBatcher(store, 48, seed=4)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(32, 64, 2, 2, cat=False),
                 SplineCNN(128, 128, 2, 2, cat=True), num_steps=5).to(DEV)
    model.eval()
    assert batcher.load()
    batch = batcher.materialize()

    def run():
        torch.manual_seed(1)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss, count, correct = model.objective(
                batch.x_s, batch.edge_index_s, batch.edge_attr_s,
                batch.x_s_batch, batch.x_t, batch.edge_index_t,
                batch.edge_attr_t, batch.x_t_batch, batch.y, batch.y_mask)
        return loss.detach(), correct, torch.autograd.grad(
            loss, list(model.parameters()), allow_unused=True)

    calls = []
    real = _backend.ops().dense_consensus_transport

    class _Spy(object):
        def __getattr__(self, name):
            if name == 'dense_consensus_transport':
                def f(*a):
                    calls.append(1)
                    return real(*a)
                return f
            return getattr(torch.ops.dgmc_amd, name)
    orig = _backend.ops
    monkeypatch.setattr(_backend, 'ops', lambda: _Spy())
    l1, c1, g1 = run()
    monkeypatch.setattr(_backend, 'ops', orig)
    assert len(calls) == 4          # 5 steps: 4 fused boundaries
    monkeypatch.setattr(dense_ops, 'FUSE_STEPS', False)
    l0, c0, g0 = run()
    torch.testing.assert_close(l1, l0, atol=1e-4, rtol=1e-4)
    assert float(c1) == float(c0)
    for a, b in zip(g1, g0):
        if a is None or b is None:
            assert a is None and b is None
            continue
        torch.testing.assert_close(a, b, atol=1e-2, rtol=1e-2)


def _step_problem(R, Ns, Nt, B, bf=torch.bfloat16):
    torch.manual_seed(R + Ns)
    c_s = torch.randint(1, Ns + 1, (B, ))
    c_t = torch.randint(1, Nt + 1, (B, ))
    c_s[0], c_t[0] = Ns, Nt
    pad_s, pad_t = 5, 7
    ptr_s = torch.zeros(B + 1, dtype=torch.int32)
    ptr_t = torch.zeros(B + 1, dtype=torch.int32)
    ptr_s[1:], ptr_t[1:] = c_s.cumsum(0), c_t.cumsum(0)
    rows_s, rows_t = int(ptr_s[-1]) + pad_s, int(ptr_t[-1]) + pad_t
    d = dict(
        R=R, c_s=c_s, c_t=c_t, ptr_s=ptr_s, ptr_t=ptr_t, rows_s=rows_s,
        rows_t=rows_t, ps=ptr_s.to(DEV), pt=ptr_t.to(DEV),
        P=torch.randn(rows_s, R, device=DEV).to(bf),
        Q=torch.randn(rows_t, R, device=DEV).to(bf),
        r_s=torch.randn(rows_s, R, device=DEV).to(bf),
        b1=torch.randn(R, device=DEV) * 0.5,
        w2=torch.randn(R, device=DEV) / R ** 0.5,
        b2=torch.randn(1, device=DEV),
        S_hat=torch.randn(B, Ns, Nt, device=DEV),
        g_t=torch.randn(rows_t, R, device=DEV).to(bf),
        add=torch.randn(B, Ns, Nt, device=DEV))
    ii, jj = torch.arange(Ns), torch.arange(Nt)
    d['mask'] = ((ii[None, :, None] < c_s[:, None, None]) &
                 (jj[None, None, :] < c_t[:, None, None])).to(DEV)
    d['idx_s'] = (ptr_s[:-1, None] + ii[None]).clamp(max=rows_s - 1).to(DEV)
    d['idx_t'] = (ptr_t[:-1, None] + jj[None]).clamp(max=rows_t - 1).to(DEV)
    d['vs'] = (ii[None] < c_s[:, None]).to(DEV)
    d['vt'] = (jj[None] < c_t[:, None]).to(DEV)
    return d


def _step_ref(d, cons, trans):
    """fp32 autograd reference: S_new (cons), S_prob / r_t (trans), and the
    gradients of <r_t, g_t> + <S_new, addend> (or <S_new, addend> alone)."""
    Pf = d['P'].float().requires_grad_()
    Qf = d['Q'].float().requires_grad_()
    b1f, w2f, b2f = (d[k].clone().requires_grad_() for k in ('b1', 'w2',
                                                           'b2'))
    Sf = d['S_hat'].clone().requires_grad_()
    mask, vs, vt = d['mask'], d['vs'], d['vt']
    Sn = Sf
    if cons:
        h = torch.relu(Pf[d['idx_s']][:, :, None] + b1f -
                       Qf[d['idx_t']][:, None, :])
        Sn = Sf + mask * (h @ w2f + b2f)
    out = {'S_new': Sn}
    loss = (Sn * d['add']).sum()
    if trans:
        Sm = Sn.masked_fill(~mask, float('-inf')).masked_fill(
            ~vs[..., None], 0.0)
        Sp = torch.softmax(Sm, -1) * mask
        rsd = d['r_s'].float()[d['idx_s']] * vs[..., None]
        rt = Sp.transpose(1, 2) @ rsd
        loss = loss + (rt * (d['g_t'].float()[d['idx_t']] *
                             vt[..., None])).sum()
        rt_packed = torch.zeros(d['rows_t'], d['R'], device=DEV)
        rt_packed[d['idx_t'][vt]] = rt.detach()[vt]
        out.update(S_prob=Sp, r_t=rt_packed)
    grads = torch.autograd.grad(loss, (Sf, Pf, Qf, b1f, w2f, b2f),
                                allow_unused=True)
    out.update(zip(('gS', 'gP', 'gQ', 'gb1', 'gw2', 'gb2'), grads))
    return out


def _check_cons_grads(d, ref, dP, dQ, dw2, db2):
    n_s, n_t = int(d['ptr_s'][-1]), int(d['ptr_t'][-1])
    torch.testing.assert_close(dP.float(), ref['gP'], atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(dQ.float(), ref['gQ'], atol=3e-2, rtol=2e-2)
    assert (dP[n_s:] == 0).all() and (dQ[n_t:] == 0).all()
    torch.testing.assert_close(dw2.sum(0), ref['gw2'], atol=2e-3, rtol=1e-3)
    torch.testing.assert_close(db2.sum(), ref['gb2'][0], atol=2e-3,
                               rtol=1e-3)


@pytest.mark.parametrize('R', [32, 64, 128, 48])
@pytest.mark.parametrize('Ns,Nt,B', [(19, 23, 37), (9, 9, 300)])
def test_step_boundary_kernels_fp32_storage(R, Ns, Nt, B):
    """Reference precision: the same step kernels on fp32 node tensors
    (P, Q, r_s, g_t, dP, dQ, joint all fp32) at fp32 tolerance."""
    ops = _backend.ops()
    d = _step_problem(R, Ns, Nt, B, torch.float32)
    S_new, S_prob, joint = ops.dense_consensus_transport(
        d['S_hat'], d['P'], d['Q'], d['b1'], d['w2'], d['b2'], d['r_s'],
        d['ps'], d['pt'], d['rows_t'])
    assert joint.dtype == torch.float32
    G, dP, dQ, dw2, db2 = ops.dense_transport_consensus_bwd(
        S_prob, d['r_s'], d['g_t'], d['add'], d['P'], d['Q'], d['b1'],
        d['w2'], d['ps'], d['pt'], None)
    ref = _step_ref(d, True, True)
    rows_s, n_s, n_t = d['rows_s'], int(d['ptr_s'][-1]), int(d['ptr_t'][-1])
    tol = dict(atol=2e-5, rtol=2e-5)
    torch.testing.assert_close(S_new, ref['S_new'].detach(), **tol)
    torch.testing.assert_close(S_prob, ref['S_prob'].detach(), **tol)
    assert torch.equal(joint[:rows_s], d['r_s'])
    torch.testing.assert_close(joint[rows_s:], ref['r_t'], **tol)
    assert (joint[rows_s + n_t:] == 0).all()
    torch.testing.assert_close(G, ref['gS'], **tol)
    torch.testing.assert_close(dP, ref['gP'], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(dQ, ref['gQ'], atol=1e-4, rtol=1e-4)
    assert (dP[n_s:] == 0).all() and (dQ[n_t:] == 0).all()
    torch.testing.assert_close(dw2.sum(0), ref['gw2'], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(db2.sum(), ref['gb2'][0], atol=1e-4,
                               rtol=1e-4)


@pytest.mark.parametrize('R', [32, 64, 128, 48])
@pytest.mark.parametrize('Ns,Nt,B', [(19, 23, 37), (64, 64, 3), (9, 9, 300)])
def test_step_boundary_kernels_vs_fp32(R, Ns, Nt, B):
    """dense_consensus_transport / dense_transport_consensus_bwd (the
    compile-time-R kernels for R in 32/64/128, the generic ones otherwise)
    against autograd on the fp32 dense expression, incl. the static-batch
    padding rows of both graphs."""
    ops = _backend.ops()
    d = _step_problem(R, Ns, Nt, B)
    S_new, S_prob, joint = ops.dense_consensus_transport(
        d['S_hat'], d['P'], d['Q'], d['b1'], d['w2'], d['b2'], d['r_s'],
        d['ps'], d['pt'], d['rows_t'])
    G, dP, dQ, dw2, db2 = ops.dense_transport_consensus_bwd(
        S_prob, d['r_s'], d['g_t'], d['add'], d['P'], d['Q'], d['b1'],
        d['w2'], d['ps'], d['pt'], None)
    ref = _step_ref(d, True, True)
    rows_s = d['rows_s']
    torch.testing.assert_close(S_new, ref['S_new'].detach(), atol=1e-4,
                               rtol=1e-4)
    torch.testing.assert_close(S_prob, ref['S_prob'].detach(), atol=1e-5,
                               rtol=1e-4)
    assert torch.equal(joint[:rows_s], d['r_s'])
    torch.testing.assert_close(joint[rows_s:].float(), ref['r_t'], atol=2e-2,
                               rtol=1e-2)
    assert (joint[rows_s + int(d['ptr_t'][-1]):] == 0).all()
    torch.testing.assert_close(G, ref['gS'], atol=1e-3, rtol=1e-3)
    _check_cons_grads(d, ref, dP, dQ, dw2, db2)
    # Loop accumulator contract: [db1 | dw2 | db2] per pair, added over uses.
    part = torch.full((B, 2 * R + 1), float('nan'), device=DEV)
    for accumulate in (False, True):
        out = ops.dense_transport_consensus_bwd(
            S_prob, d['r_s'], d['g_t'], d['add'], d['P'], d['Q'], d['b1'],
            d['w2'], d['ps'], d['pt'], None, part, accumulate)
        assert out[3] is None and out[4] is None
        torch.testing.assert_close(out[1], dP, atol=0, rtol=0)
    tot = part.sum(0)
    # (db1 from the fp32 dP rows: closer to the fp32 reference than the sum
    # of the bf16-rounded dP output)
    # (generic kernels: sum of the bf16 dP rows)
    tol = 5e-3 if R in (32, 64, 128) else 0.1
    torch.testing.assert_close(tot[:R], 2 * ref['gb1'], atol=tol, rtol=2e-2)
    torch.testing.assert_close(tot[R:2 * R], 2 * dw2.sum(0), atol=2e-3,
                               rtol=1e-3)
    torch.testing.assert_close(tot[2 * R], 2 * db2.sum(), atol=2e-3,
                               rtol=1e-3)


@pytest.mark.parametrize('R', [32, 128, 48])
@pytest.mark.parametrize('Ns,Nt,B', [(19, 23, 37), (64, 64, 3)])
def test_step_kernels_split_vs_fp32(R, Ns, Nt, B):
    """The consensus-only and transport-only step kernels (first / last
    consensus step) against the same fp32 reference."""
    ops = _backend.ops()
    d = _step_problem(R, Ns, Nt, B)
    # consensus only
    ref = _step_ref(d, True, False)
    out = ops.dense_consensus(d['S_hat'], d['P'], d['Q'], d['b1'], d['w2'],
                              d['b2'], d['ps'], d['pt'])
    torch.testing.assert_close(out, ref['S_new'].detach(), atol=1e-4,
                               rtol=1e-4)
    dP, dQ, dw2, db2 = ops.dense_consensus_bwd(
        d['add'], d['P'], d['Q'], d['b1'], d['w2'], d['ps'], d['pt'], None)
    _check_cons_grads(d, ref, dP, dQ, dw2, db2)
    part = torch.full((B, 2 * R + 1), float('nan'), device=DEV)
    out = ops.dense_consensus_bwd(d['add'], d['P'], d['Q'], d['b1'],
                                  d['w2'], d['ps'], d['pt'], None, part, False)
    assert out[2] is None and out[3] is None
    tot = part.sum(0)
    tol = 5e-3 if R in (32, 64, 128) else 0.1
    torch.testing.assert_close(tot[:R], ref['gb1'], atol=tol, rtol=2e-2)
    torch.testing.assert_close(tot[R:2 * R], dw2.sum(0), atol=2e-3,
                               rtol=1e-3)
    # transport only (plain and joint output)
    ref = _step_ref(d, False, True)
    rows_s = d['rows_s']
    for joint in (False, True):
        S, r = ops.dense_softmax_transport(d['S_hat'], d['r_s'], d['ps'],
                                           d['pt'], d['rows_t'], joint)
        torch.testing.assert_close(S, ref['S_prob'].detach(), atol=1e-5,
                                   rtol=1e-4)
        if joint:
            assert torch.equal(r[:rows_s], d['r_s'])
            r = r[rows_s:]
        torch.testing.assert_close(r.float(), ref['r_t'], atol=2e-2,
                                   rtol=1e-2)
        assert (r[int(d['ptr_t'][-1]):] == 0).all()
    g = ops.dense_softmax_transport_bwd(S, d['r_s'], d['g_t'], d['ps'],
                                        d['pt'], d['add'])
    torch.testing.assert_close(g, ref['gS'], atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize('R', [32, 128, 48])
@pytest.mark.parametrize('Ns,Nt,B', [(19, 23, 37), (9, 9, 300)])
def test_step_joint_planes_equal_split3(R, Ns, Nt, B):
    """The joint [r_s; r_t]'s bf16x6 planes written by the transport kernels
    (psi_2's slot-conv operand) == split3 of the joint, every row (incl. the
    static-batch padding rows; R = 48: the generic kernels' fill path)."""
    ops = _backend.ops()
    d = _step_problem(R, Ns, Nt, B, torch.float32)
    rows = d['rows_s'] + d['rows_t']

    def fresh():
        return torch.full((3, rows, R), float('nan'), dtype=torch.bfloat16,
                          device=DEV)
    pl = fresh()
    _, _, joint = ops.dense_consensus_transport(
        d['S_hat'], d['P'], d['Q'], d['b1'], d['w2'], d['b2'], d['r_s'],
        d['ps'], d['pt'], d['rows_t'], pl)
    _, _, ref = ops.dense_consensus_transport(
        d['S_hat'], d['P'], d['Q'], d['b1'], d['w2'], d['b2'], d['r_s'],
        d['ps'], d['pt'], d['rows_t'])
    assert torch.equal(joint, ref)
    assert torch.equal(pl, ops.split3(joint))
    pl = fresh()
    _, joint = ops.dense_softmax_transport(d['S_hat'], d['r_s'], d['ps'],
                                           d['pt'], d['rows_t'], True, pl)
    assert torch.equal(pl, ops.split3(joint))


def test_joint_planes_model_bit_identical(monkeypatch):
    """fp32 DGMC (dense, SplineCNN psi_2): psi_2's first conv reading the
    transport kernels' planes gives bit-identical loss and gradients to the
    split pass."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets.static_batch import \
        StaticPairBatcher
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.ops import slot_gemm
    groups = make_keypoint_datasets(graphs=16, feature_dim=32, seed=6)
    store = GraphStore(groups, torch.device(DEV))
    batcher = StaticPairBatcher(store, 48, seed=4)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(32, 128, 2, 2, cat=False),
                 SplineCNN(128, 128, 2, 2, cat=False), num_steps=4).to(DEV)
    assert batcher.load()
    batch = batcher.materialize()
    assert model.psi_2.takes_x6_planes(batch.x_s.new_zeros(1, 128))
    split_calls = []
    real_split = _backend.ops().split3

    class _Spy(object):
        def __getattr__(self, name):
            if name == 'split3':
                def f(*a):
                    split_calls.append(tuple(a[0].shape))
                    return real_split(*a)
                return f
            return getattr(torch.ops.dgmc_amd, name)

    def run():
        torch.manual_seed(1)
        loss, count, correct = model.objective(
            batch.x_s, batch.edge_index_s, batch.edge_attr_s,
            batch.x_s_batch, batch.x_t, batch.edge_index_t,
            batch.edge_attr_t, batch.x_t_batch, batch.y, batch.y_mask)
        return loss.detach(), torch.autograd.grad(
            loss, list(model.parameters()), allow_unused=True)
    orig = _backend.ops
    monkeypatch.setattr(_backend, 'ops', lambda: _Spy())
    l1, g1 = run()
    n1 = len(split_calls)
    monkeypatch.setattr(SplineCNN, 'takes_x6_planes', lambda self, x: False)
    l0, g0 = run()
    n0 = len(split_calls) - n1
    monkeypatch.setattr(_backend, 'ops', orig)
    if slot_gemm.F32X:
        assert n0 - n1 == 4, (n0, n1)   # one split per psi_2 call saved
    assert torch.equal(l1, l0)
    for a, b in zip(g1, g0):
        if a is None or b is None:
            assert a is None and b is None
            continue
        assert torch.equal(a, b)


@pytest.mark.parametrize('U,N,K', [(10, 1000, 384), (3, 77, 128),
                                   (17, 300, 256)])
def test_dense_wgrad_matches_fp32(U, N, K):
    """Loop-use TN weight gradient on MFMA (dense_wgrad) == fp32 sum of
    X_u^T G_u, incl. a use count above the 16-entry pointer table."""
    torch.manual_seed(U + N)
    X = torch.randn(U, N, K, device=DEV).bfloat16()
    gs = [torch.randn(N, 128, device=DEV).bfloat16() for _ in range(U)]
    assert dense_ops.dense_wgrad_supported(X, gs)
    got = dense_ops.dense_wgrad(list(X.unbind(0)), gs)
    ref_ = sum(x.float().t() @ g.float() for x, g in zip(X.unbind(0), gs))
    torch.testing.assert_close(got, ref_, atol=2e-3 * N ** 0.5 * U ** 0.5,
                               rtol=1e-3)


@pytest.mark.parametrize('K,M,N', [(11008, 256, 256), (3000, 128, 384)])
def test_matmul_tn_fp32_dense_path(K, M, N):
    """matmul_tn_fp32 on small bf16 outputs (dense_wgrad path), plain and
    accumulating into an fp32 output."""
    from deep_graph_matching_consensus_amd.ops.gemm import (_dense_tn_ok,
                                                            matmul_tn_fp32)
    a = torch.randn(K, M, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16()
    assert _dense_tn_ok(a, b)
    ref_ = a.float().t() @ b.float()
    tol = 2e-3 * K ** 0.5
    torch.testing.assert_close(matmul_tn_fp32(a, b), ref_, atol=tol,
                               rtol=1e-3)
    out = torch.ones(M, N, device=DEV)
    matmul_tn_fp32(a, b, out=out, accumulate=True)
    torch.testing.assert_close(out, ref_ + 1, atol=tol, rtol=1e-3)


def test_fold_weights_kernel():
    """fold_weights: fp32 W1 @ W_f and its bf16 images W / W^T in one
    kernel."""
    w1 = torch.randn(128, 128, device=DEV)
    wf = torch.randn(128, 384, device=DEV)
    w, wn, wnt = _backend.ops().fold_weights(w1, wf)
    ref_ = w1.double() @ wf.double()
    torch.testing.assert_close(w.double(), ref_, atol=1e-3, rtol=1e-4)
    assert torch.equal(wn, w.bfloat16())
    assert torch.equal(wnt, w.t().contiguous().bfloat16())


# Every alternative kernel path still behind a switch (each measured slower
# or kept as an exact-f32 fallback, docs/performance.md) is exercised here
# against the reference expression: (module, attribute, value).
_SWITCHES = [None, ('slot_gemm', 'ENABLED', False),
             ('slot_gemm', 'X6', False), ('slot_gemm', 'F32DY', False),
             ('slot_gemm', 'F32X', False), ('slot_gemm', 'ROWMAP_ELL', False),
             ('dense', 'NT_X6', False),
             ('dense', 'FUSE_STEPS', False)]


@pytest.mark.parametrize('switch', _SWITCHES,
                         ids=lambda s: 'default' if s is None else
                         '{}.{}={}'.format(*s))
def test_dgmc_fp32_headline_widths_vs_reference_mode(switch, monkeypatch):
    """fp32 at the flagship's layer widths (psi_1 in/out multiples of 128,
    psi_2 128 -> 128 with cat=True): the step runs the fp32 slot GEMMs,
    the folded projection on the dense fp32 GEMM, the fused pair-step and
    objective kernels; outputs, loss and every parameter gradient match the
    reference-mode expression (``/root/reference/dgmc/models/dgmc.py:
    163-244``, fp32) to fp32 tolerance (loss 1e-5 relative, gradients 1e-4
    relative to their largest entry).  ``switch``: one alternative path
    (e.g. ``slot_gemm.ENABLED=False``: GEMM over all slots + SpMM;
    ``slot_gemm.X6=False``: the exact-f32 MFMA kernels)."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, DevicePairLoader, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.ops import dense as dense_mod
    from deep_graph_matching_consensus_amd.ops import slot_gemm as sg
    if switch is not None:
        mod = {'slot_gemm': sg, 'dense': dense_mod}[switch[0]]
        assert hasattr(mod, switch[1])
        monkeypatch.setattr(mod, switch[1], switch[2])
    groups = make_keypoint_datasets(graphs=8, feature_dim=256, seed=0)
    store = GraphStore(groups, DEV)
    batch = next(iter(DevicePairLoader(store, batch_size=32, seed=0)))
    torch.manual_seed(3)
    model = DGMC(SplineCNN(256, 128, 2, 2, cat=False),
                 SplineCNN(128, 128, 2, 2, cat=True), num_steps=4).to(DEV)
    args = (batch.x_s, batch.edge_index_s, batch.edge_attr_s,
            batch.x_s_batch, batch.x_t, batch.edge_index_t,
            batch.edge_attr_t, batch.x_t_batch)
    y = torch.stack([torch.arange(batch.y.numel(), device=DEV), batch.y])
    params = list(model.parameters())

    torch.manual_seed(5)
    S_0, S_L = model(*args)
    loss = model.loss(S_0, y) + model.loss(S_L, y)
    grads = torch.autograd.grad(loss, params, allow_unused=True)
    with reference_mode():
        torch.manual_seed(5)
        R_0, R_L = model(*args)
        loss2 = model.loss(R_0, y) + model.loss(R_L, y)
        grads2 = torch.autograd.grad(loss2, params, allow_unused=True)
    assert S_L.dtype == torch.float32
    assert torch.allclose(S_0, R_0, atol=1e-5)
    assert torch.allclose(S_L, R_L, atol=1e-5)
    assert abs(loss.item() - loss2.item()) <= 1e-5 * abs(loss2.item())
    # (floor 1e-5 x the largest gradient: psi_2's final bias and the MLP's
    # output bias cancel exactly (P_i - Q_j, row softmax) - their exact
    # gradients are 0 and both paths leave only rounding)
    G = max(float(b.abs().max()) for b in grads2 if b is not None)
    for p, a, b in zip(params, grads, grads2):
        if b is None:
            continue
        a = torch.zeros_like(b) if a is None else a
        err = float((a - b).abs().max())
        assert err <= 1e-4 * float(b.abs().max()) + 1e-5 * G, p.shape
