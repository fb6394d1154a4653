"""fp32 SplineConv on the used (node, slot) pairs (csrc/hip/slot_gemm.hip).

Oracle: the dense fp64 expression ``A @ (x @ [W_0 | .. | W_{S-1}])`` of
SplineConv (``/root/reference/dgmc/models/spline.py:49``, PyG SplineConv with
mean aggregation and root weight), forward and backward (dx, dW, droot,
dbias), compared at fp32 tolerance.
"""
import pytest
import torch

from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops import slot_gemm as sg
from deep_graph_matching_consensus_amd.ops.plans import spline_plan
from deep_graph_matching_consensus_amd.runtime import loopgrad

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(autouse=True)
def _require_hip():
    assert _backend.hip_available(), 'HIP extension must be built'
    torch.manual_seed(0)


def _graph(n, e, seed=0):
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(n, (2, e), generator=g)
    pseudo = torch.rand(e, 2, generator=g)
    return ei.to(DEV), pseudo.to(DEV)


def _params(cin, cout, K=25, seed=1):
    g = torch.Generator().manual_seed(seed)
    w = (torch.rand(K, cin, cout, generator=g) - 0.5) / 8
    r = (torch.rand(cin, cout, generator=g) - 0.5) / 8
    b = torch.rand(cout, generator=g) - 0.5
    return [t.to(DEV).requires_grad_() for t in (w, r, b)]


def _oracle(op, x, w, r, b, relu):
    """fp64 dense reference."""
    A = op.to_dense().double()
    W = torch.cat([w.double().permute(1, 0, 2).reshape(w.size(1), -1),
                   r.double()], 1)
    Y = (x.double() @ W).view(-1, w.size(2))
    out = A @ Y + b.double()
    return out.relu() if relu else out


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() /
                 b.double().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize('cin,cout,relu', [(128, 128, True),
                                           (256, 256, False),
                                           (1024, 256, True)])
def test_slot_gemm_spmm_matches_fp64(cin, cout, relu):
    n, e = 700, 2800
    ei, pseudo = _graph(n, e)
    op = spline_plan(ei, pseudo, n, (5, 5), (1, 1), 1, root=True)
    x = torch.randn(n, cin, device=DEV, requires_grad=True)
    w, r, b = _params(cin, cout)
    out = sg.slot_gemm_spmm(op, x, w, r, b, relu=relu)
    ref = _oracle(op, x, w, r, b, relu)
    assert _rel(out, ref) < 2e-6
    g = torch.randn_like(out)
    grads = torch.autograd.grad(out, (x, w, r, b), g)
    refs = torch.autograd.grad(ref, (x, w, r, b), g.double())
    for name, a, bb in zip('xwrb', grads, refs):
        assert a.dtype == torch.float32
        assert _rel(a, bb) < 1e-5, name


@pytest.mark.parametrize('n,e', [(500, 2000), (20000, 60000)])
def test_compact_plan_layout(n, e):
    ei, pseudo = _graph(n, e, seed=3)
    op = spline_plan(ei, pseudo, n, (5, 5), (1, 1), 1, root=True)
    S = 26
    plan = sg.compact_plan(op, S)
    used = torch.unique(op.col.long())
    seg = plan.seg.cpu()
    assert int(plan.counts.sum()) == used.numel()
    assert (seg % sg.BM == 0).all() and int(seg[-1]) <= plan.P_cap
    pm = plan.posmap.long()
    assert (pm[used] >= 0).all()
    assert int((pm >= 0).sum()) == used.numel()
    # src / cinv invert posmap on the used columns.
    assert torch.equal(plan.src.long()[pm[used]], used // S)
    assert torch.equal(plan.cinv.long()[pm[used]], used)
    # Re-indexed entries point at their column's compact row.
    nnz = int(op.rowptr[-1])
    assert torch.equal(plan.col_c[:nnz].long(), pm[op.col[:nnz].long()])
    # Every compact row lies in its slot's segment.
    k = used % S
    p = pm[used].cpu()
    assert ((p >= seg[k.cpu()]) & (p < seg[k.cpu() + 1])).all()
    # ... in ascending source order (20000 sources: several scan rounds)
    src, cnt = plan.src.long().cpu(), plan.counts.long().cpu()
    for s_ in range(S):
        rows = src[int(seg[s_]):int(seg[s_]) + int(cnt[s_])]
        assert bool((rows[1:] > rows[:-1]).all())
    # Rows no used column maps to (segment padding, the tail) hold -1.
    free = torch.ones(plan.P_cap, dtype=torch.bool)
    free[p] = False
    assert (src[free] == -1).all() and (plan.cinv.cpu()[free] == -1).all()
    # dX row-tile lists: slot k's tiles from the tile of its first source
    # >= row0 to its segment end, in slot order (count at [tcap]).
    for row0 in (0, 1, n // 3, n - 1, n):
        for unit in (128, 256):
            got = sg.dx_tiles(plan, row0, unit).cpu()
            ref = []
            for s_ in range(S):
                a, b = int(seg[s_]), int(seg[s_ + 1])
                hit = (src[a:a + int(cnt[s_])] >= row0).nonzero()
                first = (a + int(hit[0])) // unit if hit.numel() else b // unit
                ref += list(range(min(first, b // unit), b // unit))
            tcap = plan.P_cap // unit
            assert int(got[tcap]) == min(len(ref), tcap)
            assert got[:min(len(ref), tcap)].tolist() == ref[:tcap]


def test_loop_weight_grad_equals_per_use():
    """Loop-shared weight gradient (one launch over the kept (X, dY_c) of
    every use) equals the per-use autograd sum."""
    n, e, C = 600, 2400, 128
    ei, pseudo = _graph(n, e, seed=5)
    op = spline_plan(ei, pseudo, n, (5, 5), (1, 1), 1, root=True)
    w, r, b = _params(C, C, seed=7)
    xs = [torch.randn(n, C, device=DEV) for _ in range(3)]

    def run(loop):
        with loopgrad.loop_scope(loop):
            h = 0
            for x in xs:
                h = h + sg.slot_gemm_spmm(op, x, w, r, b, relu=True,
                                          loop_key=('t', ) if loop else None)
            return torch.autograd.grad(h.square().sum(), (w, r, b))

    for a, bb in zip(run(True), run(False)):
        assert _rel(a, bb) < 1e-6


@pytest.mark.parametrize('n,cat', [(600, True), (2000, False)])
def test_relu_bias_handoff_bit_identical(n, cat):
    """Layer 0's ReLU mask and bias partials applied by layer 1's dX
    gather-sum (RB_FUSE) give bit-identical gradients to the unfused
    relu_bias_bwd, inside the consensus loop (3 uses)."""
    if not sg.X6:
        pytest.skip('bf16x6 path only')
    e, C = 4 * n, 128
    ei, pseudo = _graph(n, e, seed=13)
    op = spline_plan(ei, pseudo, n, (5, 5), (1, 1), 1, root=True)
    p0 = [t.requires_grad_() for t in _params(C, C, seed=3)]
    p1 = [t.requires_grad_() for t in _params(C, C, seed=6)]
    xs = [torch.randn(n, C, device=DEV) for _ in range(3)]
    gs = [torch.randn(n, 3 * C if cat else C, device=DEV) for _ in range(3)]

    def run(fuse):
        sg.RB_FUSE = fuse
        try:
            with loopgrad.loop_scope(True):
                loss = 0
                for x, g in zip(xs, gs):
                    x = x.clone().requires_grad_()
                    h0 = sg.slot_gemm_spmm(op, x, *p0, relu=True,
                                           loop_key=('l0', ), passthrough=cat)
                    if cat:
                        h0, x = h0
                    h1 = sg.slot_gemm_spmm(op, h0, *p1, relu=True,
                                           loop_key=('l1', ), passthrough=cat)
                    if cat:
                        h1, h0 = h1
                        h1 = torch.cat([x, h0, h1], 1)
                    loss = loss + (h1 * g).sum()
                return torch.autograd.grad(loss, p0 + p1)
        finally:
            sg.RB_FUSE = True

    for a, b in zip(run(True), run(False)):
        assert torch.equal(a, b)


def test_passthrough_gradient_added():
    n, e, C = 400, 1600, 128
    ei, pseudo = _graph(n, e, seed=9)
    op = spline_plan(ei, pseudo, n, (5, 5), (1, 1), 1, root=True)
    w, r, b = _params(C, C, seed=2)
    x = torch.randn(n, C, device=DEV, requires_grad=True)
    out, xp = sg.slot_gemm_spmm(op, x, w, r, b, relu=True, passthrough=True)
    loss = out.square().sum() + (xp * 3).sum()
    gx, = torch.autograd.grad(loss, (x, ))
    out2 = sg.slot_gemm_spmm(op, x, w, r, b, relu=True)
    gx2, = torch.autograd.grad(out2.square().sum() + (x * 3).sum(), (x, ))
    assert _rel(gx, gx2) < 1e-6


@pytest.mark.parametrize('row0', [1, 237, 599])
def test_dx_row0_matches_full_rows(row0):
    """``dx_row0`` (psi_2's r_s half needs no input gradient): the listed
    row tiles give the full input gradient on rows >= row0, zeros below;
    the weight gradients are unchanged."""
    n, e, C = 600, 2400, 128
    ei, pseudo = _graph(n, e, seed=11)
    op = spline_plan(ei, pseudo, n, (5, 5), (1, 1), 1, root=True)
    w, r, b = _params(C, C, seed=4)
    x = torch.randn(n, C, device=DEV, requires_grad=True)
    g = torch.randn(n, C, device=DEV)
    full = torch.autograd.grad(
        sg.slot_gemm_spmm(op, x, w, r, b, relu=True), (x, w, r, b), g)
    part = torch.autograd.grad(
        sg.slot_gemm_spmm(op, x, w, r, b, relu=True, dx_row0=row0),
        (x, w, r, b), g)
    assert torch.equal(part[0][row0:], full[0][row0:])
    assert not part[0][:row0].any()
    for a, bb in zip(part[1:], full[1:]):
        assert torch.equal(a, bb)


@pytest.mark.parametrize('M,nparts', [(1088, 3), (512, 1), (96, 2)])
def test_cat_matmul_f32_matches_fp64(M, nparts):
    """fp32 ``cat(parts) @ W`` on the dense LDS-DMA GEMM (parts read in
    place, rows past M clamped) and its backward (g W^T, dense TN weight
    gradient) against fp64."""
    from deep_graph_matching_consensus_amd.ops import dense as dops
    parts = [torch.randn(M, 128, device=DEV, requires_grad=True)
             for _ in range(nparts)]
    w_t = (torch.randn(128 * nparts, 128, device=DEV) / 20).requires_grad_()
    assert dops.cat_matmul_f32_supported(parts, w_t)
    out = dops.cat_matmul_f32(parts, w_t, ('t', ), 0)
    ref = torch.cat(parts, -1).double() @ w_t.double()
    assert _rel(out, ref) < 2e-6
    g = torch.randn_like(out)
    grads = torch.autograd.grad(out, parts + [w_t], g)
    refs = torch.autograd.grad(ref, parts + [w_t], g.double())
    for a, bb in zip(grads, refs):
        assert a.dtype == torch.float32
        assert _rel(a, bb) < 1e-5


def test_cat_matmul_f32_loop_weight_grad():
    """Inside a consensus loop the weight gradient of all uses is one dense
    TN launch; it equals the per-use autograd sum."""
    from deep_graph_matching_consensus_amd.ops import dense as dops
    M, uses = 640, 4
    w_t = (torch.randn(384, 128, device=DEV) / 20).requires_grad_()
    xs = [[torch.randn(M, 128, device=DEV) for _ in range(3)]
          for _ in range(uses)]

    def run(loop):
        with loopgrad.loop_scope(loop):
            h = 0
            for ps in xs:
                h = h + dops.cat_matmul_f32(ps, w_t, ('L', ),
                                            uses if loop else 0)
            return torch.autograd.grad(h.square().sum(), (w_t, ))[0]

    assert _rel(run(True), run(False)) < 1e-6


@pytest.mark.parametrize('K,M,N', [(1056, 256, 256), (2048, 128, 384),
                                   (96, 512, 128)])
def test_matmul_tn_fp32_dense_kernel(K, M, N):
    """fp32 ``a^T b`` (weight gradients of Linear layers) on the dense TN
    MFMA kernel, against fp64, plain and accumulated into ``out``."""
    from deep_graph_matching_consensus_amd.ops.gemm import matmul_tn_fp32
    a = torch.randn(K, M, device=DEV)
    b = torch.randn(K, N, device=DEV)
    ref = a.double().t() @ b.double()
    assert _rel(matmul_tn_fp32(a, b), ref) < 2e-6
    out = torch.ones(M, N, device=DEV)
    matmul_tn_fp32(a, b, out=out, accumulate=True)
    assert _rel(out, ref + 1) < 2e-6
