"""Fused RelCNN consensus encoder (csrc/hip/relconv.hip, ops/relconv.py):
psi_2 = RelCNN(32, 32, 3, cat=True, lin=True) of the DBP15K config
(``/root/reference/examples/dbp15k.py:29-33``) plus the folded consensus
projection, forward and backward, against fp64 oracles of the reference
expression (``/root/reference/dgmc/models/rel.py:25-31``: Linear maps,
scatter-mean over both flows) on the full-size DBP15K-shaped joint graph
(19,388 + 19,572 entities, hub rows included)."""
import pytest
import torch

from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair
from deep_graph_matching_consensus_amd.models import RelCNN
from deep_graph_matching_consensus_amd.ops import relconv as rc

DEV = 'cuda'


def _joint(scale=1.0, device='cpu'):
    d = make_kg_pair('zh_en', scale=scale, seed=0)
    n_s, n_t = d.x1.size(0), d.x2.size(0)
    ei = torch.cat([d.edge_index1, d.edge_index2 + n_s], 1).to(device)
    return ei, n_s, n_t


def test_rel_plan_lists_and_hubs_cpu():
    """Joint forward / backward lists, backward weights and hub flags."""
    ei, n_s, n_t = _joint(scale=0.05)
    N = n_s + n_t
    p = rc.RelPlan(ei, N, hub_threshold=8)
    src, dst = ei
    deg_in = torch.bincount(dst, minlength=N)
    deg_out = torch.bincount(src, minlength=N)
    assert torch.equal((p.ptr[1:] - p.ptr[:-1]).long(), deg_in + deg_out)
    assert torch.equal((p.split_f - p.ptr[:-1]).long(), deg_in)
    assert torch.equal((p.split_b - p.ptr[:-1]).long(), deg_out)
    i = int(torch.argmax(deg_in + deg_out))
    a, s_, b = int(p.ptr[i]), int(p.split_f[i]), int(p.ptr[i + 1])
    assert p.col_f[a:s_].tolist() == src[dst == i].tolist()
    assert p.col_f[s_:b].tolist() == dst[src == i].tolist()
    s2 = int(p.split_b[i])
    assert p.col_b[a:s2].tolist() == dst[src == i].tolist()
    assert p.col_b[s2:b].tolist() == src[dst == i].tolist()
    inv_in = 1.0 / deg_in.clamp(min=1).float()
    inv_out = 1.0 / deg_out.clamp(min=1).float()
    assert torch.equal(p.w_b[a:s2], inv_in[dst[src == i]])
    assert torch.equal(p.w_b[s2:b], inv_out[src[dst == i]])
    hub = (deg_in + deg_out) > 8
    assert torch.equal(p.hub.bool(), hub) and int(hub.sum()) > 0
    # packed kernel lists: column | (2 (row % 64) + list) << 24
    for pk, col, split in ((p.pk_f, p.col_f, p.split_f),
                           (p.pk_b, p.col_b, p.split_b)):
        assert torch.equal(pk & ((1 << 24) - 1), col)
        row = torch.repeat_interleave(torch.arange(N), deg_in + deg_out)
        lst = (torch.arange(row.numel()) >= split.long()[row]).long()
        assert torch.equal((pk[:-1] >> 24).long(), 2 * (row % 64) + lst)


def _model(seed=0):
    torch.manual_seed(seed)
    psi_2 = RelCNN(32, 32, 3, batch_norm=False, cat=True, lin=True,
                   dropout=0.0)
    mlp0 = torch.nn.Linear(32, 32)
    return psi_2.to(DEV), mlp0.to(DEV)


def _ref(psi_2, mlp0, ei, r_s, r_t, dtype):
    p2 = RelCNN(32, 32, 3, cat=True, lin=True).to(DEV).to(dtype)
    p2.load_state_dict({k: v.to(dtype) for k, v in
                        psi_2.state_dict().items()})
    w = mlp0.weight.detach().to(dtype).requires_grad_()
    rt = r_t.detach().to(dtype).requires_grad_()
    pq = rc.reference_psi2_fold(p2, w, ei, r_s.to(dtype), rt)
    return pq, p2, w, rt


def _grads(pq, dpq, leaves):
    return torch.autograd.grad(pq, leaves, dpq.to(pq.dtype))


@pytest.mark.gpu
def test_fused_psi2_forward_backward_vs_fp64():
    """PQ, d r_t and every weight gradient of one fused step: error against
    fp64 at most 4x that of the same expression in fp32 on the library
    kernels (+ 1e-6 of the value scale)."""
    ei, n_s, n_t = _joint(device=DEV)
    N = n_s + n_t
    plan = rc.rel_plan(ei, N)
    assert int(plan.hub.sum()) > 100    # wave-gathered hub rows exercised
    psi_2, mlp0 = _model()
    g = torch.Generator(device=DEV).manual_seed(3)
    r_s = torch.randn(n_s, 32, device=DEV, generator=g)
    r_t = (torch.randn(n_t, 32, device=DEV, generator=g) * 0.3) \
        .requires_grad_()
    pq = rc.psi2_fold(psi_2, mlp0.weight, plan, r_s, r_t, ('t', 0))
    dpq = torch.randn(N, 32, device=DEV, generator=g)
    params = [p for c in psi_2.convs for p in
              (c.lin1.weight, c.lin2.weight, c.root.weight, c.root.bias)]
    leaves = [r_t, mlp0.weight, psi_2.final.weight] + params
    gf = torch.autograd.grad(pq, leaves, dpq)

    def oracle(dtype):
        out, p2, w, rt = _ref(psi_2, mlp0, ei, r_s, r_t, dtype)
        pp = [p for c in p2.convs for p in
              (c.lin1.weight, c.lin2.weight, c.root.weight, c.root.bias)]
        return out, _grads(out, dpq, [rt, w, p2.final.weight] + pp)

    ref64, g64 = oracle(torch.float64)
    ref32, g32 = oracle(torch.float32)

    def check(a, b32, b64, what):
        e = float((a.detach().double() - b64).abs().max())
        e32 = float((b32.detach().double() - b64).abs().max())
        scale = float(b64.abs().max())
        assert e <= 4 * e32 + 1e-6 * scale, (what, e, e32, scale)

    check(pq, ref32, ref64, 'PQ')
    names = ['r_t', 'mlp0.weight', 'final.weight'] + [
        '{}.{}'.format(l, n) for l in range(3)
        for n in ('lin1', 'lin2', 'root.w', 'root.b')]
    for n, a, b32, b64 in zip(names, gf, g32, g64):
        check(a, b32, b64, n)


@pytest.mark.gpu
def test_fused_psi2_loop_uses_accumulate():
    """Three uses in a loop scope (the consensus loop): every use's r_t
    gradient equals the single-use one, and the weight gradients (folded
    once by the last use) equal the sum over the uses."""
    from deep_graph_matching_consensus_amd.runtime import loopgrad
    ei, n_s, n_t = _joint(scale=0.25, device=DEV)
    N = n_s + n_t
    plan = rc.rel_plan(ei, N)
    psi_2, mlp0 = _model(1)
    g = torch.Generator(device=DEV).manual_seed(4)
    r_s = [torch.randn(n_s, 32, device=DEV, generator=g) for _ in range(3)]
    r_t = [torch.randn(n_t, 32, device=DEV, generator=g).requires_grad_()
           for _ in range(3)]
    dpq = [torch.randn(N, 32, device=DEV, generator=g) for _ in range(3)]
    params = [mlp0.weight, psi_2.final.weight] + [
        p for c in psi_2.convs for p in
        (c.lin1.weight, c.lin2.weight, c.root.weight, c.root.bias)]
    single = []
    for u in range(3):
        pq = rc.psi2_fold(psi_2, mlp0.weight, plan, r_s[u], r_t[u], ('a', u))
        single.append(torch.autograd.grad(pq, [r_t[u]] + params, dpq[u]))
    with loopgrad.loop_scope():
        pqs = [rc.psi2_fold(psi_2, mlp0.weight, plan, r_s[u], r_t[u],
                            ('b', 0)) for u in range(3)]
        loss = sum((p * d).sum() for p, d in zip(pqs, dpq))
        looped = torch.autograd.grad(loss, r_t + params)
    for u in range(3):
        assert torch.allclose(looped[u], single[u][0], rtol=1e-5,
                              atol=1e-6)
    for i, p in enumerate(params):
        tot = sum(single[u][1 + i] for u in range(3))
        assert torch.allclose(looped[3 + i], tot, rtol=1e-4,
                              atol=1e-5 * float(tot.abs().max())), i


@pytest.mark.gpu
def test_dgmc_sparse_fused_psi2_vs_reference_mode(monkeypatch):
    """DBP15K-style training step with the config's psi_2 (RelCNN(32, 32,
    3)): the fused path (ops/relconv.py) == the reference expression, S_L
    and every parameter gradient (psi_2's final bias: no gradient natively,
    ~0 in the reference - it cancels in P_i - Q_j)."""
    from deep_graph_matching_consensus_amd.models import DGMC
    from deep_graph_matching_consensus_amd.runtime import reference_mode
    torch.manual_seed(0)
    d = make_kg_pair('zh_en', scale=0.05, feature_dim=24, seed=1).to(DEV)
    model = DGMC(RelCNN(24, 32, 2), RelCNN(32, 32, 3), num_steps=3,
                 k=5).to(DEV)
    y = d.train_y
    calls = []
    orig = rc.psi2_fold

    def spy(*a, **kw):
        calls.append(1)
        return orig(*a, **kw)
    monkeypatch.setattr(rc, 'psi2_fold', spy)
    torch.manual_seed(1)
    _, S_L = model(d.x1, d.edge_index1, None, None, d.x2, d.edge_index2,
                   None, None, y)
    assert len(calls) == 3, 'fused psi_2 path not taken'
    loss = model.loss(S_L, y)
    names = [n for n, _ in model.named_parameters()]
    grads = torch.autograd.grad(loss, list(model.parameters()),
                                allow_unused=True)
    negs = S_L.__idx__[:, 5:].contiguous()
    randint = torch.randint

    def native_negatives(high, size, **kw):
        if tuple(size) == (1, d.x1.size(0), negs.size(1)):
            return negs.view(size).clone()
        return randint(high, size, **kw)
    monkeypatch.setattr(torch, 'randint', native_negatives)
    with reference_mode():
        torch.manual_seed(1)
        _, R_L = model(d.x1, d.edge_index1, None, None, d.x2, d.edge_index2,
                       None, None, y)
        loss2 = model.loss(R_L, y)
        grads2 = torch.autograd.grad(loss2, list(model.parameters()),
                                     allow_unused=True)
    assert torch.equal(S_L.__idx__, R_L.__idx__)
    assert torch.allclose(S_L.__val__, R_L.__val__, atol=1e-4)
    assert torch.allclose(loss, loss2, atol=1e-4)
    for n, a, b in zip(names, grads, grads2):
        if n == 'psi_2.final.bias':
            assert a is None or float(a.abs().max()) == 0.0
            assert b is None or float(b.abs().max()) < 1e-5
            continue
        if a is None or b is None:
            assert a is None and b is None, n
            continue
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-2), n


def _relconv64(conv, x, ei, N, dtype):
    """RelConv (/root/reference/dgmc/models/rel.py:25-31) in ``dtype``:
    root(x) + scatter-mean over in-edges of lin1(x) + over out-edges of
    lin2(x)."""
    src, dst = ei
    w1, w2 = conv.lin1.weight.to(dtype), conv.lin2.weight.to(dtype)
    wr, br = conv.root.weight.to(dtype), conv.root.bias.to(dtype)
    h1, h2 = x @ w1.t(), x @ w2.t()
    out = x @ wr.t() + br
    m_in = torch.zeros_like(out).index_add_(0, dst, h1[src])
    c_in = torch.bincount(dst, minlength=N).clamp(min=1).to(dtype)
    m_out = torch.zeros_like(out).index_add_(0, src, h2[dst])
    c_out = torch.bincount(src, minlength=N).clamp(min=1).to(dtype)
    return out + m_in / c_in[:, None] + m_out / c_out[:, None]


@pytest.mark.gpu
@pytest.mark.parametrize('cin', [300, 256])
def test_psi1_relconv_layer_full_graph_vs_fp64(cin):
    """psi_1's RelConv layers of the DBP15K config (RelCNN(300, 256, 3),
    ``/root/reference/examples/dbp15k.py:29-31``) on the full-size joint
    graph (19,388 + 19,572 entities, hub rows): the native path (exact-f32
    chunked GEMM + split SpMM, models/rel.py) forward and every gradient
    against fp64, error at most 4x the same expression's in fp32 on the
    library kernels (+ 1e-6 of the value scale)."""
    from deep_graph_matching_consensus_amd.models.rel import RelConv
    ei, n_s, n_t = _joint(device=DEV)
    N = n_s + n_t
    torch.manual_seed(cin)
    conv = RelConv(cin, 256).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(N, cin, device=DEV, generator=g).requires_grad_()
    out = conv(x, ei)
    go = torch.randn(N, 256, device=DEV, generator=g)
    leaves = [x, conv.lin1.weight, conv.lin2.weight, conv.root.weight,
              conv.root.bias]
    grads = torch.autograd.grad(out, leaves, go)
    src, dst = ei.long()

    def oracle(dtype):
        xx = x.detach().to(dtype).requires_grad_()
        ps = [p.detach().to(dtype).requires_grad_() for p in leaves[1:]]
        c2 = RelConv(cin, 256).to(DEV).to(dtype)
        with torch.no_grad():
            for p, q in zip([c2.lin1.weight, c2.lin2.weight, c2.root.weight,
                             c2.root.bias], ps):
                p.copy_(q)
        y = _relconv64(c2, xx, (src, dst), N, dtype)
        gs = torch.autograd.grad(y, [xx, c2.lin1.weight, c2.lin2.weight,
                                     c2.root.weight, c2.root.bias],
                                 go.to(dtype))
        return y, gs

    y64, g64 = oracle(torch.float64)
    y32, g32 = oracle(torch.float32)

    def check(a, b32, b64, what):
        e = float((a.detach().double() - b64).abs().max())
        e32 = float((b32.double() - b64).abs().max())
        assert e <= 4 * e32 + 1e-6 * float(b64.abs().max()), (what, e, e32)

    check(out, y32, y64, 'out')
    for n, a, b32, b64 in zip(['x', 'lin1', 'lin2', 'root.w', 'root.b'],
                              grads, g32, g64):
        check(a, b32, b64, n)
