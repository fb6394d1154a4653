"""Opt-in Sinkhorn normalisation (extension; the reference uses softmax)."""
import pytest
import torch

from deep_graph_matching_consensus_amd.datasets import (
    DevicePairLoader, GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
from deep_graph_matching_consensus_amd.ops import reference as ref


def test_masked_sinkhorn_doubly_stochastic_on_valid_block():
    torch.manual_seed(0)
    B, N = 3, 7
    S_hat = torch.randn(B, N, N)
    n = torch.tensor([7, 5, 3])
    mask = ref.count_mask(n, n, N, N)
    S = ref.masked_sinkhorn(S_hat, mask, num_iters=50)
    assert torch.isfinite(S).all()
    assert (S[~mask] == 0).all()
    for b in range(B):
        blk = S[b, :n[b], :n[b]]
        assert torch.allclose(blk.sum(-1), torch.ones(n[b]), atol=1e-5)
        assert torch.allclose(blk.sum(-2), torch.ones(n[b]), atol=1e-3)
    # Zero iterations degenerate to the masked softmax.
    assert torch.allclose(ref.masked_sinkhorn(S_hat, mask, num_iters=0),
                          ref.masked_softmax(S_hat, mask), atol=1e-6)


def test_dgmc_sinkhorn_forward_backward():
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=1)
    store = GraphStore(groups, 'cpu')
    b = next(iter(DevicePairLoader(store, batch_size=6, seed=0)))
    torch.manual_seed(0)
    model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                 SplineCNN(8, 8, 2, 2, cat=True), num_steps=2,
                 normalization='sinkhorn', sinkhorn_iters=5)
    S_0, S_L = model(b.x_s, b.edge_index_s, b.edge_attr_s, b.x_s_batch,
                     b.x_t, b.edge_index_t, b.edge_attr_t, b.x_t_batch)
    assert torch.allclose(S_L.sum(-1), torch.ones(S_L.size(0)), atol=1e-5)
    y = torch.stack([torch.arange(b.y.numel()), b.y])
    loss = model.loss(S_0, y) + model.loss(S_L, y)
    loss.backward()
    assert all(p.grad is not None for p in model.mlp.parameters())


def _sinkhorn_case(B=37, Ns=19, Nt=23, seed=0):
    g = torch.Generator().manual_seed(seed)
    S_hat = torch.randn(B, Ns, Nt, generator=g) * 3
    n_s = torch.randint(1, Ns + 1, (B, ), generator=g)
    n_t = torch.randint(1, Nt + 1, (B, ), generator=g)
    n_s[0], n_t[0] = Ns, Nt
    return S_hat, n_s, n_t


# pair tiles of the register buckets (NM = 16, 24, 32, 48, 64)
SHAPES = [(20, 12, 9), (37, 19, 23), (8, 30, 28), (6, 40, 45), (9, 64, 50)]


@pytest.mark.gpu
@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('iters,tau', [(10, 1.0), (0, 1.0), (25, 0.5)])
def test_sinkhorn_kernel_matches_fp64_reference(iters, tau, shape):
    """csrc/hip/sinkhorn.hip forward + backward against the log-domain
    oracle (ops/reference.py::masked_sinkhorn) under fp64 autograd."""
    from deep_graph_matching_consensus_amd.ops import _backend
    assert _backend.hip_available()
    S_hat, n_s, n_t = _sinkhorn_case(*shape)
    B, Ns, Nt = S_hat.shape
    mask = ref.count_mask(n_s, n_t, Ns, Nt)
    Sd = S_hat.double().requires_grad_()
    P_ref = ref.masked_sinkhorn(Sd, mask, iters, tau)
    G = torch.randn(B, Ns, Nt, dtype=torch.float64)
    dS_ref, = torch.autograd.grad(P_ref, Sd, G)
    ops = _backend.ops()
    dev = 'cuda'
    S = S_hat.to(dev)
    ns, nt = n_s.int().to(dev), n_t.int().to(dev)
    P, ah, bh = ops.sinkhorn_fwd(S, ns, nt, iters, tau)
    torch.testing.assert_close(P.cpu().double(), P_ref.detach(), atol=2e-6,
                               rtol=1e-5)
    dS = ops.sinkhorn_bwd(G.float().to(dev), S, ns, nt, ah, bh, iters, tau)
    torch.testing.assert_close(dS.cpu().double(), dS_ref, atol=2e-5,
                               rtol=1e-4)


@pytest.mark.gpu
def test_dgmc_sinkhorn_gpu_matches_cpu():
    """The opt-in Sinkhorn model on the GPU (HIP kernel) equals the CPU
    oracle path (eval mode, same random indicators)."""
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=1)
    out = {}
    for dev in ('cpu', 'cuda'):
        store = GraphStore(groups, dev)
        b = next(iter(DevicePairLoader(store, batch_size=6, seed=0)))
        torch.manual_seed(0)
        model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                     SplineCNN(8, 8, 2, 2, cat=True), num_steps=2,
                     normalization='sinkhorn', sinkhorn_iters=5).to(dev)
        model.eval()
        r = torch.randn(2, b.x_s.size(0), 8).to(dev)

        def fake_randn(*a, **k):
            return r.to(k.get('dtype', r.dtype))
        orig = torch.randn
        torch.randn = fake_randn
        try:
            S_0, S_L = model(b.x_s, b.edge_index_s, b.edge_attr_s,
                             b.x_s_batch, b.x_t, b.edge_index_t,
                             b.edge_attr_t, b.x_t_batch)
        finally:
            torch.randn = orig
        y = torch.stack([torch.arange(b.y.numel(), device=dev), b.y])
        loss = model.loss(S_0, y) + model.loss(S_L, y)
        grads = torch.autograd.grad(loss, list(model.mlp.parameters()))
        out[dev] = (S_L.detach().cpu(), [g.cpu() for g in grads])
    torch.testing.assert_close(out['cuda'][0], out['cpu'][0], atol=1e-4,
                               rtol=1e-3)
    for a, b in zip(out['cuda'][1], out['cpu'][1]):
        torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('R,iters', [(64, 10), (128, 5), (256, 0)])
def test_sinkhorn_transport_kernel_matches_fp64(R, iters, shape):
    """The fused Sinkhorn + transport kernel (joint ``[r_s; P^T r_s]``,
    optional ``P``) and its backward (``dL/dP = G_P + r_s g_t^T`` through
    the Sinkhorn Jacobians, plus a passthrough addend) against fp64
    autograd of the oracle."""
    from deep_graph_matching_consensus_amd.ops import _backend
    assert _backend.hip_available()
    S_hat, n_s, n_t = _sinkhorn_case(*shape, seed=R)
    B, Ns, Nt = S_hat.shape
    mask = ref.count_mask(n_s, n_t, Ns, Nt)
    g = torch.Generator().manual_seed(1)
    ptr_s = torch.cat([torch.zeros(1, dtype=torch.long), n_s.cumsum(0)])
    ptr_t = torch.cat([torch.zeros(1, dtype=torch.long), n_t.cumsum(0)])
    rows_s, rows_t = int(ptr_s[-1]), int(ptr_t[-1])
    r_s = torch.randn(rows_s, R, generator=g, dtype=torch.float64)
    Sd = S_hat.double().requires_grad_()
    P = ref.masked_sinkhorn(Sd, mask, iters, 1.0)
    r_t = []
    for b in range(B):
        blk = P[b, :n_s[b], :n_t[b]]
        r_t.append(blk.t() @ r_s[ptr_s[b]:ptr_s[b + 1]])
    joint = torch.cat([r_s] + r_t)
    gj = torch.randn(rows_s + rows_t, R, generator=g, dtype=torch.float64)
    gP = torch.randn(B, Ns, Nt, generator=g, dtype=torch.float64)
    add = torch.randn(B, Ns, Nt, generator=g, dtype=torch.float64)
    dS_ref, = torch.autograd.grad((joint * gj).sum() + (P * gP).sum(), Sd,
                                  retain_graph=True)
    dS_ref = dS_ref + add
    ops = _backend.ops()
    dev = 'cuda'
    S = S_hat.to(dev)
    ps, pt = ptr_s.int().to(dev), ptr_t.int().to(dev)
    rs = r_s.float().to(dev)
    out = ops.sinkhorn_transport(S, rs, ps, pt, rows_t, iters, 1.0, True)
    torch.testing.assert_close(out[0].cpu().double(), joint.detach(),
                               atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(out[1].cpu().double(), P.detach(), atol=2e-6,
                               rtol=1e-5)
    dS = ops.sinkhorn_transport_bwd(gP.float().to(dev), gj.float().to(dev),
                                    rs, S, ps, pt, out[2], out[3], iters,
                                    1.0, add.float().to(dev))
    torch.testing.assert_close(dS.cpu().double(), dS_ref, atol=1e-4,
                               rtol=1e-4)
    # without P / addend
    out2 = ops.sinkhorn_transport(S, rs, ps, pt, rows_t, iters, 1.0, False)
    assert torch.equal(out2[0], out[0])
    dS2 = ops.sinkhorn_transport_bwd(None, gj.float().to(dev), rs, S, ps, pt,
                                     out[2], out[3], iters, 1.0, None)
    dS2_ref, = torch.autograd.grad((joint * gj).sum(), Sd)
    torch.testing.assert_close(dS2.cpu().double(), dS2_ref, atol=1e-4,
                               rtol=1e-4)


@pytest.mark.gpu
def test_dgmc_sinkhorn_fused_gpu_matches_cpu():
    """The fused Sinkhorn consensus loop (R = 64: one kernel per step for
    normalisation + transport, psi_2's final Linear folded) equals the CPU
    oracle path: outputs and every parameter gradient."""
    from deep_graph_matching_consensus_amd.models import dgmc as dgmc_mod
    assert dgmc_mod.SINKHORN_FUSED
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=1)
    out = {}
    for dev in ('cpu', 'cuda'):
        store = GraphStore(groups, dev)
        b = next(iter(DevicePairLoader(store, batch_size=6, seed=0)))
        torch.manual_seed(0)
        model = DGMC(SplineCNN(16, 32, 2, 2, cat=False),
                     SplineCNN(64, 32, 2, 2, cat=True), num_steps=3,
                     normalization='sinkhorn', sinkhorn_iters=6).to(dev)
        r = torch.randn(3, b.x_s.size(0), 64).to(dev)

        def fake_randn(*a, **k):
            return r.to(k.get('dtype', r.dtype))
        orig = torch.randn
        torch.randn = fake_randn
        try:
            S_0, S_L = model(b.x_s, b.edge_index_s, b.edge_attr_s,
                             b.x_s_batch, b.x_t, b.edge_index_t,
                             b.edge_attr_t, b.x_t_batch)
        finally:
            torch.randn = orig
        y = torch.stack([torch.arange(b.y.numel(), device=dev), b.y])
        loss = model.loss(S_0, y) + model.loss(S_L, y)
        params = [p for p in model.parameters() if p.requires_grad]
        grads = torch.autograd.grad(loss, params, allow_unused=True)
        out[dev] = (S_0.detach().cpu(), S_L.detach().cpu(),
                    [None if g is None else g.cpu() for g in grads])
    torch.testing.assert_close(out['cuda'][0], out['cpu'][0], atol=1e-4,
                               rtol=1e-3)
    torch.testing.assert_close(out['cuda'][1], out['cpu'][1], atol=1e-4,
                               rtol=1e-3)
    for a, b in zip(out['cuda'][2], out['cpu'][2]):
        if a is None or b is None:
            assert a is None or float(a.abs().max()) == 0
            continue
        torch.testing.assert_close(a, b, atol=2e-4, rtol=2e-3)
