"""Padded static batches (hipGraph path) must match dynamic batches."""
import numpy as np
import pytest
import torch

from deep_graph_matching_consensus_amd.datasets import (
    GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.datasets.static_batch import \
    StaticPairBatcher
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
from deep_graph_matching_consensus_amd.ops import _backend


def _setup(device='cpu'):
    groups = make_keypoint_datasets(graphs=8, feature_dim=16, seed=4)
    store = GraphStore(groups, device)
    batcher = StaticPairBatcher(store, 12, seed=0)
    torch.manual_seed(0)
    model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                 SplineCNN(8, 8, 2, 2, cat=True), num_steps=0).to(device)
    model.eval()
    return store, batcher, model


def _run(model, batch, rows, mask):
    S_0, S_L = model(batch.x_s, batch.edge_index_s, batch.edge_attr_s,
                     batch.x_s_batch, batch.x_t, batch.edge_index_t,
                     batch.edge_attr_t, batch.x_t_batch)
    y = torch.stack([rows, batch.y])
    return S_0, S_L, model.loss(S_0, y, mask=mask)


@pytest.mark.skipif(not _backend.host_available(),
                    reason='native host library not built')
def test_static_equals_dynamic_cpu():
    store, batcher, model = _setup()
    s, t = batcher.next_ids()
    dyn = store.collate(s, t)
    assert batcher.load(s, t)
    sta = batcher.materialize()
    n_s = dyn.x_s.size(0)
    assert sta.x_s.size(0) == batcher.cap_s > n_s
    assert int(sta.y_mask.sum()) == n_s
    assert torch.equal(sta.y[:n_s], dyn.y)

    a0, _, la = _run(model, dyn, torch.arange(n_s), None)
    grads_a = torch.autograd.grad(la, list(model.parameters()),
                                  allow_unused=True)
    b0, _, lb = _run(model, sta, torch.arange(batcher.cap_s), sta.y_mask)
    grads_b = torch.autograd.grad(lb, list(model.parameters()),
                                  allow_unused=True)
    N_t = a0.size(1)
    assert torch.allclose(a0, b0[:n_s, :N_t], atol=1e-6)
    assert torch.allclose(la, lb, atol=1e-6)
    for ga, gb in zip(grads_a, grads_b):
        if ga is None:
            assert gb is None or gb.abs().max() == 0
        else:
            assert torch.allclose(ga, gb, atol=1e-5)


@pytest.mark.skipif(not _backend.host_available(),
                    reason='native host library not built')
def test_static_consensus_finite_cpu():
    store, batcher, model = _setup()
    model.num_steps = 2
    model.train()
    assert batcher.load()
    sta = batcher.materialize()
    _, S_L, loss = _run(model, sta, torch.arange(batcher.cap_s), sta.y_mask)
    loss.backward()
    assert torch.isfinite(loss)
    for p in model.parameters():
        assert p.grad is None or torch.isfinite(p.grad).all()


@pytest.mark.skipif(not _backend.host_available(),
                    reason='native host library not built')
def test_rank_shard_smaller_than_batch():
    """8-rank sharding of a small store: every rank's shard has fewer source
    graphs than the batch; every batch still has exactly B pairs with
    consistent pair pointers (regression: a short id list shifted the
    static buffer layout)."""
    from deep_graph_matching_consensus_amd.datasets import DevicePairLoader
    groups = make_keypoint_datasets(graphs=8, feature_dim=16, seed=4)
    store = GraphStore(groups, 'cpu')
    B, world = 64, 8
    for rank in range(world):
        sources = np.arange(store.num_graphs)[rank::world]
        assert len(sources) < B
        batcher = StaticPairBatcher(store, B, sources=sources, seed=rank)
        n = store.node_ptr[1:] - store.node_ptr[:-1]
        for _ in range(3):
            s, t = batcher.next_ids()
            assert len(s) == len(t) == B
            assert set(s.tolist()) <= set(sources.tolist())
            assert batcher.load(s, t)
            ptr = batcher.v['ptr_s'].clone()
            assert int(ptr[0]) == 0 and int(ptr[-1]) == int(n[s].sum())
            assert bool((ptr[1:] >= ptr[:-1]).all())
        with pytest.raises(ValueError):
            batcher.load(s[:B - 1], t[:B - 1])
        loader = DevicePairLoader(store, B, sources=sources, seed=rank)
        it = loader.forever()
        for _ in range(3):
            assert next(it).num_graphs == B


def test_capacity_covers_probe():
    store, batcher, _ = _setup()
    n = store.node_ptr[1:] - store.node_ptr[:-1]
    rng = np.random.default_rng(7)
    for _ in range(20):
        s, t = batcher.next_ids()
        assert n[s].sum() < batcher.cap_s and n[t].sum() < batcher.cap_t


@pytest.mark.gpu
def test_assembled_spline_plan_matches_generic_build():
    """The per-graph plan assembly (plan_assembly.hip) reproduces the generic
    per-batch spline operator bit for bit on every valid row, for A and A^T."""
    from deep_graph_matching_consensus_amd.ops import plans
    from deep_graph_matching_consensus_amd.ops.sparse import spmm
    store, batcher, model = _setup('cuda')
    for _ in range(2):   # second step: a different batch in the same buffers
        assert batcher.load()
        batch = batcher.materialize()
        cs, ct = batcher.cap_s, batcher.cap_t
        N = cs + ct
        ei_u = batcher.v['ei']
        ea_u = torch.cat([batch.edge_attr_s, batch.edge_attr_t])
        ea_view = batcher.v['ea_val'] if batcher.ea_dim else \
            batch.edge_attr_s._base
        op = plans.spline_plan(ei_u, ea_view, N, (5, 5), (1, 1), 1, True)
        assert type(op).__name__ == '_StaticSlotOperator'
        ref_op = plans.spline_plan(ei_u.clone(), ea_u, N, (5, 5), (1, 1), 1,
                                   True)
        assert type(ref_op).__name__ == 'SparseOperator'
        ptr_s = batcher.v['ptr_s'].cpu()
        ptr_t = batcher.v['ptr_t'].cpu()
        valid = torch.zeros(N, dtype=torch.bool)
        valid[:int(ptr_s[-1])] = True
        valid[cs:cs + int(ptr_t[-1])] = True
        valid = valid.cuda()
        x = torch.randn(N * 26, 32, device='cuda')
        ya, yb = spmm(op, x), spmm(ref_op, x)
        assert torch.equal(ya[valid], yb[valid])
        g = torch.randn(N, 32, device='cuda') * valid.view(-1, 1)
        za, zb = spmm(op.t(), g), spmm(ref_op.t(), g)
        assert torch.equal(za, zb)
        assert int(op.rowptr[-1]) == int(op.t().rowptr[-1])
        # entry rows written by the assembler == rows derived from rowptr
        E = int(op.rowptr[-1])
        rows = torch.repeat_interleave(
            torch.arange(N, device='cuda'),
            (op.rowptr[1:] - op.rowptr[:-1]).long())
        assert torch.equal(op.row[:E], rows)
        assert torch.equal(op.rowptr[1:] >= op.rowptr[:-1],
                           torch.ones(N, dtype=torch.bool, device='cuda'))


@pytest.mark.gpu
def test_static_batch_union_views_gpu():
    store, batcher, model = _setup('cuda')
    assert batcher.load()
    batch = batcher.materialize()
    cs = batcher.cap_s
    # x_s / x_t are row blocks of one gathered tensor; DGMC re-joins them
    # without a copy.
    from deep_graph_matching_consensus_amd.models.dgmc import _cat_rows
    joint = _cat_rows(batch.x_s, batch.x_t)
    assert joint.data_ptr() == batch.x_s.data_ptr()
    assert torch.equal(joint, torch.cat([batch.x_s, batch.x_t]))
    ei = torch.cat([batch.edge_index_s, batch.edge_index_t + cs], dim=1)
    assert torch.equal(ei, batcher.v['ei'])


def test_static_batch_typed_tail_matches_derived_views():
    """The collator's typed tail (local target edges, bool mask, int32 ptr /
    counts, gathered edge attributes) equals what the step used to derive on
    the device with cast / subtraction / gather kernels."""
    store, batcher, _ = _setup()
    for _ in range(2):
        assert batcher.load()
        v = batcher.v
        cs, es = batcher.cap_s, batcher.ecap_s
        assert torch.equal(v['ei_tl'], v['ei'][:, es:] - cs)
        assert torch.equal(v['ymask_b'], v['ymask'].to(torch.bool))
        assert torch.equal(v['ptr32_s'], v['ptr_s'].to(torch.int32))
        assert torch.equal(v['ptr32_t'], v['ptr_t'].to(torch.int32))
        assert torch.equal(v['cnt32_s'],
                           (v['ptr_s'][1:] - v['ptr_s'][:-1]).to(torch.int32))
        assert torch.equal(v['cnt32_t'],
                           (v['ptr_t'][1:] - v['ptr_t'][:-1]).to(torch.int32))
        assert batcher.ea_dim == store.edge_attr.size(1)
        assert torch.equal(v['ea_val'],
                           batcher.edge_attr.index_select(0, v['ea']))
        batch = batcher.materialize()
        assert batch.y_mask.dtype == torch.bool
        assert torch.equal(batch.edge_index_t, v['ei'][:, es:] - cs)
