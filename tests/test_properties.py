"""Hypothesis property tests for the data layer: CSR construction and
transpose, packed<->dense layouts, PyG-style collation and the native
pair collator."""
import numpy as np
import torch
from hypothesis import given, settings, strategies as st

from deep_graph_matching_consensus_amd.graph import Batch, Data
from deep_graph_matching_consensus_amd.graph.dense import (DenseLayout,
                                                           MaskLayout)
from deep_graph_matching_consensus_amd.graph.meta import BatchInfo
from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops.sparse import SparseOperator

SETTINGS = dict(max_examples=40, deadline=None)


@settings(**SETTINGS)
@given(st.integers(1, 12), st.integers(1, 12), st.integers(0, 60),
       st.integers(0, 2**31 - 1))
def test_csr_from_coo_and_transpose(R, C, nnz, seed):
    g = torch.Generator().manual_seed(seed)
    row = torch.randint(R, (nnz, ), generator=g)
    col = torch.randint(C, (nnz, ), generator=g)
    val = torch.randn(nnz, generator=g)
    dense = torch.zeros(R, C).index_put_((row, col), val, accumulate=True)
    op = SparseOperator.from_coo(row, col, val, R, C)
    assert op.rowptr[0] == 0 and op.rowptr[-1] == nnz
    assert (op.rowptr[1:] >= op.rowptr[:-1]).all()
    assert torch.allclose(op.to_dense(), dense, atol=1e-6)
    assert torch.allclose(op.t().to_dense(), dense.t(), atol=1e-6)
    assert op.t().t() is op


@settings(**SETTINGS)
@given(st.lists(st.integers(0, 300), min_size=1, max_size=20),
       st.sampled_from([1, 4, 64]))
def test_piece_plan_covers_every_entry_once(degrees, T):
    """piece_plan: every row gets max(1, ceil(deg / T)) pieces, in row
    order; pieces tile each row's entries exactly; unused slots map to R."""
    from deep_graph_matching_consensus_amd.ops.sparse import piece_plan
    deg = torch.tensor(degrees)
    rowptr = torch.zeros(len(degrees) + 1, dtype=torch.int32)
    rowptr[1:] = torch.cumsum(deg, 0)
    nnz = int(deg.sum())
    pptr, prow, pbeg, pend = piece_plan(rowptr, nnz, T)
    R = len(degrees)
    assert prow.numel() == R + nnz // T + 1
    seen = torch.zeros(nnz, dtype=torch.int64)
    for v in range(prow.numel()):
        code = int(prow[v])
        if code == R:
            assert v >= int(pptr[-1])
            continue
        r = code if code >= 0 else -code - 1
        npieces = int(pptr[r + 1] - pptr[r])
        assert (code < 0) == (npieces > 1)
        q = v - int(pptr[r])
        beg = int(rowptr[r]) + q * T
        end = min(int(rowptr[r + 1]), beg + T)
        assert 0 <= q < npieces
        assert (int(pbeg[v]), int(pend[v])) == (beg, end)
        seen[beg:end] += 1
    assert (seen == 1).all()
    assert ((pptr[1:] - pptr[:-1]) ==
            torch.clamp_min((deg + T - 1) // T, 1)).all()


@settings(**SETTINGS)
@given(st.lists(st.integers(0, 9), min_size=1, max_size=8),
       st.integers(1, 4))
def test_dense_layout_round_trip_matches_mask_layout(counts, C):
    counts = [max(c, 0) for c in counts]
    n = sum(counts)
    x = torch.randn(n, C)
    batch = torch.repeat_interleave(torch.arange(len(counts)),
                                    torch.tensor(counts))
    info = BatchInfo(np.array(counts, dtype=np.int64))
    lay = DenseLayout(info, torch.device('cpu'))
    dense = lay.to_dense(x)
    assert dense.shape == (len(counts), max(counts), C)
    assert torch.equal(lay.to_sparse(dense), x)
    ref = MaskLayout(batch, n, torch.device('cpu'))
    if ref.B == lay.B:                  # trailing empty graphs are invisible
        assert torch.equal(ref.to_dense(x), dense)   # to the reference mask
    assert int(lay.mask.sum()) == n


@settings(**SETTINGS)
@given(st.lists(st.tuples(st.integers(1, 6), st.integers(0, 10)),
                min_size=1, max_size=5), st.integers(0, 2**31 - 1))
def test_batch_from_data_list_increments(shapes, seed):
    g = torch.Generator().manual_seed(seed)
    data_list = []
    for n, e in shapes:
        ei = torch.randint(n, (2, e), generator=g)
        data_list.append(Data(x=torch.randn(n, 3, generator=g),
                              edge_index=ei))
    b = Batch.from_data_list(data_list)
    offs = np.cumsum([0] + [n for n, _ in shapes])
    assert b.num_graphs == len(shapes)
    assert b.x.size(0) == offs[-1]
    col = 0
    for i, (n, e) in enumerate(shapes):
        part = b.edge_index[:, col:col + e]
        assert torch.equal(part - int(offs[i]), data_list[i].edge_index)
        col += e
    assert torch.equal(b.batch, torch.repeat_interleave(
        torch.arange(len(shapes)), torch.tensor([n for n, _ in shapes])))


@settings(max_examples=15, deadline=None)
@given(st.integers(2, 12), st.integers(0, 2**31 - 1))
def test_native_collate_matches_numpy(batch_size, seed):
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets import device_loader
    if not _backend.host_available():
        return
    groups = make_keypoint_datasets(graphs=4, feature_dim=8, seed=3)
    store = GraphStore(groups, 'cpu')
    rng = np.random.default_rng(seed)
    s_ids = rng.integers(0, store.num_graphs, batch_size)
    t_ids = store.sample_partners(s_ids, rng)
    a = store._collate_host(s_ids, t_ids)
    b = device_loader._collate_numpy(store, s_ids, t_ids)
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert np.array_equal(np.asarray(u), np.asarray(v))
