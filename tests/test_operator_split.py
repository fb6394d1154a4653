"""Row split of static skewed operators (``SparseOperator.split_rows``, the
plan of ``spmm.hip::spmm_split_kernel``) and the relational plan's static
flag - CPU checks of the host-side plan (the kernel itself is checked
against the oracle in ``tests/test_hip_kernels.py``)."""
import torch

from deep_graph_matching_consensus_amd.ops.plans import relational_plan
from deep_graph_matching_consensus_amd.ops.sparse import PIECE, SparseOperator


def test_split_rows_partitions_rows_by_length():
    g = torch.Generator().manual_seed(0)
    deg = torch.randint(0, 3 * PIECE, (97, ), generator=g)
    deg[3] = 500
    deg[4] = PIECE
    deg[5] = PIECE + 1
    row = torch.repeat_interleave(torch.arange(97), deg)
    col = torch.randint(50, (row.numel(), ), generator=g)
    op = SparseOperator.from_coo(row, col, torch.ones(row.numel()), 97, 50)
    short, long_ = op.split_rows()
    assert short.dtype == torch.int32 and long_.dtype == torch.int32
    both = torch.cat([short, long_]).long().sort().values
    assert torch.equal(both, torch.arange(97))
    counts = op.rowptr[1:] - op.rowptr[:-1]
    assert bool((counts[short.long()] <= PIECE).all())
    assert bool((counts[long_.long()] > PIECE).all())
    assert 4 in short.tolist() and 5 in long_.tolist() and 3 in long_.tolist()
    assert op.split_rows() is op.split_rows()          # cached


def test_relational_plan_is_static_and_balanced():
    g = torch.Generator().manual_seed(1)
    ei = torch.randint(40, (2, 300), generator=g)
    plan = relational_plan(ei, 40)
    assert plan.balanced and plan.static
    assert plan.t().balanced and plan.t().static
