"""Training candidate set of the sparse path (K12, csrc/hip/candidates.hip)
against the ATen expression of ``/root/reference/dgmc/models/dgmc.py:190-195``
(randint + cat + ``__include_gt__``): top-k columns copied, negatives in
``[0, N_t)`` and roughly uniform, every ground truth present, only the last
column of a row patched, fresh negatives per call and under graph replay."""
import pytest
import torch

from deep_graph_matching_consensus_amd.models import DGMC
from deep_graph_matching_consensus_amd.ops import _backend

pytestmark = pytest.mark.gpu


def _case(B=3, N_s=700, N_t=900, k=10, G=1500, seed=0):
    g = torch.Generator().manual_seed(seed)
    topk = torch.stack([torch.randperm(N_t, generator=g)[:k]
                        for _ in range(B * N_s)]).view(B, N_s, k)
    rows = torch.randperm(B * N_s, generator=g)[:G]
    # Half of the ground truths already among the top-k, half not.
    cols = torch.randint(N_t, (G, ), generator=g)
    cols[::2] = topk.view(-1, k)[rows[::2], 3]
    return topk.cuda(), rows.cuda(), cols.cuda()


def test_train_candidates_matches_aten_semantics():
    topk, rows, cols = _case()
    B, N_s, k = topk.shape
    N_t, kr = 900, 10
    out = _backend.ops().train_candidates(topk, N_t, kr, rows, cols)
    assert out.shape == (B, N_s, k + kr) and out.dtype == torch.long
    flat, tk = out.view(-1, k + kr), topk.view(-1, k)
    # top-k columns untouched except a patched last column (kr = 0 case
    # below); negatives in range.
    assert torch.equal(flat[:, :k], tk)
    neg = flat[:, k:]
    assert int(neg.min()) >= 0 and int(neg.max()) < N_t
    # Oracle: the reference's __include_gt__ applied to the kernel's own
    # negatives before the patch.
    unpatched = flat.clone()
    present = (unpatched[rows] == cols.view(-1, 1)).any(-1)
    assert bool(present.all())
    # Rows with a ground truth: equal to the DGMC helper on the same input
    # with the last column restored where it was patched.
    expect = DGMC._include_gt(out.clone(), torch.arange(B * N_s,
                                                        device=out.device),
                              torch.stack([rows, cols]))
    assert torch.equal(expect, out)
    # Non-ground-truth rows keep their negatives; negatives look uniform.
    # (multinomial counts: coefficient of variation ~ 1 / sqrt(mean))
    hist = torch.bincount(neg.reshape(-1), minlength=N_t).float()
    mean = float(hist.mean())
    assert float(hist.std()) / mean < 1.2 / mean ** 0.5
    assert int(hist.min()) > 0


def test_train_candidates_gt_patch_and_no_negatives():
    topk, rows, cols = _case(B=1, N_s=400, N_t=500, k=4, G=300, seed=1)
    out = _backend.ops().train_candidates(topk, 500, 0, rows, cols)
    flat, tk = out.view(-1, 4), topk.view(-1, 4)
    was = (tk[rows] == cols.view(-1, 1)).any(-1)
    # Missing ground truths overwrite the last top-k column only.
    assert torch.equal(flat[rows[~was], 3], cols[~was])
    assert torch.equal(flat[rows[~was], :3], tk[rows[~was], :3])
    assert torch.equal(flat[rows[was]], tk[rows[was]])
    other = torch.ones(flat.size(0), dtype=torch.bool, device=flat.device)
    other[rows] = False
    assert torch.equal(flat[other], tk[other])


def test_train_candidates_fresh_negatives_and_graph_replay():
    topk, rows, cols = _case(G=0)
    ops = _backend.ops()
    torch.manual_seed(0)
    a = ops.train_candidates(topk, 900, 10, rows, cols)
    b = ops.train_candidates(topk, 900, 10, rows, cols)
    assert not torch.equal(a, b)
    torch.manual_seed(0)
    assert torch.equal(ops.train_candidates(topk, 900, 10, rows, cols), a)
    # Captured: every replay draws new negatives from the generator offset.
    static = {}
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.train_candidates(topk, 900, 10, rows, cols)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static['out'] = ops.train_candidates(topk, 900, 10, rows, cols)
    g.replay()
    first = static['out'].clone()
    g.replay()
    assert not torch.equal(first, static['out'])
    assert torch.equal(first[..., :10], topk)


# (DBP15K size: 2 radix digits; 140k columns: 3 digits; a partial tile;
# 2.4M entries: more than 256 tiles, the scanned count table)
@pytest.mark.parametrize('B,N_s,N_t,k', [(1, 1937, 1960, 20), (4, 50, 70, 7),
                                         (1, 19388, 19572, 10),
                                         (2, 3000, 70000, 5), (1, 3, 5, 2),
                                         (1, 200000, 60000, 12)])
def test_candidate_csc_matches_stable_argsort(B, N_s, N_t, k):
    g = torch.Generator().manual_seed(B)
    # Skewed targets (a few hubs), like top-k of random-init embeddings.
    w = torch.rand(N_t, generator=g) ** 8
    S_idx = torch.multinomial(w, B * N_s * k, replacement=True,
                              generator=g).view(B, N_s, k).cuda()
    col, rowptr, colptr, perm, row_of = _backend.ops().candidate_csc(
        S_idx, N_t)
    offs = (torch.arange(B, device='cuda') * N_t).view(B, 1, 1)
    ref_col = (S_idx + offs).reshape(-1)
    ref_perm = torch.argsort(ref_col, stable=True)
    counts = torch.bincount(ref_col, minlength=B * N_t)
    ref_colptr = torch.cat([counts.new_zeros(1), counts.cumsum(0)])
    assert torch.equal(col.long(), ref_col)
    assert torch.equal(rowptr.long(),
                       torch.arange(B * N_s + 1, device='cuda') * k)
    assert torch.equal(perm.long(), ref_perm)
    assert torch.equal(colptr.long(), ref_colptr)
    assert torch.equal(row_of.long(), ref_perm // k)
