"""bf16x6 slot GEMM (csrc/hip/slot_gemm_x6.hip) at the headline shapes.

The gate for making it the default fp32 path ("bf16x6"): on
every headline GEMM shape - psi_1 1024->256 and 256->256, psi_2 128->128,
forward (gathered X W_s) and input gradient (dY_c W_s^T) - the max error
against an fp64 oracle must not exceed that of the exact-f32 MFMA kernel
(``slot_gemm2`` / ``slot_gemm``, a k-ordered fmaf chain) on the same
inputs.  The operator is the PascalVOC-shaped static training batch of the
benchmark (512 pairs, union of source and target graphs, ~10k nodes).
"""
import pytest
import torch

from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops import slot_gemm as sg
from deep_graph_matching_consensus_amd.ops.plans import spline_plan

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def headline_plan():
    from deep_graph_matching_consensus_amd.datasets import (
        PASCAL_VOC_CATEGORIES, GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.datasets.static_batch import \
        StaticPairBatcher
    assert _backend.hip_available()
    groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, graphs=64,
                                    feature_dim=16, seed=0)
    store = GraphStore(groups, DEV, valid_pairs=True)
    b = StaticPairBatcher(store, 512, seed=0)
    assert b.load()
    b.materialize()
    N = b.cap_s + b.cap_t
    op = spline_plan(b.v['ei'], b.v['ea_val'], N, (5, 5), (1, 1), 1,
                     root=True)
    plan = sg.compact_plan(op, 26)
    plan.test_op = op
    return N, plan


def _slot_rows(plan):
    seg = plan.seg.cpu().tolist()
    src = plan.src.long()
    return [(s, seg[s], seg[s + 1]) for s in range(len(seg) - 1)], src


def _oracle_fwd(plan, x, w, r):
    """fp64 Y[p] = x[src p] W_{slot p} (rows with src < 0: left at 0)."""
    W = torch.cat([w, r[None]], 0).double()
    Y = torch.zeros(plan.src.numel(), w.size(2), dtype=torch.float64,
                    device=DEV)
    slots, src = _slot_rows(plan)
    for s, a, b in slots:
        rows = src[a:b]
        ok = rows >= 0
        Y[a:b][ok] = x.double()[rows[ok]] @ W[s]
    return Y


def _oracle_dx(plan, dy, w, r):
    """fp64 Z[p] = dY[p] W_{slot p}^T."""
    W = torch.cat([w, r[None]], 0).double()
    Z = torch.zeros(dy.size(0), w.size(1), dtype=torch.float64, device=DEV)
    slots, src = _slot_rows(plan)
    for s, a, b in slots:
        Z[a:b] = dy.double()[a:b] @ W[s].t()
    return Z


def _valid(plan):
    return plan.src.long() >= 0


def _err(a, ref, rows):
    return float((a.double() - ref)[rows].abs().max())


@pytest.mark.parametrize('cin,cout', [(128, 128), (256, 256), (1024, 256)])
def test_x6_forward_error_not_above_exact_f32(headline_plan, cin, cout):
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(cin)
    x = torch.randn(N, cin, device=DEV, generator=g)
    w = torch.randn(25, cin, cout, device=DEV, generator=g) / cin ** 0.5
    r = torch.randn(cin, cout, device=DEV, generator=g) / cin ** 0.5
    y6 = ops.slot_gemm_x6(ops.split3(x), plan.src, plan.seg,
                          ops.slot_weight_x3(w, r, True), True, None)
    y32 = ops.slot_gemm2(x, plan.src, plan.seg, ops.slot_weight_t(w, r),
                         None, True)
    ref = _oracle_fwd(plan, x, w, r)
    rows = _valid(plan)
    e6, e32 = _err(y6, ref, rows), _err(y32, ref, rows)
    assert e6 <= e32, (e6, e32)
    assert e6 < 1e-5 * float(ref[rows].abs().max())


@pytest.mark.parametrize('cin,cout', [(128, 128), (256, 256), (1024, 256)])
def test_x6_input_grad_error_not_above_exact_f32(headline_plan, cin, cout):
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(7 + cin)
    P = plan.src.numel()
    dy = torch.randn(P, cout, device=DEV, generator=g)
    w = torch.randn(25, cin, cout, device=DEV, generator=g) / cout ** 0.5
    r = torch.randn(cin, cout, device=DEV, generator=g) / cout ** 0.5
    z6 = ops.slot_gemm_x6(ops.split3(dy), plan.src, plan.seg,
                          ops.slot_weight_x3(w, r, False), False, None)
    if cout >= 256:
        z32 = ops.slot_gemm2(dy, plan.src, plan.seg, w.contiguous(),
                             r.contiguous(), False)
    else:
        z32 = ops.slot_gemm(dy, plan.src, plan.seg, w.contiguous(),
                            r.contiguous(), True, None)
    ref = _oracle_dx(plan, dy, w, r)
    rows = torch.zeros(P, dtype=torch.bool, device=DEV)
    rows[:int(plan.seg[-1])] = True
    e6, e32 = _err(z6, ref, rows), _err(z32, ref, rows)
    assert e6 <= e32, (e6, e32)


def test_x6_dx_tile_list(headline_plan):
    """With a row-tile list (psi_2's target-source rows) exactly the listed
    tiles are computed, equal to the full pass on those rows."""
    N, plan = headline_plan
    ops = _backend.ops()
    P = plan.src.numel()
    dy = torch.randn(P, 128, device=DEV)
    w = torch.randn(25, 128, 128, device=DEV) / 12
    r = torch.randn(128, 128, device=DEV) / 12
    b3 = ops.slot_weight_x3(w, r, False)
    full = ops.slot_gemm_x6(ops.split3(dy), plan.src, plan.seg, b3, False,
                            None)
    tiles = sg.dx_tiles(plan, N // 2, unit=256)
    part = ops.slot_gemm_x6(ops.split3(dy), plan.src, plan.seg, b3, False,
                            tiles)
    cnt = int(tiles[-1])
    assert 0 < cnt < P // 256
    for t in tiles[:cnt].tolist():
        assert torch.equal(part[t * 256:(t + 1) * 256],
                           full[t * 256:(t + 1) * 256])


@pytest.mark.parametrize('cin,cout', [(128, 128), (256, 256), (1024, 256)])
def test_x6_input_grad_fp32_operand_equals_planes(headline_plan, cin, cout):
    """fp32 dY_c split inside the dX kernel's LDS staging gives bit-for-bit
    the planes path's result (same split, same MFMA order), full and with
    a row-tile list."""
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(5 + cin)
    P = plan.src.numel()
    dy = torch.randn(P, cout, device=DEV, generator=g)
    w = torch.randn(25, cin, cout, device=DEV, generator=g) / cout ** 0.5
    r = torch.randn(cin, cout, device=DEV, generator=g) / cout ** 0.5
    b3 = ops.slot_weight_x3(w, r, False)
    for tiles in (None, sg.dx_tiles(plan, N // 2, unit=256)):
        zp = ops.slot_gemm_x6(ops.split3(dy), plan.src, plan.seg, b3, False,
                              tiles)
        zf = ops.slot_gemm_x6(dy, plan.src, plan.seg, b3, False, tiles)
        if tiles is None:
            used = int(plan.seg[-1])      # rows past seg[S] are not written
            assert torch.equal(zf[:used], zp[:used]), float(
                (zf[:used] - zp[:used]).abs().max())
        else:
            for t in tiles[:int(tiles[-1])].tolist():
                assert torch.equal(zf[t * 256:(t + 1) * 256],
                                   zp[t * 256:(t + 1) * 256])


@pytest.mark.parametrize('cin,cout,uses', [(128, 128, 10), (256, 256, 1),
                                           (1024, 256, 1)])
def test_x6_weight_grad_fp32_dy_equals_planes(headline_plan, cin, cout,
                                              uses):
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(13 + cin)
    P = plan.src.numel()
    used = int(plan.seg[-1])
    xf = [torch.randn(N, cin, device=DEV, generator=g) for _ in range(uses)]
    xs = [ops.split3(x) for x in xf]
    dys = []
    for _ in range(uses):
        d = torch.randn(P, cout, device=DEV, generator=g)
        d[used:] = 0
        d[plan.src.long() < 0] = 0
        dys.append(d)
    rounds = 1 if cin == 128 else (2 if cin == 256 else 6)
    wp = ops.slot_wgrad_x6(xs, [ops.split3(d) for d in dys], plan.src,
                           plan.seg, rounds)
    wf = ops.slot_wgrad_x6(xs, dys, plan.src, plan.seg, rounds)
    assert torch.equal(wf, wp), float((wf - wp).abs().max())
    # fp32 X rows as well (split in the kernel)
    wff = ops.slot_wgrad_x6(xf, dys, plan.src, plan.seg, rounds)
    assert torch.equal(wff, wp), float((wff - wp).abs().max())


@pytest.mark.parametrize('cin,cout,uses', [(128, 128, 10), (256, 256, 1),
                                           (1024, 256, 1)])
def test_x6_weight_grad_gathered_dy_equals_rowmap(headline_plan, cin, cout,
                                                  uses):
    """dY_c rows built inside the weight gradient's staging from the node
    gradient g' and the rowmap entry table (no dY_c tensor) give bit-for-bit
    the result on the rowmap SpMM's dY_c (same fmaf chains, same order)."""
    N, plan = headline_plan
    ops = _backend.ops()
    At = plan.test_op.t()
    ell = sg.rowmap_ranges(plan, At)
    assert ell.numel() == 8 * plan.src.numel()
    g = torch.Generator(device=DEV).manual_seed(29 + cin)
    xs = [ops.split3(torch.randn(N, cin, device=DEV, generator=g))
          for _ in range(uses)]
    gs = [torch.randn(N, cout, device=DEV, generator=g) for _ in range(uses)]
    dys = [ops.slot_spmm_rowmap(At.rowptr, At.col, At.val, plan.cinv, gu,
                                plan.seg, ell, False) for gu in gs]
    rounds = 1 if cin == 128 else (2 if cin == 256 else 6)
    wd = ops.slot_wgrad_x6(xs, dys, plan.src, plan.seg, rounds)
    wg = ops.slot_wgrad_x6(xs, gs, plan.src, plan.seg, rounds, ell, At.col,
                           At.val)
    assert torch.equal(wg, wd), float((wg - wd).abs().max())
    # rows with more than three entries take the (col, val) walk
    n = ell.view(-1, 8)[:, 3]
    assert int((n > 3).sum()) > 0


def test_x6_f32dy_training_step_matches_planes(monkeypatch):
    """The fp32-X forward and fp32-dY backward give the plane path's
    output and gradients."""
    from deep_graph_matching_consensus_amd.nn.conv import SplineConv
    torch.manual_seed(0)
    N = 600
    ei = torch.randint(N, (2, 4 * N), device=DEV)
    ea = torch.rand(ei.size(1), 2, device=DEV)
    conv = SplineConv(128, 128, 2, kernel_size=5).to(DEV)
    x = torch.randn(N, 128, device=DEV, requires_grad=True)
    grads = []
    for flag in (False, True):
        monkeypatch.setattr(sg, 'F32DY', flag)
        monkeypatch.setattr(sg, 'F32X', flag)
        conv.zero_grad()
        x.grad = None
        conv(x, ei, ea).square().sum().backward()
        grads.append([x.grad.clone()] +
                     [p.grad.clone() for p in conv.parameters()])
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('cin,cout', [(128, 128), (256, 256), (1024, 256)])
def test_x6_forward_fp32_gather_equals_planes(headline_plan, cin, cout):
    """Gathered fp32 X rows split in the forward kernel's staging give bit
    for bit the plane path's Y."""
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(3 + cin)
    x = torch.randn(N, cin, device=DEV, generator=g)
    w = torch.randn(25, cin, cout, device=DEV, generator=g) / cin ** 0.5
    r = torch.randn(cin, cout, device=DEV, generator=g) / cin ** 0.5
    wt3 = ops.slot_weight_x3(w, r, True)
    yp = ops.slot_gemm_x6(ops.split3(x), plan.src, plan.seg, wt3, True, None)
    yf = ops.slot_gemm_x6(x, plan.src, plan.seg, wt3, True, None)
    used = int(plan.seg[-1])
    assert torch.equal(yf[:used], yp[:used]), float(
        (yf[:used] - yp[:used]).abs().max())


def test_split3_reconstructs_fp32():
    ops = _backend.ops()
    x = torch.randn(1000, 64, device=DEV) * torch.logspace(
        -20, 20, 64, device=DEV)
    p = ops.split3(x).double()
    rec = p[0] + p[1] + p[2]
    rel = (rec - x.double()).abs() / x.double().abs()
    assert float(rel.max()) < 2 ** -24


def _oracle_wgrad(plan, xs, dys, S):
    """fp64 dW[s] = sum_u X_u[src]^T dY_u over slot s's compact rows."""
    slots, src = _slot_rows(plan)
    out = []
    for s, a, b in slots:
        rows = src[a:b]
        ok = rows >= 0
        acc = 0
        for x, dy in zip(xs, dys):
            acc = acc + x.double()[rows[ok]].t() @ dy.double()[a:b][ok]
        out.append(acc)
    return torch.stack(out)


@pytest.mark.parametrize('cin,cout,uses', [(128, 128, 10), (256, 256, 1),
                                           (1024, 256, 1)])
def test_x6_weight_grad_error_not_above_exact_f32(headline_plan, cin, cout,
                                                  uses):
    """psi_2's 10-use loop gradient and psi_1's two layers."""
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(11 + cin)
    P = plan.src.numel()
    used = int(plan.seg[-1])
    xs = [torch.randn(N, cin, device=DEV, generator=g) for _ in range(uses)]
    dys = []
    for _ in range(uses):
        d = torch.randn(P, cout, device=DEV, generator=g)
        d[used:] = 0
        d[plan.src.long() < 0] = 0           # padding rows carry no gradient
        dys.append(d)
    rounds = 1 if cin == 128 else (2 if cin == 256 else 6)
    w6 = ops.slot_wgrad_x6([ops.split3(x) for x in xs],
                           [ops.split3(d) for d in dys], plan.src, plan.seg,
                           rounds)
    w32 = ops.slot_wgrad_f32(xs, dys, plan.src, plan.seg, rounds)
    ref = _oracle_wgrad(plan, xs, dys, 26)
    e6 = float((w6.double() - ref).abs().max())
    e32 = float((w32.double() - ref).abs().max())
    assert e6 <= e32, (e6, e32)


def test_rowmap_planes_equal_split_of_fp32(headline_plan):
    """The row-mapped SpMM's bf16x6 plane output is exactly split3 of its
    fp32 output on every row the consumers read (rows < seg[S])."""
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.randn(N, 128, device=DEV)
    # any CSR over N*S columns works for the kernel: a random sparse A^T
    R = N * 26
    gen = torch.Generator().manual_seed(3)
    nnz = 4 * N
    rows = torch.randint(R, (nnz, ), generator=gen).sort()[0]
    rowptr = torch.zeros(R + 1, dtype=torch.long)
    rowptr[1:] = torch.bincount(rows, minlength=R).cumsum(0)
    col = torch.randint(N, (nnz, ), generator=gen).int()
    val = torch.rand(nnz, generator=gen)
    rowptr, col, val = rowptr.int().to(DEV), col.to(DEV), val.to(DEV)
    f32 = ops.slot_spmm_rowmap(rowptr, col, val, plan.cinv, g, plan.seg,
                               None, False)
    p3 = ops.slot_spmm_rowmap(rowptr, col, val, plan.cinv, g, plan.seg,
                              None, True)
    used = int(plan.seg[-1])
    assert torch.equal(p3[:, :used], ops.split3(f32)[:, :used])


def test_rowmap_entry_table_equals_ranges(headline_plan):
    """The inline (col, val) entry table gives the range walk's rows bit for
    bit, including rows with more than three entries (table fallback)."""
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.randn(N, 128, device=DEV)
    R = N * 26
    gen = torch.Generator().manual_seed(4)
    rows = torch.randint(R, (4 * N, ), generator=gen)
    heavy = plan.cinv[plan.cinv >= 0][:64].cpu().long()
    rows = torch.cat([rows, heavy.repeat_interleave(7)]).sort()[0]
    rowptr = torch.zeros(R + 1, dtype=torch.long)
    rowptr[1:] = torch.bincount(rows, minlength=R).cumsum(0)
    col = torch.randint(N, (rows.numel(), ), generator=gen).int()
    val = torch.rand(rows.numel(), generator=gen)
    rowptr, col, val = rowptr.int().to(DEV), col.to(DEV), val.to(DEV)
    rg = ops.slot_rowmap_ranges(rowptr, plan.cinv)
    ell = ops.slot_rowmap_ell(rowptr, col, val, plan.cinv)
    assert int((ell[:, 3] > 3).sum()) >= 64
    used = int(plan.seg[-1])
    for planes in (False, True):
        a = ops.slot_spmm_rowmap(rowptr, col, val, plan.cinv, g, plan.seg,
                                 rg, planes)
        b = ops.slot_spmm_rowmap(rowptr, col, val, plan.cinv, g, plan.seg,
                                 ell, planes)
        if planes:
            assert torch.equal(a[:, :used], b[:, :used])
        else:
            assert torch.equal(a[:used], b[:used])


def test_spmm_planes_feed_next_conv(monkeypatch):
    """Plane path: a non-last fp32 SplineConv's
    aggregation also writes the bf16x6 planes of its output (== split3 of
    it, bitwise); the next conv consumes them instead of splitting, with an
    identical result."""
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, DevicePairLoader, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.nn.conv import SplineConv
    assert sg.X6
    ops = _backend.ops()
    torch.manual_seed(0)
    groups = make_keypoint_datasets(graphs=8, feature_dim=128, seed=0)
    store = GraphStore(groups, DEV)
    b = next(iter(DevicePairLoader(store, batch_size=16, seed=0)))
    c0 = SplineConv(128, 128, dim=2, kernel_size=5).to(DEV)
    c1 = SplineConv(128, 128, dim=2, kernel_size=5).to(DEV)
    x = b.x_s.float()
    h = c0(x, b.edge_index_s, b.edge_attr_s, act='relu', planes_out=True)
    pl = getattr(h, '_dgmc_x6', None)
    assert pl is not None and pl[1] == h._version
    assert torch.equal(pl[0], ops.split3(h.detach().contiguous()))
    y1 = c1(h, b.edge_index_s, b.edge_attr_s, act='relu')
    y2 = c1(h.detach().clone(), b.edge_index_s, b.edge_attr_s, act='relu')
    assert torch.equal(y1, y2)
    with torch.no_grad():
        h.add_(0)             # an in-place write bumps the version: stale
    assert h._dgmc_x6[1] != h._version


@pytest.mark.parametrize('cin,cout', [(1024, 256), (256, 256), (128, 128),
                                       (300, 68)])
def test_slot_weight_x3_images_equal_split3(cin, cout):
    """Weight images of the slot GEMMs (forward: transposed, through the
    64 x 64 LDS tile kernel where in / out allow it; dX: as stored) are
    exactly the three-term split of the (transposed) fp32 weights."""
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(cin + cout)
    w = torch.randn(25, cin, cout, device=DEV, generator=g)
    r = torch.randn(cin, cout, device=DEV, generator=g)
    full = torch.cat([w, r[None]], 0)                   # [S, in, out]
    img_t = ops.slot_weight_x3(w, r, True)
    ref_t = ops.split3(full.transpose(1, 2).contiguous().view(-1, cin))
    assert torch.equal(img_t, ref_t.view(3, 26, cout, cin))
    img = ops.slot_weight_x3(w, r, False)
    ref = ops.split3(full.contiguous().view(-1, cout))
    assert torch.equal(img, ref.view(3, 26, cin, cout))


@pytest.mark.parametrize('M,parts,Nn', [(10944, 3, 128), (10944, 1, 384),
                                        (1000, 2, 64), (33, 4, 128)])
def test_dense_nt_x6_error_not_above_exact_f32(M, parts, Nn):
    """The folded projection's NT GEMM on bf16x6 (fp32 parts read in place,
    split in registers): max error vs fp64 <= the exact-f32 MFMA kernel's;
    rows past M untouched-safe (M not a multiple of the tile)."""
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(M + parts)
    ps = [torch.randn(M, 128, device=DEV, generator=g) for _ in range(parts)]
    bt = torch.randn(Nn, 128 * parts, device=DEV, generator=g) / 12
    ref = torch.cat(ps, 1).double() @ bt.double().t()
    y6 = ops.dense_nt_x6(ps, bt)
    assert y6.shape == (M, Nn)
    # pre-split B planes: the same products, bit for bit
    assert torch.equal(ops.dense_nt_x6(ps, bt, ops.split3(bt)), y6)
    e6 = float((y6.double() - ref).abs().max())
    if Nn % 64 == 0 and M >= 64:
        y32 = ops.dense_nt_f32(ps, bt)
        e32 = float((y32.double() - ref).abs().max())
        assert e6 <= e32 * 1.0001 + 1e-7, (e6, e32)
    assert e6 < 1e-5 * float(ref.abs().max())


def test_cu_reserve_keeps_results_and_hog_exits(headline_plan):
    """``set_cu_reserve``: the persistent x6 forward on CUs - 16 gives the
    same bits (each tile is computed by one workgroup either way); the
    ``cu_hog`` micro-benchmark kernel (tools/bench_cu_reserve.py) runs on
    its own, holds one CU per block and exits on its wall-clock bound."""
    N, plan = headline_plan
    ops = _backend.ops()
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(N, 256, device=DEV, generator=g)
    w = torch.randn(25, 256, 256, device=DEV, generator=g) / 16
    r = torch.randn(256, 256, device=DEV, generator=g) / 16
    wt3 = ops.slot_weight_x3(w, r, True)
    rows = plan.src.long() >= 0
    y0 = ops.slot_gemm_x6(x, plan.src, plan.seg, wt3, True, None)
    prev = _backend.set_cu_reserve(16)
    try:
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            done = ops.cu_hog(x, 8, 200.0)
        y1 = ops.slot_gemm_x6(x, plan.src, plan.seg, wt3, True, None)
        torch.cuda.synchronize()
    finally:
        _backend.set_cu_reserve(prev)
    assert torch.equal(y0[rows], y1[rows])
    assert done.tolist() == [1] * 8
