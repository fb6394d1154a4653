"""Micro-benchmark of the fused gather-MFMA kernel (dgmc_amd::gather_gemm).

Times the kernel for psi_2-like shapes while varying the slot count S and
the locality of the sources, against the unfused GEMM + SpMM pair.
"""
import torch
from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops.sparse import SparseOperator

assert _backend.hip_available()
dev = 'cuda'
ops = _backend.ops()


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def make_op(N, S, deg, local):
    E = N * deg
    row = torch.arange(N, device=dev).repeat_interleave(deg)
    if local:
        j = (row + torch.randint(-10, 11, (E,), device=dev)).clamp(0, N - 1)
    else:
        j = torch.randint(N, (E,), device=dev)
    # 4 basis slots per edge (SplineConv degree 1, dim 2)
    k0 = torch.randint(S - 1, (E,), device=dev)
    rows, cols, vals = [], [], []
    for d in range(4):
        rows.append(row)
        cols.append(j * S + (k0 + d) % (S - 1))
        vals.append(torch.rand(E, device=dev) / deg)
    ar = torch.arange(N, device=dev)
    rows.append(ar)
    cols.append(ar * S + S - 1)
    vals.append(torch.ones(N, device=dev))
    return SparseOperator.from_coo(torch.cat(rows), torch.cat(cols),
                                   torch.cat(vals), N, N * S)


N, K, C = 9216, 128, 128
for S in (2, 8, 26):
    for local in (True, False):
        op = make_op(N, S, 5, local)
        sc = op.slot_csr(S)
        x = torch.randn(N, K, device=dev).bfloat16()
        w = (torch.randn(K, S * C, device=dev) / K ** .5).bfloat16()
        wt = w.t().contiguous()
        t_f = timeit(lambda: ops.gather_gemm(x, sc.rowptr, sc.col, sc.val, wt,
                                             C * K, K, S, C, None, True,
                                             torch.bfloat16, None))
        t_g = timeit(lambda: x @ w)
        y = (x @ w).view(-1, C)
        t_s = timeit(lambda: ops.spmm_csr(op.rowptr, op.col, op.val, y, None,
                                          None, None, True, torch.bfloat16))
        print('S=%2d local=%d fused %.1f us | gemm %.1f + spmm %.1f us | '
              'nnz %d' % (S, local, t_f, t_g, t_s, op.nnz), flush=True)

# Stamps (DGMC_GG_DEBUG & 4): wall_clock64 runs at 100 MHz on gfx950.
import os
if int(os.environ.get('DGMC_GG_DEBUG', '0')) & 4:
    for S in (2, 26):
        op = make_op(N, S, 5, True)
        sc = op.slot_csr(S)
        x = torch.randn(N, K, device=dev).bfloat16()
        w = (torch.randn(K, S * C, device=dev) / K ** .5).bfloat16()
        wt = w.t().contiguous()
        for _ in range(3):
            ops.gather_gemm(x, sc.rowptr, sc.col, sc.val, wt, C * K, K, S, C,
                            None, True, torch.bfloat16, None)
        torch.cuda.synchronize()
        st = ops.gather_gemm_stamps()[:4].tolist()
        print('S=%d stamps (us from start):' % S,
              [(v - st[0]) / 100.0 for v in st])
