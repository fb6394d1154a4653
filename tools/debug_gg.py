"""Debug: fused gather_gemm backward vs unfused (dY via SpMM, dX via GEMM)."""
import torch
from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops.sparse import SparseOperator

assert _backend.hip_available()
torch.manual_seed(0)
dev = 'cuda'
for (K, C, S) in [(128, 128, 26), (32, 32, 3)]:
    N, E = 300, 2000
    row = torch.randint(N, (E,), device=dev)
    j = torch.randint(N, (E,), device=dev)
    k = torch.randint(S - 1, (E,), device=dev)
    val = torch.rand(E, device=dev)
    ar = torch.arange(N, device=dev)
    op = SparseOperator.from_coo(torch.cat([row, ar]),
                                 torch.cat([j * S + k, ar * S + S - 1]),
                                 torch.cat([val, torch.ones(N, device=dev)]),
                                 N, N * S)
    opt = op.t()
    g = torch.randn(N, C, device=dev).bfloat16()
    w_lp = (torch.randn(K, S * C, device=dev) / K ** .5).bfloat16()
    dy_ref = (opt.to_dense() @ g.float())               # [N*S, C]
    gx_ref = dy_ref.view(N, S * C) @ w_lp.float().t()   # [N, K]
    dy = torch.empty(N * S, C, device=dev, dtype=torch.bfloat16)
    gx = _backend.ops().gather_gemm(g, opt.rowptr, opt.col, opt.val, w_lp, C,
                                    S * C, S, K, None, False, g.dtype, dy)
    torch.cuda.synchronize()
    e_dy = (dy.float() - dy_ref).abs()
    e_gx = (gx.float() - gx_ref).abs()
    print('K,C,S', K, C, S, 'dy err', e_dy.max().item(), 'dy scale',
          dy_ref.abs().max().item(), 'gx err', e_gx.max().item(), 'gx scale',
          gx_ref.abs().max().item())
    bad = (e_gx > 0.05 * gx_ref.abs().max()).nonzero()
    print(' bad gx entries', bad.shape[0], bad[:10].tolist())
    # forward-style call on the same data with explicit transposed weight
    wt = w_lp.t().contiguous()  # [S*C, K]
    x = torch.randn(N, K, device=dev).bfloat16()
    sc = op.slot_csr(S)
    out = _backend.ops().gather_gemm(x, sc.rowptr, sc.col, sc.val, wt, C * K,
                                     K, S, C, None, False, x.dtype, None)
    out_ref = op.to_dense() @ (x.float() @ w_lp.float()).view(-1, C)
    print(' fwd err', (out.float() - out_ref).abs().max().item(),
          out_ref.abs().max().item())
