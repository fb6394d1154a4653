"""psi_1 layer-0 projection GEMM ``[M, 1024] x [1024, 6656]`` (bf16) time vs
the row count M (static-batch capacity): tile-quantisation check of the
library GEMM (hipBLASLt default heuristic, TunableOp off)."""
import torch


def t(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1000


w = torch.randn(1024, 6656, device='cuda').bfloat16()
w1 = torch.randn(256, 6656, device='cuda').bfloat16()
for M in (9984, 10240, 10304, 10496, 10752, 10944, 11008, 11264):
    x = torch.randn(M, 1024, device='cuda').bfloat16()
    x1 = torch.randn(M, 256, device='cuda').bfloat16()
    us = t(lambda: x @ w)
    us1 = t(lambda: x1 @ w1)
    print('M=%d  L0 %.1f us (%.2f PF/s, %.2f ns/row)   '
          'L1 %.1f us (%.2f ns/row)'
          % (M, us, 2 * M * 1024 * 6656 / us / 1e9, us * 1e3 / M, us1,
             us1 * 1e3 / M), flush=True)
