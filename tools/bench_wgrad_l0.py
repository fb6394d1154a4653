"""Micro-benchmark of the psi_1 layer-0 weight gradient shapes (fp32-output
GEMM variants)."""
import os.path as osp, sys, time
import torch
sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))
dev='cuda'
K, M, N = 10304, 1024, 6656
a = torch.randn(K, M, device=dev).bfloat16()
b = torch.randn(K, N, device=dev).bfloat16()
def bench(f, n=20):
    for _ in range(3): f()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/n*1e6
F32 = torch.float32
print('mm fp32 out', bench(lambda: torch.mm(a.t(), b, out_dtype=F32)))
for s in (2, 4, 8):
    k = K//s
    a3 = a[:k*s].view(s, k, M).transpose(1, 2); b3 = b[:k*s].view(s, k, N)
    print('bmm split', s,
          bench(lambda: torch.bmm(a3, b3, out_dtype=F32)))
print('mm bf16 out (untuned)', bench(lambda: torch.mm(a.t(), b)))
print('mm fp32 out b^T a',
      bench(lambda: torch.mm(b.t(), a, out_dtype=F32)))
at = a.t().contiguous(); bt = b.t().contiguous()
print('mm fp32 out contiguous A^T',
      bench(lambda: torch.mm(at, b, out_dtype=F32)))
print('mm fp32 out (B^T)^T',
      bench(lambda: torch.mm(at, bt.t(), out_dtype=F32)))
