"""hipBLASLt layout variants for psi_2's skinny GEMMs (K=128 forward,
K=3328 input-gradient).  Times each formulation of the same product.

    python tools/gemm_layouts.py [--nodes 9216]
"""
import argparse

import torch


def timeit(fn, iters=50, warmup=10):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--nodes', type=int, default=9216)
    args = p.parse_args()
    N, K, S, C = args.nodes, 128, 26, 128
    dev, dt = 'cuda', torch.bfloat16
    x = torch.randn(N, K, device=dev, dtype=dt)
    w = torch.randn(K, S * C, device=dev, dtype=dt)       # [in, S*out]
    wt = w.t().contiguous()                               # [S*out, in]
    out = torch.empty(N, S * C, device=dev, dtype=dt)
    outT = torch.empty(S * C, N, device=dev, dtype=dt)
    gb = 2 * N * S * C * 2 / 1e9   # GB written
    res = {}
    res['fwd x@w (NN)'] = timeit(lambda: torch.mm(x, w, out=out))
    res['fwd x@wt.t() (NT)'] = timeit(lambda: torch.mm(x, wt.t(), out=out))
    res['fwd (wt@x.t()).T'] = timeit(lambda: torch.mm(wt, x.t(), out=outT))
    res['fwd bmm S x [N,128]x[128,128]'] = timeit(
        lambda: torch.bmm(x.expand(S, N, K), w.view(K, S, C).transpose(0, 1)))
    for k, v in res.items():
        print('%-36s %7.1f us  %5.2f TB/s(out)' % (k, v, gb / 2 / v * 1e3))
    dY = torch.randn(N, S * C, device=dev, dtype=dt)
    dx = torch.empty(N, K, device=dev, dtype=dt)
    res = {}
    res['dX dY@w.t() (NT)'] = timeit(lambda: torch.mm(dY, w.t(), out=dx))
    res['dX dY@wt (NN)'] = timeit(lambda: torch.mm(dY, wt, out=dx))
    dxT = torch.empty(K, N, device=dev, dtype=dt)
    res['dX (w@dY.t()).T'] = timeit(lambda: torch.mm(w, dY.t(), out=dxT))
    res['dX fp32 out'] = timeit(lambda: torch.mm(dY, wt,
                                                 out_dtype=torch.float32))
    for k, v in res.items():
        print('%-36s %7.1f us  %5.2f TB/s(in)' % (k, v, gb / 2 / v * 1e3))


if __name__ == '__main__':
    main()
