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
    args, _ = p.parse_known_args()
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


if __name__ == '__main__' and '--custom' not in __import__('sys').argv:
    main()


def custom():
    """dgmc_amd::gemm_abt vs hipBLASLt on the same shapes (+ max error)."""
    import os.path as osp
    import sys
    sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))
    from deep_graph_matching_consensus_amd.ops import _backend
    assert _backend.hip_available()
    ops = _backend.ops()
    N, K, S, C = 9216, 128, 26, 128
    dev, dt = 'cuda', torch.bfloat16
    x = torch.randn(N, K, device=dev, dtype=dt)
    w = torch.randn(K, S * C, device=dev, dtype=dt) / K ** .5
    wt = w.t().contiguous()
    ref = x @ w
    y = ops.gemm_abt(x, wt)
    print('custom fwd  err %.3e' % (y.float() - ref.float()).abs().max())
    t = timeit(lambda: ops.gemm_abt(x, wt))
    print('custom fwd  %7.1f us  %5.2f TB/s(out)'
          % (t, N * S * C * 2 / t / 1e6))
    dY = torch.randn(N, S * C, device=dev, dtype=dt)
    ref = dY @ w.t()
    dx = ops.gemm_abt(dY, w)
    print('custom dX   err %.3e (ref max %.2f)' % (
        (dx.float() - ref.float()).abs().max(), ref.float().abs().max()))
    t = timeit(lambda: ops.gemm_abt(dY, w))
    print('custom dX   %7.1f us  %5.2f TB/s(in)'
          % (t, N * S * C * 2 / t / 1e6))
    acc = ref.clone()
    ops.gemm_abt(dY, w, acc, True)
    print('custom dX accumulate err %.3e' % (acc.float() - 2 * ref.float())
          .abs().max())


if __name__ == '__main__' and '--custom' in __import__('sys').argv:
    custom()
