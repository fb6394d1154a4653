"""Micro-benchmark of the encoder GEMM shapes (hipBLASLt via torch) and
split-K alternatives for the small-output / long-K backward GEMMs.

    python tools/gemm_bench.py [--nodes 9216]
"""
import argparse

import torch


def timeit(fn, iters=50, warmup=10):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(True), torch.cuda.Event(True)
    start.record()
    for _ in range(iters):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / iters * 1000.0  # us


def splitk(a_t, b, s):
    """a_t: [K, M] (i.e. A^T stored K-major), b: [K, N] -> A @ B, split K."""
    K, M = a_t.shape
    N = b.shape[1]
    k = K // s
    a3 = a_t[:k * s].view(s, k, M).transpose(1, 2)
    b3 = b[:k * s].view(s, k, N)
    return torch.bmm(a3, b3, out_dtype=torch.float32).sum(0)


def splitk_dx(y, w, s):
    """y [N, C], w [cin, C] -> y @ w^T with C split into s batches."""
    N, C = y.shape
    cin = w.shape[0]
    k = C // s
    y3 = y[:, :k * s].reshape(N, s, k).transpose(0, 1)
    w3 = w[:, :k * s].reshape(cin, s, k).permute(1, 2, 0)
    return torch.bmm(y3, w3, out_dtype=torch.float32).sum(0)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--nodes', type=int, default=9216)
    args = p.parse_args()
    N = args.nodes
    dt = torch.bfloat16
    dev = 'cuda'
    rows = []

    def report(name, us, flop):
        rows.append((name, us, flop / us / 1e6))
        print('{:58s} {:9.1f} us {:8.1f} TF/s'.format(name, us,
                                                     flop / us / 1e6),
              flush=True)

    for cin, cols in [(128, 3328), (256, 6656), (1024, 6656), (384, 128)]:
        x = torch.randn(N, cin, device=dev, dtype=dt)
        w = torch.randn(cin, cols, device=dev, dtype=dt)
        y = torch.randn(N, cols, device=dev, dtype=dt)
        flop = 2.0 * N * cin * cols
        report('fwd  [{},{}]@[{},{}]'.format(N, cin, cin, cols),
               timeit(lambda: x @ w), flop)
        report('dX   [{},{}]@[{},{}]^T'.format(N, cols, cin, cols),
               timeit(lambda: y @ w.t()), flop)
        report('dW   [{},{}]^T@[{},{}]'.format(N, cin, N, cols),
               timeit(lambda: x.t() @ y), flop)
        report('dW   fp32-out mm', timeit(
            lambda: torch.mm(x.t(), y, out_dtype=torch.float32)), flop)
        for s in (4, 8, 16):
            report('dW   split-K bmm s={}'.format(s),
                   timeit(lambda: splitk(x, y, s)), flop)
        for s in (4, 8):
            report('dX   split-K bmm s={}'.format(s),
                   timeit(lambda: splitk_dx(y, w, s)), flop)


if __name__ == '__main__':
    main()
