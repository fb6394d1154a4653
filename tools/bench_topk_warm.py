"""Warm vs cold start of the exact top-k filter (csrc/hip/topk.hip::
topk_warm_kernel) on the DBP15K shape: the op time with no state, with the
state of the same embeddings, and with the state of embeddings perturbed
by relative noise (a stand-in for consecutive training steps).

    python tools/bench_topk_warm.py [--reps 5] [--json out.json]
"""
import argparse
import json
import os.path as osp
import sys

sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))

import torch  # noqa: E402

from deep_graph_matching_consensus_amd.ops import sparse_corr  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps, 3)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--reps', type=int, default=5)
    p.add_argument('--json', default=None)
    args = p.parse_args()
    g = torch.Generator(device='cuda').manual_seed(0)
    Ns, Nt, C = 19388, 19572, 256
    h_s = torch.randn(1, Ns, C, device='cuda', generator=g)
    h_t = torch.randn(1, Nt, C, device='cuda', generator=g)
    out = {'cold_ms': timed(lambda: sparse_corr.top_k(h_s, h_t, 10),
                            args.reps)}
    for noise in (0.0, 0.05, 0.3, 1.0):
        st = torch.full((1, Ns, 32), -1, dtype=torch.long, device='cuda')
        hs0 = h_s + noise * torch.randn(h_s.shape, device='cuda',
                                        generator=g)
        ht0 = h_t + noise * torch.randn(h_t.shape, device='cuda',
                                        generator=g)
        sparse_corr.top_k(hs0, ht0, 10, warm=st)        # the "last step"
        saved = st.clone()

        def run():
            st.copy_(saved)
            return sparse_corr.top_k(h_s, h_t, 10, warm=st)
        out['warm_noise_{}_ms'.format(noise)] = timed(run, args.reps)
    print(json.dumps(out), flush=True)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
