"""Time dgmc_amd::topk_dot (exact-f32 and split-bf16 kernels) on DBP15K-sized
inputs (the kernels' ``dbg`` ablation argument is a diagnostic-build
knob, fixed to 0 in production launches)."""
import sys
import os.path as osp
import torch
sys.path.insert(0, osp.dirname(osp.dirname(osp.abspath(__file__))))
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402

assert _backend.hip_available()
ops = _backend.ops()
shapes = [(15000, 15000, 256, 10), (19388, 19572, 256, 10),
          (15000, 15000, 256, 20), (4096, 4096, 64, 10), (1, 2, 2, 2)]
for (Ns, Nt, C, k) in shapes[:-1]:
    hs = torch.randn(1, Ns, C, device='cuda')
    ht = torch.randn(1, Nt, C, device='cuda')
    res = {}
    for exact in (True, False):
        for _ in range(2):
            ops.topk_dot(hs, ht, k, exact)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        for _ in range(5):
            idx = ops.topk_dot(hs, ht, k, exact)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 5
        res[exact] = idx
        print('Ns=%d Nt=%d C=%d k=%d exact=%d: %.3f ms  %.1f TF/s' % (
            Ns, Nt, C, k, exact, ms, 2 * Ns * Nt * C / ms / 1e9), flush=True)
    same = (res[True] == res[False]).float().mean().item()
    print('   agreement exact vs bf16x3: %.5f' % same, flush=True)
