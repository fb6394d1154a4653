"""Chunked NT GEMM (csrc/hip/gemm_f32.hip) on the DBP15K node-GEMM shapes:
time per tile configuration (forced through DGMC_GEMM_F32_CFG = 1 / 2 / 3 =
128x128 / 128x64 / 64x64, diagnostic library only) and arithmetic (exact
f32 / bf16x6), next to the host cost model's pick (cfg 0).

    python tools/build_native.py --diag
    DGMC_AMD_DIAG=1 python tools/micro/bench_nt_f32_cfg.py
"""
import json
import os
import os.path as osp
import subprocess
import sys

SHAPES = {'map_300x768': (38960, [300], 768),
          'map_256x768': (38960, [256], 768),
          'final_1068x256': (38960, [300, 256, 256, 256], 256)}


def child(cfg):
    import torch
    sys.path.insert(0, osp.dirname(osp.dirname(osp.dirname(
        osp.abspath(__file__)))))
    from deep_graph_matching_consensus_amd.ops import _backend
    ops = _backend.ops()
    out = {}
    for name, (M, widths, Nn) in SHAPES.items():
        parts = [torch.randn(M, w, device='cuda') for w in widths]
        bt = torch.randn(Nn, sum(widths), device='cuda')
        for x6 in (False, True):
            for _ in range(3):
                ops.gemm_nt_f32(parts, bt, None, False, None, x6)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(True), torch.cuda.Event(True)
            a.record()
            for _ in range(20):
                ops.gemm_nt_f32(parts, bt, None, False, None, x6)
            b.record()
            torch.cuda.synchronize()
            out['%s_%s' % (name, 'x6' if x6 else 'f32')] = round(
                a.elapsed_time(b) * 50, 1)
    print(json.dumps({'cfg': cfg, 'us': out}), flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1:
        child(int(sys.argv[1]))
    else:
        for cfg in (0, 1, 2, 3):
            env = dict(os.environ, DGMC_GEMM_F32_CFG=str(cfg))
            subprocess.run([sys.executable, __file__, str(cfg)], env=env,
                           check=True)
