"""Top-k filter-pass ablation on the DBP15K zh_en shape (19388 x 19572,
C = 256): times mode 2 (default exact: filter + re-score), mode 0 (filter
only, k list) and the filter with a 16-candidate list; run it under
DGMC_TOPK_DEBUG=1 (selection skipped) / 2 (MFMA skipped) to split the
filter kernel's time.  The knob exists only in the diagnostic library:

    python tools/build_native.py --diag
    DGMC_AMD_DIAG=1 DGMC_TOPK_DEBUG=1 python tools/micro/topk_ablation.py
"""
import json
import os
import os.path as osp
import sys

import torch

sys.path.insert(0, osp.dirname(osp.dirname(osp.dirname(osp.abspath(
    __file__)))))
from deep_graph_matching_consensus_amd.ops import _backend  # noqa: E402

ops = _backend.ops()
torch.manual_seed(0)
hs = torch.randn(1, 19388, 256, device='cuda')
ht = torch.randn(1, 19572, 256, device='cuda')
out = {'debug': os.environ.get('DGMC_TOPK_DEBUG', '0'),
       'diag_lib': _backend.diag_requested()}
for name, k, mode in (('exact_k10', 10, 2), ('x3_k10', 10, 0),
                      ('x3_k16', 16, 0)):
    for _ in range(2):
        ops.topk_dot(hs, ht, k, mode)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(5):
        ops.topk_dot(hs, ht, k, mode)
    b.record()
    torch.cuda.synchronize()
    out[name + '_ms'] = round(a.elapsed_time(b) / 5, 3)
print(json.dumps(out), flush=True)
