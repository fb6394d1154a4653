"""Op-level profile of the flagship training step (torch.profiler).

    python tools/profile_step.py [--steps 3] [--rows 40] [bench args...]

Prints the top ops by device time with input shapes, and writes a Chrome
trace to gpurun_out/trace_step.json.  Complements ``rocprofv3 --stats``
(kernel level) with the aten-op/shape attribution needed to map library
GEMMs back to model layers.
"""
import argparse
import os
import os.path as osp
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--steps', type=int, default=3)
    p.add_argument('--rows', type=int, default=45)
    p.add_argument('--sort', default='device_time_total')
    p.add_argument('--trace', action='store_true',
                   help='also write a Chrome trace (large)')
    args, rest = p.parse_known_args()
    os.makedirs(osp.join(ROOT, 'gpurun_out'), exist_ok=True)

    captured = {}
    real_main = bench.main

    # Run bench warmup, then profile `steps` timed steps.
    bargs = ['--steps', str(args.steps), '--warmup', '3'] + rest
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    with profile(activities=acts, record_shapes=True) as prof:
        real_main(bargs)
    captured['prof'] = prof
    print(prof.key_averages(group_by_input_shape=True).table(
        sort_by=args.sort, row_limit=args.rows, max_name_column_width=60,
        max_shapes_column_width=80))
    if args.trace:
        prof.export_chrome_trace(osp.join(ROOT, 'gpurun_out',
                                          'trace_step.json'))


if __name__ == '__main__':
    main()
