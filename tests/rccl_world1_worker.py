"""World-size-1 RCCL rehearsal of the captured data-parallel step.

Run as a script (by ``tests/test_rccl_step.py`` and under ``rocprofv3`` for
``profiles/``)::

    python tests/rccl_world1_worker.py [--steps 6] [--json out.json]

1. trains ``--steps`` graph-mode steps with NO process group (the
   single-process path: one pack kernel + flagged HIP Adam);
2. initialises an RCCL (``nccl``) process group of ONE rank and trains the
   same model from the same seeds in graph mode.  ``PairTrainer`` now takes
   the real data-parallel path (``reducer.in_step``): AccumulateGrad steals
   the gradients, the hook completing each bucket packs it and launches
   ``dist.all_reduce(AVG, async_op=True)``, ``finish()`` waits on the works,
   then the non-finite check and Adam - all captured in the step's
   hipGraph and replayed;
3. checks the parameters are bit-identical (AVG over one rank is exact).

The headline model (``/root/reference/examples/pascal.py:46-52``) with
``bucket_bytes`` = 4 MiB, so the 36 MiB gradient is cut into many buckets
(= many captured all-reduces).
"""
import argparse
import json
import os
import os.path as osp
import socket
import sys

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def train(steps, batch_size, seed=0):
    from deep_graph_matching_consensus_amd.datasets import (
        GraphStore, make_keypoint_datasets)
    from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
    from deep_graph_matching_consensus_amd.train import PairTrainer
    device = torch.device('cuda', 0)
    torch.manual_seed(seed)
    groups = make_keypoint_datasets(graphs=16, seed=seed)
    store = GraphStore(groups, device)
    model = DGMC(SplineCNN(1024, 256, 2, 2, cat=False, dropout=0.5),
                 SplineCNN(128, 128, 2, 2, cat=True, dropout=0.0),
                 num_steps=10).to(device)
    trainer = PairTrainer(model, store, batch_size, mode='graph', bf16=False,
                          seed=seed, buckets=False, bucket_bytes=4 << 20)
    for _ in range(steps):
        trainer.step()
    torch.cuda.synchronize()
    params = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    info = {'in_step': bool(trainer.reducer.in_step),
            'distributed': bool(trainer.reducer.distributed),
            'buckets': len(trainer.reducer.buckets),
            'stats': trainer.read_stats()}
    return params.cpu(), info


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--steps', type=int, default=6)
    p.add_argument('--batch-size', type=int, default=128)
    p.add_argument('--json', default=None)
    args = p.parse_args(argv)
    import torch.distributed as dist

    ref, ref_info = train(args.steps, args.batch_size)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()),
                      RANK='0', WORLD_SIZE='1', LOCAL_RANK='0')
    os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '1')
    dist.init_process_group('nccl', rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))
    assert dist.get_backend() == 'nccl'
    got, info = train(args.steps, args.batch_size)
    dist.destroy_process_group()
    diff = (got - ref).abs().max().item()
    out = {'steps': args.steps, 'equal': bool(torch.equal(got, ref)),
           'max_abs_diff': diff, 'rccl': info, 'single': ref_info,
           'numel': got.numel()}
    line = json.dumps(out)
    print(line, flush=True)
    if args.json:
        with open(args.json, 'w') as f:
            f.write(line + '\n')
    ok = out['equal'] and info['in_step'] and info['distributed']
    return 0 if ok else 1


if __name__ == '__main__':
    sys.exit(main())
