"""Command line entry point with presets for the BASELINE configurations.

    python -m deep_graph_matching_consensus_amd.cli train --preset pascal \
        [flags]
    python -m deep_graph_matching_consensus_amd.cli bench --preset willow \
        [flags]
    python -m deep_graph_matching_consensus_amd.cli list

``train`` runs the matching example driver (``examples/<preset>.py``, the
reference's flag names and defaults, SURVEY.md section 5 "Config / flags");
``bench`` runs ``bench.py`` (the driver's benchmark contract) with the
preset's config.  Extra flags are passed through unchanged.
"""
import argparse
import os.path as osp
import runpy
import sys

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))

# preset -> (example script, bench --config or None, description)
PRESETS = {
    'er': ('er_gin.py', None,
           'BASELINE 1: 20-node Erdos-Renyi pair, GIN psi, L=10 (CPU ok)'),
    'willow': ('willow.py', 'willow',
               'BASELINE 2: WILLOW-shaped keypoints, SplineCNN, batch 512'),
    'pascal': ('pascal.py', 'pascal',
               'BASELINE 3/5: PascalVOC-shaped keypoints, SplineCNN, dense'),
    'pascal_pf': ('pascal_pf.py', None,
                  'PascalPF synthetic random-graph training'),
    'dbp15k': ('dbp15k.py', 'dbp15k',
               'BASELINE 4: DBP15K-shaped KG alignment, RelCNN, top-k 10'),
}


def _run_script(path, argv):
    old = sys.argv
    sys.argv = [path] + list(argv)
    try:
        runpy.run_path(path, run_name='__main__')
    finally:
        sys.argv = old


def main(argv=None):
    p = argparse.ArgumentParser(prog='deep_graph_matching_consensus_amd')
    p.add_argument('command', choices=['train', 'bench', 'list'])
    p.add_argument('--preset', default='pascal', choices=sorted(PRESETS))
    args, rest = p.parse_known_args(argv)
    if args.command == 'list':
        for name, (script, cfg, doc) in sorted(PRESETS.items()):
            print('%-10s %-14s bench=%-7s %s' % (name, script, cfg, doc))
        return 0
    script, cfg, _ = PRESETS[args.preset]
    if args.command == 'train':
        _run_script(osp.join(ROOT, 'examples', script), rest)
        return 0
    if cfg is None:
        raise SystemExit('preset %r has no benchmark config' % args.preset)
    _run_script(osp.join(ROOT, 'bench.py'), ['--config', cfg] + rest)
    return 0


if __name__ == '__main__':
    sys.exit(main())
