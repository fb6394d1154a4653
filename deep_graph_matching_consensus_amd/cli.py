"""Command line entry point with presets for the BASELINE configurations.

    python -m deep_graph_matching_consensus_amd.cli train --preset pascal \
        [flags]
    python -m deep_graph_matching_consensus_amd.cli bench --preset willow \
        [flags]
    python -m deep_graph_matching_consensus_amd.cli list
    python -m deep_graph_matching_consensus_amd.cli info [--json]

``train`` runs the matching example driver (``examples/<preset>.py``, the
reference's flag names and defaults, SURVEY.md section 5 "Config / flags");
``bench`` runs ``bench.py`` (the driver's benchmark contract) with the
preset's config.  Extra flags are passed through unchanged.  ``info``
reports what a bug report needs: the device (arch, CUs), whether the native
libraries load and match their sources (the build manifest written by
``tools/build_native.py``), the registered op count and every
``DGMC_AMD_*`` switch set in the environment.
"""
import argparse
import glob
import hashlib
import json
import os
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


def _sha256(path):
    h = hashlib.sha256()
    with open(path, 'rb') as f:
        for chunk in iter(lambda: f.read(1 << 20), b''):
            h.update(chunk)
    return h.hexdigest()


def build_status(root=ROOT):
    """Compare ``build/native/manifest.json`` with the sources and libraries
    on disk: ``{'manifest': bool, 'stale_sources': [...], 'changed_libs':
    [...], 'arch': str}`` (stale = edited, added or removed since the build
    that wrote the manifest)."""
    path = osp.join(root, 'build', 'native', 'manifest.json')
    if not osp.exists(path):
        return {'manifest': False, 'stale_sources': [], 'changed_libs': [],
                'arch': None}
    with open(path) as f:
        man = json.load(f)
    srcs = {osp.relpath(p, root): p
            for p in glob.glob(osp.join(root, 'csrc', '*', '*'))
            if osp.isfile(p)}
    recorded = man.get('sources', {})
    stale = sorted(k for k in set(srcs) | set(recorded)
                   if k not in srcs or k not in recorded or
                   _sha256(srcs[k]) != recorded[k])
    changed = sorted(k for k, h in man.get('libraries', {}).items()
                     if not osp.exists(osp.join(root, k)) or
                     _sha256(osp.join(root, k)) != h)
    return {'manifest': True, 'stale_sources': stale,
            'changed_libs': changed, 'arch': man.get('arch')}


def info():
    """Environment / native-library report (a dict)."""
    import torch
    from .ops import _backend
    out = {'torch': torch.__version__,
           'hip': getattr(torch.version, 'hip', None),
           'gpu': None}
    # (device_count does not initialise the GPU; properties do, which is
    # fine here: nothing is exec'd afterwards)
    if torch.cuda.device_count() > 0 and torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        out['gpu'] = {'name': p.name,
                      'arch': getattr(p, 'gcnArchName', None),
                      'cus': p.multi_processor_count,
                      'memory_gib': round(p.total_memory / 2 ** 30, 1),
                      'count': torch.cuda.device_count()}
    out['libraries'] = {
        kind: {'path': _backend.library_path(kind),
               'loaded': bool(_backend.hip_available() if kind == 'hip'
                              else _backend.host_available())}
        for kind in ('hip', 'host')}
    names = getattr(torch._C, '_dispatch_get_all_op_names', lambda: [])()
    out['ops'] = len([n for n in names if n.startswith('dgmc_amd::')])
    out['build'] = build_status()
    out['diagnostic_library'] = _backend.diag_requested()
    out['switches'] = {k: v for k, v in sorted(os.environ.items())
                       if k.startswith('DGMC_AMD_')}
    return out


def main(argv=None):
    p = argparse.ArgumentParser(prog='deep_graph_matching_consensus_amd')
    p.add_argument('command', choices=['train', 'bench', 'list', 'info'])
    p.add_argument('--preset', default='pascal', choices=sorted(PRESETS))
    p.add_argument('--json', action='store_true', help='info: one JSON line')
    args, rest = p.parse_known_args(argv)
    if args.command == 'info':
        rep = info()
        if args.json:
            print(json.dumps(rep, sort_keys=True))
        else:
            for k, v in rep.items():
                print('%-20s %s' % (k, v))
        return 0 if rep['libraries']['host']['loaded'] else 1
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
