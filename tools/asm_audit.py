"""Static audit of the gfx950 code objects of the in-tree HIP kernels.

Compiles every ``csrc/hip/*.hip`` (or the ones named) to device assembly
with the build's flags and reports, per kernel: VGPRs / AGPRs, SGPRs,
scratch (private segment) bytes, static LDS, the number of vector memory
loads, how many of them are *serialised* (the next vector-memory wait after
the load is ``vmcnt(0)`` with no other load issued in between - one full
memory round trip per load), and scratch loads / stores.

Serialised loads and scratch are the two code-generation traps that made
early versions of the gather kernels latency bound: ``cond ? load : 0``
compiled to a divergent branch whose other side overwrote the load's
registers (forcing a wait per load), and a not-fully-unrolled loop indexed
a register array dynamically (spilled to scratch).

    python tools/asm_audit.py [files...] [--kernel SUBSTR] [--json out]
"""
import argparse
import glob
import json
import os
import os.path as osp
import re
import subprocess
import sys
import tempfile

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')


def _flags():
    import torch.utils.cpp_extension as ce
    incs = ' '.join('-I' + p for p in ce.include_paths())
    return ('-O3 -std=c++17 -fPIC -D_GLIBCXX_USE_CXX11_ABI=1 -DUSE_ROCM=1 '
            '-D__HIP_PLATFORM_AMD__=1 -munsafe-fp-atomics -I{} {}'.format(
                osp.join(ROOT, 'csrc', 'hip'), incs)).split()


def compile_asm(src, out):
    cmd = [osp.join(ROCM, 'bin', 'hipcc'), '--offload-arch=gfx950',
           '--cuda-device-only', '-S', '-o', out, '-x', 'hip', src] + _flags()
    subprocess.run(cmd, check=True)


_META = re.compile(r'^\s+\.(name|vgpr_count|agpr_count|sgpr_count|'
                   r'private_segment_fixed_size|group_segment_fixed_size):'
                   r'\s+(\S+)')


def parse(asm_text):
    """{kernel: stats} from one assembly file."""
    bodies = {}
    cur = None
    for line in asm_text.splitlines():
        m = re.match(r'^(_Z\S+):\s*(;.*)?$', line)
        if m:
            cur = m.group(1)
            bodies[cur] = []
            continue
        if cur is not None:
            # (a kernel may hold several s_endpgm: early exits)
            if line.startswith('.Lfunc_end'):
                cur = None
                continue
            bodies[cur].append(line.strip())
    meta, rec = {}, {}
    in_kernels = False
    for line in asm_text.splitlines():
        if line.strip() == 'amdhsa.kernels:':
            in_kernels = True
        if not in_kernels:
            continue
        m = _META.match(line)
        if m:
            k, v = m.group(1), m.group(2)
            if k == 'name':
                if rec.get('name'):
                    meta[rec['name']] = rec
                rec = {'name': v}
            else:
                rec[k] = int(v)
    if rec.get('name'):
        meta[rec['name']] = rec
    out = {}
    for name, body in bodies.items():
        loads = serial = 0
        pending = 0          # loads issued since the last vmcnt wait
        last_single = False
        for ins in body:
            if re.match(r'(global|buffer)_load', ins):
                loads += 1
                pending += 1
                last_single = pending == 1
            elif re.match(r's_waitcnt\s.*vmcnt\((\d+)\)', ins):
                n = int(re.search(r'vmcnt\((\d+)\)', ins).group(1))
                if n == 0 and pending == 1 and last_single:
                    serial += 1
                if n == 0:
                    pending = 0
        m = meta.get(name, {})
        out[name] = {
            'vgpr': m.get('vgpr_count'), 'agpr': m.get('agpr_count'),
            'sgpr': m.get('sgpr_count'),
            'scratch': m.get('private_segment_fixed_size'),
            'lds_static': m.get('group_segment_fixed_size'),
            'vmem_loads': loads, 'serialised_loads': serial,
            'scratch_ops': sum(1 for i in body if i.startswith('scratch_')),
            # flat_* memory ops: usually LDS reached through a generic
            # pointer (no address_space(3)) - slower, and every wait on
            # them covers both the vector-memory and the LDS counters
            'flat_ops': sum(1 for i in body
                            if re.match(r'flat_(load|store|atomic)', i)),
            'instructions': len([i for i in body if i and
                                 not i.startswith(('.', ';'))]),
        }
    return out


def _demangle(names):
    try:
        r = subprocess.run(['c++filt'], input='\n'.join(names),
                           capture_output=True, text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def main():
    p = argparse.ArgumentParser()
    p.add_argument('files', nargs='*')
    p.add_argument('--kernel', default=None)
    p.add_argument('--json', default=None)
    args = p.parse_args()
    files = args.files or sorted(glob.glob(osp.join(ROOT, 'csrc', 'hip',
                                                    '*.hip')))
    report = {}
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            out = osp.join(td, osp.basename(f) + '.s')
            compile_asm(f, out)
            with open(out) as fh:
                stats = parse(fh.read())
            for k, v in stats.items():
                v['file'] = osp.basename(f)
                report[k] = v
    names = sorted(report)
    if args.kernel:
        names = [n for n in names if args.kernel in n]
    pretty = _demangle(names)
    hdr = '{:<9} {:>4} {:>4} {:>7} {:>6} {:>6} {:>5}  {}'.format(
        'file', 'vgpr', 'sgpr', 'scratch', 'loads', 'serial', 'flat',
        'kernel')
    print(hdr)
    for n, pn in zip(names, pretty):
        r = report[n]
        short = re.sub(r'\(.*', '', pn.replace('(anonymous namespace)::', '')
                       ).replace('dgmc::', '')
        print('{:<9} {:>4} {:>4} {:>7} {:>6} {:>6} {:>5}  {}'.format(
            r['file'][:9], r['vgpr'] or 0, r['sgpr'] or 0, r['scratch'] or 0,
            r['vmem_loads'], r['serialised_loads'], r['flat_ops'],
            short[:90]))
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(report, f, indent=1, sort_keys=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
