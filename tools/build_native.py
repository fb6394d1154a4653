"""Direct hipcc / g++ build of the in-tree native libraries (via ninja).

torch's ``CUDAExtension`` runs a hipify pass over the sources on ROCm; our
kernels are written for CDNA4 directly, so we drive ``hipcc`` ourselves:

    python tools/build_native.py            # incremental (ninja)
    python tools/build_native.py --clean

Outputs (loaded with ``torch.ops.load_library``):
  deep_graph_matching_consensus_amd/_C_hip.so   gfx950 kernels + op registry
  deep_graph_matching_consensus_amd/_C_host.so  host C++ runtime (OpenMP)

``--diag`` builds ``_C_hip_diag.so`` instead (``-DDGMC_DIAG``: the kernel
ablation / margin / split knobs of ``csrc/hip/common.h::diag_env_int`` read
the environment); it is loaded only when ``DGMC_AMD_DIAG=1``.  The
production library ignores those variables.
"""
import argparse
import glob
import os
import os.path as osp
import shutil
import subprocess
import sys

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
PKG = osp.join(ROOT, 'deep_graph_matching_consensus_amd')
BUILD = osp.join(ROOT, 'build', 'native')
ARCH = os.environ.get('DGMC_AMD_ARCH', 'gfx950')
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type='cuda')
    lib = osp.join(osp.dirname(torch.__file__), 'lib')
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _ninja_escape(p):
    return p.replace('$', '$$').replace(' ', '$ ').replace(':', '$:')


def write_ninja(debug=False, diag=False):
    inc, lib, abi = _torch_paths()
    build_dir = BUILD + '_diag' if diag else BUILD
    os.makedirs(build_dir, exist_ok=True)
    incs = ' '.join('-isystem ' + p for p in inc)
    common = ('-fPIC -std=c++17 -D_GLIBCXX_USE_CXX11_ABI={} '
              '-D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 {}').format(abi, incs)
    opt = '-O0 -g' if debug else '-O3'
    hipcc = osp.join(ROCM, 'bin', 'hipcc')
    hip_flags = ('{} {} -x hip --offload-arch={} -fno-gpu-rdc '
                 '-munsafe-fp-atomics -I{}{}'.format(
                     opt, common, ARCH, osp.join(ROOT, 'csrc', 'hip'),
                     ' -DDGMC_DIAG=1' if diag else ''))
    host_flags = '{} {} -fopenmp -Wall -Wno-unused-function -I{}'.format(
        opt, common, osp.join(ROOT, 'csrc', 'host'))
    libs_hip = ('-L{0} -Wl,-rpath,{0} -lc10 -ltorch -ltorch_cpu -lc10_hip '
                '-ltorch_hip -L{1}/lib -lamdhip64').format(lib, ROCM)
    libs_host = '-L{0} -Wl,-rpath,{0} -lc10 -ltorch -ltorch_cpu -fopenmp'\
        .format(lib)

    lines = [
        'ninja_required_version = 1.3',
        'rule hipcc',
        '  command = {} {} -MD -MF $out.d -c $in -o $out'.format(hipcc,
                                                                 hip_flags),
        '  depfile = $out.d', '  deps = gcc',
        '  description = HIPCC $in',
        'rule hostcxx',
        '  command = g++ {} -MD -MF $out.d -c $in -o $out'.format(host_flags),
        '  depfile = $out.d', '  deps = gcc',
        '  description = CXX $in',
        # (linked to a temporary name and renamed: a snapshot of the tree
        # taken during a build never sees a half-written library)
        'rule link_hip',
        '  command = {} -shared -fPIC --offload-arch={} -fno-gpu-rdc $in -o '
        '$out.tmp {} && mv -f $out.tmp $out'.format(hipcc, ARCH, libs_hip),
        '  description = LINK $out',
        'rule link_host',
        '  command = g++ -shared -fPIC $in -o $out.tmp {} && mv -f $out.tmp '
        '$out'.format(libs_host),
        '  description = LINK $out',
    ]
    targets = []
    hip_src = sorted(glob.glob(osp.join(ROOT, 'csrc', 'hip', '*.hip')) +
                     glob.glob(osp.join(ROOT, 'csrc', 'hip', '*.cpp')))
    objs = []
    for src in hip_src:
        obj = osp.join(build_dir, 'hip', osp.basename(src) + '.o')
        lines.append('build {}: hipcc {}'.format(_ninja_escape(obj),
                                                 _ninja_escape(src)))
        objs.append(obj)
    out = osp.join(PKG, '_C_hip_diag.so' if diag else '_C_hip.so')
    lines.append('build {}: link_hip {}'.format(
        _ninja_escape(out), ' '.join(_ninja_escape(o) for o in objs)))
    targets.append(out)

    host_src = sorted(glob.glob(osp.join(ROOT, 'csrc', 'host', '*.cpp')))
    if host_src and not diag:
        objs = []
        for src in host_src:
            obj = osp.join(BUILD, 'host', osp.basename(src) + '.o')
            lines.append('build {}: hostcxx {}'.format(_ninja_escape(obj),
                                                       _ninja_escape(src)))
            objs.append(obj)
        out = osp.join(PKG, '_C_host.so')
        lines.append('build {}: link_host {}'.format(
            _ninja_escape(out), ' '.join(_ninja_escape(o) for o in objs)))
        targets.append(out)
    lines.append('default ' + ' '.join(_ninja_escape(t) for t in targets))
    with open(osp.join(build_dir, 'build.ninja'), 'w') as f:
        f.write('\n'.join(lines) + '\n')
    return targets


def build(jobs=None, debug=False, verbose=False, diag=False):
    """Incremental ninja build (gcc-style depfiles track every included
    header; ninja also rebuilds an object whose command line changed), then
    a dry run that must report nothing left to do, and a manifest
    (``build/native/manifest.json``: sha256 of every source and library) of
    what the libraries were built from."""
    targets = write_ninja(debug, diag)
    build_dir = BUILD + '_diag' if diag else BUILD
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = ['ninja', '-C', build_dir, '-j', str(jobs)]
    if verbose:
        cmd.append('-v')
    subprocess.check_call(cmd)
    dry = subprocess.run(['ninja', '-C', build_dir, '-n'], check=True,
                         capture_output=True, text=True).stdout
    if 'no work to do' not in dry:
        raise RuntimeError('native build not up to date after ninja:\n' +
                           dry)
    if not diag:
        _write_manifest(targets)
    return targets


def _sha256(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, 'rb') as f:
        for chunk in iter(lambda: f.read(1 << 20), b''):
            h.update(chunk)
    return h.hexdigest()


def _write_manifest(targets):
    import json
    srcs = sorted(glob.glob(osp.join(ROOT, 'csrc', '*', '*')))
    man = {'arch': ARCH,
           'sources': {osp.relpath(p, ROOT): _sha256(p) for p in srcs
                       if osp.isfile(p)},
           'libraries': {osp.relpath(t, ROOT): _sha256(t) for t in targets}}
    with open(osp.join(BUILD, 'manifest.json'), 'w') as f:
        json.dump(man, f, indent=1, sort_keys=True)


def clean():
    shutil.rmtree(BUILD, ignore_errors=True)
    shutil.rmtree(BUILD + '_diag', ignore_errors=True)
    for so in glob.glob(osp.join(PKG, '_C_*.so')):
        os.remove(so)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--clean', action='store_true')
    p.add_argument('--debug', action='store_true')
    p.add_argument('-j', '--jobs', type=int, default=None)
    p.add_argument('-v', '--verbose', action='store_true')
    p.add_argument('--diag', action='store_true',
                   help='diagnostic library _C_hip_diag.so (-DDGMC_DIAG)')
    args = p.parse_args(argv)
    if args.clean:
        clean()
        return 0
    for t in build(args.jobs, args.debug, args.verbose, args.diag):
        print('built', osp.relpath(t, ROOT))
    return 0


if __name__ == '__main__':
    sys.exit(main())
