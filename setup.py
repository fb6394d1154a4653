"""Package + in-tree native build.

    python setup.py build_ext --inplace     # == python tools/build_native.py

The native libraries are compiled by ``tools/build_native.py`` (hipcc for
gfx950 + g++, driven by ninja) rather than torch's ``CUDAExtension``, which
would run a hipify pass over sources that are already written for CDNA4.
"""
import os.path as osp
import sys

from setuptools import Command, find_packages, setup
from setuptools.command.build_ext import build_ext

ROOT = osp.dirname(osp.abspath(__file__))
PKG = 'deep_graph_matching_consensus_amd'
__version__ = '1.0.0'


class NativeBuild(build_ext):
    def run(self):
        sys.path.insert(0, osp.join(ROOT, 'tools'))
        import build_native
        build_native.build()


class NativeClean(Command):
    user_options = []

    def initialize_options(self):
        pass

    def finalize_options(self):
        pass

    def run(self):
        sys.path.insert(0, osp.join(ROOT, 'tools'))
        import build_native
        build_native.clean()


setup(
    name='deep_graph_matching_consensus_amd',
    version=__version__,
    description='MI355X-native Deep Graph Matching Consensus',
    packages=find_packages(include=[PKG, PKG + '.*']),
    package_data={PKG: ['_C_*.so', 'runtime/tuned/*.csv']},
    cmdclass={'build_ext': NativeBuild, 'clean_native': NativeClean},
)
