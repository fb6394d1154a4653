"""MI355X-native Deep Graph Matching Consensus.

A from-scratch re-design of ``dgmc`` (Fey et al., ICLR 2020) for AMD Instinct
MI355X (gfx950): PyTorch-ROCm for orchestration, hand-written HIP kernels for
message passing and the consensus loop, RCCL data parallelism.
"""
from . import graph
from . import models
from . import utils
from .models.dgmc import DGMC

__version__ = '1.0.0'

__all__ = [
    'graph',
    'models',
    'utils',
    'DGMC',
    '__version__',
]
