"""Encoders and the DGMC matching module (``dgmc.models`` API)."""
from .mlp import MLP
from .gin import GIN
from .spline import SplineCNN
from .rel import RelCNN, RelConv
from .dgmc import DGMC

__all__ = [
    'MLP',
    'GIN',
    'SplineCNN',
    'RelCNN',
    'RelConv',
    'DGMC',
]
