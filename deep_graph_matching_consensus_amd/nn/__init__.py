"""Graph neural network layers built on the native sparse operators."""
from .conv import SplineConv, GINConv
from .inits import reset, uniform

__all__ = ['SplineConv', 'GINConv', 'reset', 'uniform']
