"""Pair-data utilities (``dgmc.utils`` API)."""
from .data import PairData, PairDataset, ValidPairDataset

__all__ = [
    'PairData',
    'PairDataset',
    'ValidPairDataset',
]
