"""PyG-free graph data layer: containers, collation, transforms, packing."""
from .data import Data, Batch
from .loader import DataLoader, Collater
from .meta import BatchInfo, batch_info, register_batch_info
from .dense import DenseLayout, dense_layout, to_dense_batch
from . import transforms

__all__ = [
    'Data', 'Batch', 'DataLoader', 'Collater', 'BatchInfo', 'batch_info',
    'register_batch_info', 'DenseLayout', 'dense_layout', 'to_dense_batch',
    'transforms',
]
