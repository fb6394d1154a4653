"""Synthetic, shape-faithful datasets + the HBM-resident pair loader."""
from .keypoints import (PASCAL_VOC_CATEGORIES, WILLOW_CATEGORIES,
                        KeypointCategory, KeypointGraphDataset,
                        keypoint_transform, make_keypoint_datasets)
from .device_loader import GraphStore, DevicePairLoader

__all__ = [
    'PASCAL_VOC_CATEGORIES', 'WILLOW_CATEGORIES', 'KeypointCategory',
    'KeypointGraphDataset', 'keypoint_transform', 'make_keypoint_datasets',
    'GraphStore', 'DevicePairLoader',
]
