"""Native op layer: HIP kernels on MI355X, PyTorch oracles on CPU."""
from ._backend import hip_available, host_available, use_hip
from .sparse import SparseOperator, spmm
from .plans import (spline_plan, adjacency_plan, relational_plan,
                    compute_spline_basis, clear_plan_cache)
from . import dense, sparse_corr, reference

__all__ = [
    'hip_available', 'host_available', 'use_hip', 'SparseOperator', 'spmm',
    'spline_plan', 'adjacency_plan', 'relational_plan',
    'compute_spline_basis', 'clear_plan_cache', 'dense', 'sparse_corr',
    'reference',
]
