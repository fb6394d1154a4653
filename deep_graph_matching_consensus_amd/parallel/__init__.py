"""Data parallelism over RCCL (GPU) / gloo (CPU)."""
from .dist import (init_distributed, is_distributed, rank, world_size,
                   barrier, all_reduce_max, all_reduce_sum, all_gather_state,
                   shutdown,
                   env_rank, env_world_size, env_local_rank)
from .ddp import (GradBucketAllReducer, captured_allreduce_preflight,
                  sequence_digest)

__all__ = [
    'init_distributed', 'is_distributed', 'rank', 'world_size', 'barrier',
    'all_reduce_max', 'all_reduce_sum', 'all_gather_state', 'shutdown',
    'env_rank',
    'env_world_size', 'env_local_rank', 'GradBucketAllReducer',
    'captured_allreduce_preflight', 'sequence_digest',
]
