"""Runtime: execution modes, hipGraph capture, profiling hooks."""
from .mode import reference_mode, is_reference_mode, set_reference_mode

__all__ = ['reference_mode', 'is_reference_mode', 'set_reference_mode']
