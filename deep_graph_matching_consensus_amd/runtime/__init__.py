"""Runtime: execution modes, forward caches, hipGraph capture."""
from .mode import reference_mode, is_reference_mode, set_reference_mode
from .cache import forward_cache, cached
from .graphs import GraphedStep, graph_capture_supported
from .loopgrad import loop_scope
from .profiling import trace_range, mark, enable as enable_profiling

__all__ = ['reference_mode', 'is_reference_mode', 'set_reference_mode',
           'forward_cache', 'cached', 'GraphedStep',
           'graph_capture_supported', 'loop_scope', 'trace_range', 'mark',
           'enable_profiling']
