"""Runtime utilities: roctx tracing ranges, HIP-event step timers, hang watchdog, HIP-graph replay,
the high-priority step stream."""
from . import roctx
from .hipgraph import GraphedCallable
from .streams import MainStream
from .timers import StepTimer
from .watchdog import Watchdog

__all__ = ["roctx", "GraphedCallable", "MainStream", "StepTimer", "Watchdog"]
