"""Runtime utilities: roctx tracing ranges, HIP-event step timers, hang watchdog, HIP-graph replay."""
from . import roctx
from .hipgraph import GraphedCallable
from .timers import StepTimer
from .watchdog import Watchdog

__all__ = ["roctx", "GraphedCallable", "StepTimer", "Watchdog"]
