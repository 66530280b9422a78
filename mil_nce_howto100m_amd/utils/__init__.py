"""Runtime utilities: roctx tracing ranges, HIP-event step timers, hang watchdog."""
from . import roctx
from .timers import StepTimer
from .watchdog import Watchdog

__all__ = ["roctx", "StepTimer", "Watchdog"]
