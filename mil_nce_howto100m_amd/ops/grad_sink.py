"""Who to tell when a kernel wrote a parameter's gradient in place (see hip_ops "Direct
gradient writes"). The data-parallel bucketer registers itself here; pure Python, so it can be
imported on CPU-only hosts without loading the HIP library."""
_SINK = None


def set_sink(fn) -> None:
    global _SINK
    _SINK = fn


def notify(param) -> None:
    if _SINK is not None:
        _SINK(param)
