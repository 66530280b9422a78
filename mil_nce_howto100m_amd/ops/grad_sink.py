"""Who to tell when a kernel wrote a parameter's gradient in place (see hip_ops "Direct
gradient writes"). The data-parallel bucketer registers itself here; pure Python, so it can be
imported on CPU-only hosts without loading the HIP library.

Deferred writes: a gradient whose final write runs on a side stream (the split-K wgrad slab
reduction, hip_ops.conv_wgrad(defer=True)) registers that stream's completion event with
``defer``; ``drain`` makes the current stream wait for all of them. Every consumer of the flat
gradient buffer drains first: the bucketer before each all-reduce and in ``finish`` (which the
trainer calls before the optimizer step); the first deferral of a backward pass also queues a
drain as an autograd end-of-pass callback."""
_SINK = None
_PENDING = []
_ON_DRAIN = []  # run (once) by the next drain before it waits: e.g. hip_ops' batched slab reductions


_AFTER_DRAIN = []  # run by every drain after the current stream waits (persistent registrations)
_STREAMS = []  # extra compute streams (hip_ops branch streams): joined by every drain / join


def add_stream(stream) -> None:
    if stream not in _STREAMS:
        _STREAMS.append(stream)


def on_drain(fn) -> None:
    if fn not in _ON_DRAIN:
        _ON_DRAIN.append(fn)


def after_drain(fn) -> None:
    if fn not in _AFTER_DRAIN:
        _AFTER_DRAIN.append(fn)


def set_sink(fn) -> None:
    global _SINK
    _SINK = fn


def notify(param) -> None:
    if _SINK is not None:
        _SINK(param)


def defer(event) -> None:
    if not _PENDING:
        # join at the end of the running backward pass too, so gradients are complete when
        # .backward() returns whoever reads them (a no-op if a bucket launch drained already)
        try:
            import torch
            torch.autograd.Variable._execution_engine.queue_callback(drain)
        except RuntimeError:  # not inside a backward pass: the explicit drain() points remain
            pass
    _PENDING.append(event)


def drain() -> None:
    while _ON_DRAIN:
        _ON_DRAIN.pop(0)()
    if _PENDING or _STREAMS:
        import torch
        s = torch.cuda.current_stream()
        for e in _PENDING:
            s.wait_event(e)
        _PENDING.clear()
        for st in _STREAMS:
            if st != s:
                s.wait_stream(st)
    for fn in _AFTER_DRAIN:
        fn()


def join(stream) -> None:
    """Make ``stream`` (not the current one) wait for every deferred gradient write so far: a
    bucket all-reduce issued from it sees complete gradients while the compute stream keeps going.
    The writes stay pending for the next ``drain``."""
    while _ON_DRAIN:
        _ON_DRAIN.pop(0)()
    for e in _PENDING:
        stream.wait_event(e)
    for st in _STREAMS:
        if st != stream:
            stream.wait_stream(st)


def pending() -> int:
    return len(_PENDING) + len(_ON_DRAIN)
