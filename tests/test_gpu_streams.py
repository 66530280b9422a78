"""The training step's high-priority stream (utils/streams.py MainStream): it is the highest
priority the device offers, work queued on the previous stream is ordered before its kernels, and
the previous stream waits for its work at exit."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_main_stream_priority_and_ordering():
    from mil_nce_howto100m_amd.utils import MainStream
    dev = torch.device("cuda")
    prev = torch.cuda.current_stream(dev)
    a = torch.empty(1 << 24, device=dev)
    a.fill_(1.0)
    b = a * 3.0  # queued on the previous stream, possibly still running at entry
    with MainStream(dev, enabled=True) as ms:
        lo, hi = torch.cuda.Stream.priority_range()
        assert ms.stream.priority == min(lo, hi) and ms.priority == ms.stream.priority
        assert torch.cuda.current_stream(dev) == ms.stream
        c = b + 1.0  # reads the previous stream's result
        d = c.sum()
    assert torch.cuda.current_stream(dev) == prev
    assert float(d.item()) == 4.0 * (1 << 24)  # read on the previous stream after exit


def test_main_stream_disabled_is_a_no_op():
    from mil_nce_howto100m_amd.utils import MainStream
    dev = torch.device("cuda")
    prev = torch.cuda.current_stream(dev)
    with MainStream(dev, enabled=False) as ms:
        assert torch.cuda.current_stream(dev) == prev and ms.priority == 0
