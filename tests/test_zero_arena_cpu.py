"""Zero arena (ops/hip_ops.py::_ZeroArena): the per-step pool of zero-initialised fp32 accumulators."""
import torch

from mil_nce_howto100m_amd.ops import hip_ops


def test_zero_arena_sizing_reuse_and_rezero():
    a = hip_ops._ZeroArena()
    dev = torch.device("cpu")
    # inactive: plain zeros
    assert a.zeros((2, 3), dev).abs().sum() == 0 and a.buf is None
    # first active step only records the demand
    a.begin(dev)
    t = a.zeros((3, 5), dev)
    a.end()
    assert a.buf is None and a.demand == 64
    # second step allocates the recorded demand; what does not fit falls back to fresh zeros
    a.begin(dev)
    x, y = a.zeros((3, 5), dev), a.zeros((2, 70), dev)
    assert x.data_ptr() == a.buf.data_ptr() and a.buf.numel() == 64
    assert y.data_ptr() != a.buf.data_ptr() and float(y.abs().sum()) == 0
    x += 7
    assert float(a.buf[:15].sum()) == 7 * 15
    a.end()
    # third step grows to the new demand (64 + 192): fresh zeros, both slices inside, 256-B aligned
    a.begin(dev)
    assert a.buf.numel() == 64 + 192 and float(a.buf.abs().sum()) == 0
    x, y = a.zeros((3, 5), dev), a.zeros((2, 70), dev)
    assert y.data_ptr() - x.data_ptr() == 64 * 4
    v0 = y._version
    x += 1  # slices are not views of one base: separate autograd version counters
    assert y._version == v0
    y += 2
    a.end()
    # fourth step re-zeroes only what was handed out, in place
    ptr = a.buf.data_ptr()
    a.begin(dev)
    assert a.buf.data_ptr() == ptr and float(a.buf.abs().sum()) == 0
    a.end()
    assert a.zeros((4,), dev).numel() == 4  # inactive again
    del t
