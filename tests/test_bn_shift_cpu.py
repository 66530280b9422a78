"""Pre-BN storage shift bookkeeping (ops/hip_ops.py ``_bn_shift``), CPU only: which per-channel
shift the conv epilogues get. The numerics of the shifted storage are pinned on the GPU
(tests/test_gpu_ops.py::test_bn_shifted_storage_large_mean, profiles/r4_fulldepth.md)."""
import torch

from mil_nce_howto100m_amd.ops import hip_ops as h


def test_single_bn_uses_its_running_mean(monkeypatch):
    monkeypatch.setattr(h, "_BN_SHIFT", True)
    rm = torch.randn(16)
    assert h._bn_shift([rm], True) is rm           # finalize updates it in place: next step's shift
    assert h._bn_shift([rm], False) is None        # eval stores y unshifted
    monkeypatch.setattr(h, "_BN_SHIFT", False)
    assert h._bn_shift([rm], True) is None


def test_group_shift_buffer_is_persistent_and_follows_python_writes(monkeypatch):
    monkeypatch.setattr(h, "_BN_SHIFT", True)
    a, b = torch.zeros(8), torch.ones(16)
    s = h._bn_shift([a, b], True)
    assert torch.equal(s, torch.cat([a, b]))
    assert h._bn_shift([a, b], True) is s          # no concatenation per step
    b.copy_(torch.full((16,), 3.0))               # load_state_dict / user writes bump the version
    s2 = h._bn_shift([a, b], True)
    assert s2 is not s and torch.equal(s2, torch.cat([a, b]))


def test_no_shift_for_non_contiguous_or_missing_running_means(monkeypatch):
    monkeypatch.setattr(h, "_BN_SHIFT", True)
    rm = torch.randn(32)[::2]
    assert h._bn_shift([rm], True) is None
    assert h._bn_shift([None], True) is None
    assert h._bn_shift([torch.randn(8, dtype=torch.float64)], True) is None
