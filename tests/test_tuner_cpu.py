"""Autotuner candidate sets and split-K geometry (pure Python, ops/hip_ops.py): which wgrad K / N
tiles and kernel variants the tuner may try for the S3D-G layer shapes, and the grad_sink
deferral bookkeeping used by the side-stream slab reduction."""
import os

from mil_nce_howto100m_amd.ops import grad_sink
from mil_nce_howto100m_amd.ops import hip_ops as h


def _plan(x_shape, cout, k):
    pad = tuple(kk // 2 for kk in k)
    return h.conv_plan(x_shape, (cout, x_shape[-1]) + k, (1, 1, 1), pad)


def test_wgrad_k_tiles_follow_the_reduction_width():
    # (3,1,1) over 192 channels: Ktot 576 -> 128 pads (640), 64 and 192 divide it
    p = _plan((4, 8, 25, 25, 192), 192, (3, 1, 1))
    assert p.Ktot == 576 and p.w_tk == 128
    assert set(h._wgrad_tks(p)) == {128, 64, 192}
    # 1x1 over 256 channels: 128 divides, 192 does not -> the default only
    p = _plan((4, 8, 25, 25, 256), 288, (1, 1, 1))
    assert h._wgrad_tks(p) == (128,)
    # (1,3,3) over 64 channels: Ktot 576 again
    p = _plan((4, 8, 50, 50, 64), 192, (1, 3, 3))
    assert 192 in h._wgrad_tks(p)


def test_wgrad_variants_per_tile():
    # 192-wide K tiles: register-staged only, the 2-deep variant only at N tile 64 (VGPR budget)
    assert h._wide_w_impls(64, 192) == (2, 5)
    assert h._wide_w_impls(96, 192) == (2,)
    assert h._wide_w_impls(128, 192) == (2,)
    assert h._wide_w_impls(192, 64) == (2, 5)
    assert h._wide_w_impls(192, 128) == (2,)
    assert h._wide_w_impls(128, 128) == h._W_IMPLS
    assert h._wgrad_tiles_for(192, 192) == [64, 96, 128]
    assert h._wgrad_tiles_for(64, 192) == [64]


def test_wgrad_split_geometry():
    for occ in h._W_OCCS:
        npad, kpad, splits = h._wgrad_geom(192, 576, 5_120_000, 96, 192, occ)
        assert npad == 192 and kpad == 576
        tiles = (npad // 96) * (kpad // 192)
        # as many workgroups as `occ` per CU hold without a partial last round (rounded down to
        # whole splits), never more splits than 256-row chunks
        assert occ * h._NUM_CU - tiles < splits * tiles <= occ * h._NUM_CU
        assert splits <= h._ceil(5_120_000, 256)
    # tiny reduction: one split
    assert h._wgrad_geom(64, 64, 100, 64, 64, 4)[2] == 1


def test_persistent_grids_round_down():
    """Persistent grids and split counts fill the resident capacity without overshooting it
    (hip_ops._fill, csrc/common.h fill_splits): 512 target workgroups over 3 N tiles -> 170 each."""
    assert h._fill(512, 3) == 170 and h._fill(512, 1) == 512 and h._fill(2, 3) == 1
    assert h._grid_for(5_120_000, 192, 64, 2) * 3 <= 2 * h._NUM_CU


def test_grad_sink_deferral_bookkeeping():
    class _Ev:
        pass

    assert grad_sink.pending() == 0
    grad_sink.defer(_Ev())  # outside a backward pass: no end-of-pass callback, still tracked
    grad_sink.defer(_Ev())
    assert grad_sink.pending() == 2
    grad_sink._PENDING.clear()  # drain() needs a HIP stream; on CPU just reset
    grad_sink.drain()  # nothing pending: no stream access
    assert grad_sink.pending() == 0


def test_deferred_reduce_is_opt_in():
    assert h._DEFER_WGRAD == (os.environ.get("MILNCE_DEFER_WGRAD") == "1")


def test_forward_tuner_pairs_variants_with_grid_sizes(monkeypatch):
    """The forward / dgrad tuner times (kernel variant, persistent grid) pairs; a grid whose
    partial-statistics rows would not fit the caller's buffer is never launched."""
    M, npad, bn = 256 * 8 * 50 * 50, 64, 64  # conv_2c dgrad: one 64-wide N tile
    seen = []

    def fake_tune(launch, codes, default=None, sig=""):
        for c in codes:
            launch(c)
        return max(codes)  # the last (variant, grid) pair

    monkeypatch.setattr(h, "_tune", fake_tune)
    monkeypatch.setattr(h, "_FWD_WGS_TUNE", (2, 3))
    impl, grid = h._tune_fwd(lambda i, g: seen.append((i, g)), (3, 4), M, npad, bn)
    assert {g for _, g in seen} == {2 * h._NUM_CU, 3 * h._NUM_CU}
    assert {i for i, _ in seen} == {3, 4}
    assert (impl, grid) == (4, 3 * h._NUM_CU)
    assert h._stats_rows(M, npad, bn) == 3 * h._NUM_CU
    seen.clear()
    impl, grid = h._tune_fwd(lambda i, g: seen.append((i, g)), (3, 4), M, npad, bn, max_rows=2 * h._NUM_CU)
    assert {g for _, g in seen} == {2 * h._NUM_CU} and grid == 2 * h._NUM_CU


class _FakeEvent:
    def __init__(self, *a, **k):
        self.recorded = None

    def record(self, stream=None):
        self.recorded = stream

    def query(self):
        return True


class _FakeStream:
    cuda_stream = 0


def test_reduce_batcher_one_launch_per_batch_and_no_double_target(monkeypatch):
    """The side stream's split-K reductions queue up and go out as one launch (flushed by the next
    drain, or when 16 are pending), never with two accumulations into the same gradient in one
    launch (those would race), and every flush registers its completion event with grad_sink."""
    calls = []
    monkeypatch.setattr(h, "call", lambda name, *a: calls.append((name, a[1])))
    monkeypatch.setattr(h, "_side_streams", lambda dev: [_FakeStream()])
    monkeypatch.setattr(h.torch.cuda, "Event", _FakeEvent)
    monkeypatch.setattr(grad_sink, "_PENDING", [])
    monkeypatch.setattr(grad_sink, "_ON_DRAIN", [])
    waited = []
    monkeypatch.setattr(grad_sink, "drain", lambda: (list(map(lambda f: f(), list(grad_sink._ON_DRAIN))),
                                                     waited.append(len(grad_sink._PENDING))))
    rb = h._ReduceBatcher()
    item = lambda grad: (1000, grad, 4, 64, 576, 64, 64, 64, 9)  # noqa: E731
    rb.add(object(), [item(1), item(2)], "cuda:0")
    rb.add(object(), [item(3)], "cuda:0")
    assert calls == [] and len(rb.items) == 3
    rb.add(object(), [item(2)], "cuda:0")  # gradient 2 again: the pending batch goes out first
    assert calls == [("milnce_wgrad_reduce_batch", 3)] and len(rb.items) == 1
    assert len(grad_sink._PENDING) == 1
    for g in range(10, 25):  # 1 + 15 = 16 pending -> flush without a drain
        rb.add(object(), [item(g)], "cuda:0")
    assert calls[-1] == ("milnce_wgrad_reduce_batch", 16) and rb.items == []
    rb.add(object(), [item(99)], "cuda:0")
    rb.flush()
    assert calls[-1] == ("milnce_wgrad_reduce_batch", 1) and rb.items == [] and rb.slabs == []


def test_side_keep_releases_after_completion_or_drain(monkeypatch):
    monkeypatch.setattr(grad_sink, "_AFTER_DRAIN", [])
    monkeypatch.setattr(grad_sink, "_ON_DRAIN", [])
    monkeypatch.setattr(grad_sink, "_PENDING", [])

    class Ev:
        def __init__(self, done):
            self.done = done

        def query(self):
            return self.done

    keep = h._SideKeep()
    keep.add(Ev(False), ("a",))
    keep.add(Ev(True), ("b",))
    assert len(keep.q) == 2  # the head is still running: nothing behind it is released either
    keep.q[0] = (Ev(True), ("a",))
    keep.add(None, ("c",))  # drain-only entry (no event)
    assert [t for _, t in keep.q] == [("c",)]
    grad_sink.drain()  # after the wait: everything goes
    assert len(keep.q) == 0
