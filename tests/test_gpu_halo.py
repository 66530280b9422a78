"""Box-tiled ("halo") conv kernels (csrc/conv_halo.hip) against fp32 PyTorch on the same bf16
operands: odd channel counts, planes not divisible by the box, both channel chunk sizes."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [
    # (B, T, H, W, Cin, Cout, k)
    (2, 8, 50, 50, 64, 192, (1, 3, 3)),
    (2, 8, 50, 50, 192, 192, (3, 1, 1)),
    (3, 8, 25, 25, 96, 128, (1, 3, 3)),
    (2, 4, 13, 13, 160, 320, (1, 3, 3)),
    (2, 4, 13, 13, 112, 224, (1, 3, 3)),
    (3, 2, 7, 7, 48, 128, (1, 3, 3)),
    (2, 4, 13, 13, 208, 208, (3, 1, 1)),
    (4, 2, 7, 7, 32, 128, (3, 1, 1)),
    (2, 8, 25, 25, 16, 32, (1, 3, 3)),
]


@pytest.mark.parametrize("cc", [64, 128])
@pytest.mark.parametrize("shape", SHAPES)
def test_halo_wgrad_matches_fp32(shape, cc):
    from mil_nce_howto100m_amd.ops import hip_ops as h
    B, T, H, W, Cin, Cout, k = shape
    if cc == 128 and k[0] == 1:
        pytest.skip("128-channel chunks: temporal kernel only")
    pad = tuple(kk // 2 for kk in k)
    torch.manual_seed(sum(shape[:6]) + cc)
    x = torch.randn(B, T, H, W, Cin, device="cuda").to(torch.bfloat16)
    dy = torch.randn(B, T, H, W, Cout, device="cuda").to(torch.bfloat16)
    plan = h.conv_plan(x.shape, (Cout, Cin) + k, (1, 1, 1), pad)
    assert h._halo_wgrad_supported(plan, x)
    out = torch.full((Cout, Cin) + k, 0.5, device="cuda")
    h._halo_wgrad(dy, x, plan, cc, out, 1)  # accumulate onto 0.5
    ref = torch.nn.grad.conv3d_weight(x.permute(0, 4, 1, 2, 3).float(), (Cout, Cin) + k,
                                      dy.permute(0, 4, 1, 2, 3).float(), stride=1, padding=pad)
    torch.cuda.synchronize()
    err = ((out - 0.5 - ref).norm() / ref.norm()).item()
    assert err < 2e-5, err


@pytest.mark.parametrize("B,K,scale", [(8, 4, 1.0), (100, 4, 0.05), (256, 4, 0.05), (256, 1, 0.05), (130, 2, 0.05),
                                        (96, 8, 0.05), (2048, 4, 0.05)])
def test_fused_milnce_matches_fp64(B, K, scale):
    """Fused MIL-NCE (csrc/milnce_fused.hip, no [Bg, Bg*K] tensor) vs the loss.py formula in fp64:
    loss and both gradients to 1e-4 relative; B not a multiple of the 64-tile, every K that divides 64."""
    from mil_nce_howto100m_amd.ops import aten
    from mil_nce_howto100m_amd.ops import hip_ops as h
    torch.manual_seed(B + K)
    v = (torch.randn(B, 512, device="cuda") * scale).requires_grad_(True)
    t = (torch.randn(B * K, 512, device="cuda") * scale).requires_grad_(True)
    assert h.milnce_fused_ok(v, t)
    loss = h.milnce_loss(v, t, fused=True)
    (loss * 1.7).backward()
    vr = v.detach().double().cpu().requires_grad_(True)
    tr = t.detach().double().cpu().requires_grad_(True)
    lr = aten.milnce_loss(vr, tr)
    (lr * 1.7).backward()
    # split-bf16 logits (hi*hi + hi*lo + lo*hi, 16 significant bits per operand): 1e-4 relative
    assert abs(loss.item() - lr.item()) < 1e-4 * max(1.0, abs(lr.item())), (loss.item(), lr.item())
    rel = lambda a, b: ((a.double().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(v.grad, vr.grad) < 1e-4 and rel(t.grad, tr.grad) < 1e-4, (rel(v.grad, vr.grad), rel(t.grad, tr.grad))


def test_fused_milnce_memory_and_time_at_8192():
    """BASELINE config 5's global batch (Bg = 8192, K = 4): the fused loss's workspace (partials and
    the split-bf16 operand copies, ~170 MiB) instead of two 1 GiB logit / dlogit tensors."""
    import time
    from mil_nce_howto100m_amd.ops import hip_ops as h
    B, K = 8192, 4
    v = (torch.randn(B, 512, device="cuda") * 0.05).requires_grad_(True)
    t = (torch.randn(B * K, 512, device="cuda") * 0.05).requires_grad_(True)
    out = {}
    for fused in (True, False):
        for _ in range(3):  # steady state on the last repetition
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats()
            base = torch.cuda.memory_allocated()
            t0 = time.perf_counter()
            loss = h.milnce_loss(v, t, fused=fused)
            loss.backward()
            torch.cuda.synchronize()
            out[fused] = (float(loss.detach()), (torch.cuda.max_memory_allocated() - base) / 2 ** 20,
                          time.perf_counter() - t0)
            v.grad = t.grad = None
    print(f"fused: loss {out[True][0]:.5f} peak +{out[True][1]:.0f} MiB {out[True][2] * 1e3:.1f} ms | "
          f"materialised: loss {out[False][0]:.5f} peak +{out[False][1]:.0f} MiB {out[False][2] * 1e3:.1f} ms")
    assert abs(out[True][0] - out[False][0]) < 1e-4 * abs(out[False][0])
    assert out[True][1] < 400 and out[False][1] > 1000


@pytest.mark.parametrize("B", [256, 1024, 2048])
def test_fused_milnce_speed_report(B):
    """Steady-state time of the fused vs materialising loss (forward + backward) at the global
    batches of 1, 4 and 8 GPUs (printed; the dispatch threshold in ops/hip_ops.py follows it)."""
    import time
    from mil_nce_howto100m_amd.ops import hip_ops as h
    v = (torch.randn(B, 512, device="cuda") * 0.05).requires_grad_(True)
    t = (torch.randn(B * 4, 512, device="cuda") * 0.05).requires_grad_(True)
    res = {}
    for fused in (True, False):
        for rep in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h.milnce_loss(v, t, fused=fused).backward()
            torch.cuda.synchronize()
            res[fused] = (time.perf_counter() - t0) * 1e3
    print(f"B {B}: fused {res[True]:.3f} ms, materialised {res[False]:.3f} ms")


@pytest.mark.parametrize("batch", [True, False])
@pytest.mark.parametrize("k,halo", [((1, 3, 3), True), ((1, 3, 3), False), ((3, 1, 1), False), ((1, 1, 1), False)])
def test_deferred_wgrad_reduce_matches_inline(k, halo, batch, monkeypatch):
    """conv_wgrad(defer=True): the wgrad runs on the side stream (its slab reductions batched into
    one launch, or one each) and lands in the accumulated gradient once grad_sink.drain() joined
    it -- same values as the inline reduce, also when the main stream immediately reuses freed
    memory for new work."""
    from mil_nce_howto100m_amd.ops import grad_sink
    from mil_nce_howto100m_amd.ops import hip_ops as h
    monkeypatch.setattr(h, "_DEFER_WGRAD", True)
    monkeypatch.setattr(h, "_REDUCE_BATCH", batch)
    torch.manual_seed(7)
    B, T, H, W, Cin, Cout = 4, 8, 25, 25, 64, 192
    pad = tuple(kk // 2 for kk in k)
    x = torch.randn(B, T, H, W, Cin, device="cuda").to(torch.bfloat16)
    dy = torch.randn(B, T, H, W, Cout, device="cuda").to(torch.bfloat16)
    plan = h.conv_plan(x.shape, (Cout, Cin) + k, (1, 1, 1), pad)
    if halo:
        if not h._halo_wgrad_supported(plan, x):
            pytest.skip("no halo kernel for this shape")
        plan.w_tn, plan.w_impl, plan.w_occ = 64, 164, 2
    else:
        plan.w_tn, plan.w_impl, plan.w_occ = 128, 2, 4
    ref = torch.full((Cout, Cin) + k, 0.25, device="cuda")
    h.conv_wgrad(dy, x, plan, out=ref)
    out = torch.full((Cout, Cin) + k, 0.25, device="cuda")
    for _ in range(3):  # three deferred accumulations, each followed by main-stream allocations
        h.conv_wgrad(dy, x, plan, out=out, defer=True)
        junk = [torch.full((1 << 20,), 9.0, device="cuda") for _ in range(8)]
        del junk
    # batched: each call targets the same gradient, so every add flushes the previous one
    assert grad_sink.pending() == 3
    grad_sink.drain()
    assert grad_sink.pending() == 0
    expect = (ref - 0.25) * 3 + 0.25
    torch.cuda.synchronize()
    err = ((out - expect).norm() / (expect - 0.25).norm()).item()
    assert err < 1e-6, err
    # the batched reduction sums each element in the per-launch order: bitwise the same
    out1 = torch.full((Cout, Cin) + k, 0.25, device="cuda")
    h.conv_wgrad(dy, x, plan, out=out1, defer=True)
    grad_sink.drain()
    monkeypatch.setattr(h, "_REDUCE_BATCH", not batch)
    out2 = torch.full((Cout, Cin) + k, 0.25, device="cuda")
    h.conv_wgrad(dy, x, plan, out=out2, defer=True)
    grad_sink.drain()
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
