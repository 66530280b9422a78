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
    assert h._halo_wgrad_ok(plan, x)
    out = torch.full((Cout, Cin) + k, 0.5, device="cuda")
    h._halo_wgrad(dy, x, plan, cc, out, 1)  # accumulate onto 0.5
    ref = torch.nn.grad.conv3d_weight(x.permute(0, 4, 1, 2, 3).float(), (Cout, Cin) + k,
                                      dy.permute(0, 4, 1, 2, 3).float(), stride=1, padding=pad)
    torch.cuda.synchronize()
    err = ((out - 0.5 - ref).norm() / ref.norm()).item()
    assert err < 2e-5, err
