"""Box-tiled forward / dgrad (csrc/conv_box.hip, impls 14 / 15 on 8-wave workgroups, 16 / 17 on
4-wave workgroups two per CU) against the fp32 reference.

The box kernels sum the taps in (channel block, tap) order instead of v3/v4's (tap, channel
block), so they are compared with the fp32 conv (bf16-rounded operands) and with v3's BN
statistics / producer-BN partials, not bitwise. Shapes cover the layouts' edge cases: tiles that
cross many (clip, frame) planes (small and odd planes), the conv_2c plane (50 x 50), every
supported T for the temporal box (P = min(256 / T, 448 / (T + 2)) positions per tile), N tiles 64 / 96 / 128 / 160 / 192, and a
channel count over several 64-wide blocks (box reloads mid-tile). The 4-wave variants sum every
output in the same order as the 8-wave ones of the same MFMA shape (16 vs 14, 17 vs 15), so their
outputs and input gradients must be bitwise equal.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CASES = [
    # B, T, H, W, Cin, Cout, k, p
    (3, 8, 11, 13, 64, 192, (1, 3, 3), (0, 1, 1)),
    (2, 8, 50, 50, 64, 192, (1, 3, 3), (0, 1, 1)),
    (2, 4, 7, 7, 128, 128, (1, 3, 3), (0, 1, 1)),
    (2, 2, 25, 25, 192, 64, (1, 3, 3), (0, 1, 1)),
    (3, 8, 9, 9, 192, 192, (3, 1, 1), (1, 0, 0)),
    (2, 4, 13, 13, 128, 64, (3, 1, 1), (1, 0, 0)),
    (2, 16, 5, 5, 64, 128, (3, 1, 1), (1, 0, 0)),
    (2, 8, 25, 25, 256, 192, (3, 1, 1), (1, 0, 0)),
    # channel counts that are not multiples of 64: a partial (zero-filled) last channel block
    (2, 8, 25, 25, 96, 128, (1, 3, 3), (0, 1, 1)),
    (3, 4, 13, 13, 224, 224, (3, 1, 1), (1, 0, 0)),
    (2, 4, 13, 13, 24, 64, (1, 3, 3), (0, 1, 1)),
    (2, 4, 13, 13, 48, 48, (3, 1, 1), (1, 0, 0)),
    # N tiles of 96 / 160 (impl 14: the weight stage rows are padded to 128 / 192)
    (2, 8, 25, 25, 64, 96, (1, 3, 3), (0, 1, 1)),
    (3, 4, 13, 13, 96, 160, (1, 3, 3), (0, 1, 1)),
    (2, 8, 13, 13, 160, 160, (3, 1, 1), (1, 0, 0)),
    (2, 4, 7, 7, 96, 320, (3, 1, 1), (1, 0, 0)),
    # T = 2: P = 112 positions per frame, the tile's last 32 rows idle
    (3, 2, 7, 7, 192, 384, (3, 1, 1), (1, 0, 0)),
    (2, 2, 11, 11, 96, 160, (3, 1, 1), (1, 0, 0)),
    # the layers of a 8 x 64^2 clip (tests/test_gpu_gradcache.py): tiny planes, T = 1 (only the
    # centre tap of a (3,1,1) conv in range), tiles spanning many clips
    (4, 4, 16, 16, 64, 192, (1, 3, 3), (0, 1, 1)),
    (4, 4, 16, 16, 192, 192, (3, 1, 1), (1, 0, 0)),
    (4, 4, 8, 8, 16, 32, (1, 3, 3), (0, 1, 1)),
    (4, 4, 8, 8, 32, 32, (3, 1, 1), (1, 0, 0)),
    (4, 2, 4, 4, 96, 208, (1, 3, 3), (0, 1, 1)),
    (4, 2, 4, 4, 208, 208, (3, 1, 1), (1, 0, 0)),
    (4, 1, 2, 2, 160, 320, (1, 3, 3), (0, 1, 1)),
    (4, 1, 2, 2, 320, 320, (3, 1, 1), (1, 0, 0)),
    (4, 1, 2, 2, 48, 128, (3, 1, 1), (1, 0, 0)),
]


@pytest.mark.parametrize("case", CASES)
def test_conv_box_matches_reference(case, monkeypatch):
    from mil_nce_howto100m_amd.ops import hip_ops as h
    monkeypatch.setattr(h, "_BOX4_FALLBACK", False)  # pinned variants: see the 4-wave refusals
    torch.manual_seed(21)
    B, T, H, W, cin, cout, k, p = case
    x = torch.randn(B, T, H, W, cin, device=DEV).to(torch.bfloat16)
    w = torch.randn(cout, cin, *k, device=DEV) * (2.0 / (cin * k[0] * k[1] * k[2])) ** 0.5
    plan = h.conv_plan(x.shape, w.shape, (1, 1, 1), p)
    wp, wd = h._pack(w, plan, 0), h._pack(w, plan, 1)
    dy = torch.randn(plan.B, plan.To, plan.Ho, plan.Wo, cout, device=DEV).to(torch.bfloat16)
    stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device=DEV)
    ss = torch.cat([torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5,
                    torch.randn(cin, device=DEV), torch.randn(cin, device=DEV) * 0.2])
    xr = x.float().requires_grad_(True)
    yr = F.conv3d(xr.permute(0, 4, 1, 2, 3), w.to(torch.bfloat16).float(), None, 1, p).permute(0, 2, 3, 4, 1)
    yr.backward(dy.float())
    geo = h._box_geo(plan)
    fw = [i for i in h._BOX_IMPLS if h._box_ok(plan.bn, cin, plan.Kpad, i, geo)]
    dg = [i for i in h._BOX_IMPLS if h._box_ok(plan.d_bn, cout, plan.d_Kpad, i, geo)]
    if not (fw or dg):
        pytest.skip(f"no box variant for N tiles {plan.bn} / {plan.d_bn} at {geo}")

    def run(fi, di, grid_wgs):
        plan.pin_f, plan.pin_d = fi, di
        plan.grid_m = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(fi, plan.bn), grid_wgs)
        plan.d_grid_m = h._grid_for(plan.M, plan.d_Npad, h._box_eff_bn(di, plan.d_bn), grid_wgs)
        y = h.conv_forward_raw(x, wp, plan, stats)
        st = stats[:plan.grid_m * 2 * plan.Npad].view(plan.grid_m, 2, plan.Npad).double().sum(0)
        dx = h.conv_dgrad(dy, wd, plan, (x, ss, cin))
        part, nparts, ps = h.take_bn_partials(dx)
        pst = part[:nparts * 2 * ps].view(nparts, 2, ps).double().sum(0)
        return y, st, dx, pst

    ref = run(4, 4, 2)
    got = {}
    try:
        for impl in sorted(set(fw) | set(dg)):
            for wgs in (1, 2):
                fi = impl if impl in fw else 4
                di = impl if impl in dg else 4
                try:
                    y, st, dx, pst = run(fi, di, wgs)
                except h.UnsupportedVariant:
                    # a 4-wave variant whose epilogue / prologue constants overflow its 80 KiB (the
                    # tuner skips it the same way)
                    assert impl in h._BOX4_IMPLS, impl
                    break
                assert _rel(y, yr) < 1e-2, (impl, wgs)
                assert torch.allclose(st, ref[1], rtol=2e-3, atol=1e-1), ("stats", impl, wgs)
                assert _rel(dx, xr.grad) < 1e-2, (impl, wgs)
                assert torch.allclose(pst, ref[3], rtol=2e-2, atol=1.0), ("partials", impl, wgs)
                # deterministic outputs (the statistics go through LDS atomics: not bitwise)
                y2, _, dx2, _ = run(fi, di, wgs)
                assert torch.equal(y, y2) and torch.equal(dx, dx2), (impl, wgs)
                got[impl] = (y if impl in fw else None, dx if impl in dg else None)
        # 4-wave vs 8-wave workgroups of the same MFMA shape: the same sums in the same order
        for i8, i4 in ((14, 16), (15, 17)):
            if i8 in got and i4 in got:
                for a, b, what in zip(got[i8], got[i4], ("y", "dx")):
                    if a is not None and b is not None:
                        assert torch.equal(a, b), (what, i8, i4)
    finally:
        plan.pin_f = plan.pin_d = 0


def _pin_tuned(h):
    """Pin every plan to its plain-call decisions (forward with statistics, dgrad with partials
    first), so two arms that differ only in the fusion flags launch the same variants on the same
    grids (each call context is tuned on its own, hip_ops._decision). Returns an unpin callable."""
    for pl in h._PLANS.values():
        for kinds, dgrad in ((("fwd|st", "fwd", "fwdpro|st|fz", "fwdpro|st|nf"), False),
                             (("dgrad|p", "dgrad", "dgradbn|p", "dgradbn"), True)):
            dec = next((pl.ctx[k] for k in kinds if k in pl.ctx), None)
            if dec is None or (pl.pin_d if dgrad else pl.pin_f):
                continue
            if dgrad:
                pl.pin_d, pl.d_grid_m = dec
            else:
                pl.pin_f, pl.grid_m = dec

    def unpin():
        for pl in h._PLANS.values():
            pl.pin_f = pl.pin_d = 0
    return unpin


def _box_impl(bn, nw=8):
    if nw == 4:  # (a 192-wide tile with the prologue constants overflows impl 17's 80 KiB: 16 splits it)
        return 17 if bn in (64, 128) else 16
    return 15 if bn in (64, 128, 192) else 14


@pytest.mark.parametrize("nw", [8, 4])
@pytest.mark.parametrize("shape,cin,cmid,k", [((2, 8, 50, 50), 64, 192, (3, 3, 3)),
                                             ((3, 8, 11, 13), 128, 128, (3, 3, 3)),
                                             ((3, 4, 13, 13), 112, 224, (3, 3, 3)),
                                             ((3, 4, 13, 13), 96, 160, (3, 3, 3))])
def test_bn_prologue_fusion_bitwise(shape, cin, cmid, k, nw):
    """A separable S3D-G unit (spatial conv -> BN -> ReLU -> temporal conv) with the spatial BN +
    ReLU applied inside the temporal conv's box kernel (hip_ops "pro" placeholders, csrc/conv_box.hip
    PRO 2: z written as the kernel's by-product) and the spatial BN's backward apply inside its
    dgrad (PRO 3: dy written as the by-product) is bitwise the unfused path (bn_relu_apply /
    bn_bwd_apply passes, then the same box kernels): outputs, input gradient, every parameter
    gradient and the running statistics; and in no-grad mode (PRO 1: no z written)."""
    import copy
    from mil_nce_howto100m_amd.models.s3dg import STConv3D
    from mil_nce_howto100m_amd.ops import hip_ops as h
    torch.manual_seed(5)
    unit = STConv3D(cin, cmid, list(k), padding=1, separable=True).cuda().train()
    x = torch.randn(*shape, cin, device=DEV).to(torch.bfloat16)
    g = torch.randn(*shape, cmid, device=DEV).to(torch.bfloat16)
    old, old_b = h._PRO_FUSE, h._BNBWD_FUSE
    res = {}
    try:
        # tune every plan of both paths first, then pin the box kernels: both arms must run the
        # same kernels from their first forward on (its BN statistics set the running mean, i.e.
        # the pre-BN storage shift of the second forward)
        for fuse in (False, True):
            h._PRO_FUSE = h._BNBWD_FUSE = fuse
            copy.deepcopy(unit)(x.clone().requires_grad_(True)).backward(g)
        # the box-tiled kernel on the temporal conv
        plan = h.conv_plan(tuple(shape) + (cmid,), (cmid, cmid, k[0], 1, 1), (1, 1, 1), (1, 0, 0))
        plan.pin_f = _box_impl(plan.bn, nw)
        if not h._box_ok(plan.bn, cmid, plan.Kpad, plan.pin_f, h._box_geo(plan)):
            pytest.skip(f"no {nw}-wave box variant for N tile {plan.bn}")
        plan.grid_m = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(plan.pin_f, plan.bn), 2 if nw == 4 else 1)
        # and on the spatial conv's dgrad: its BN backward (dy) is then staged by that dgrad
        # (conv_dgrad_bnbwd, PRO 3) when fused
        plan1 = h.conv_plan(tuple(shape) + (cin,), (cmid, cin, 1, k[1], k[2]), (1, 1, 1), (0, 1, 1))
        if plan1.d_bn <= 128:
            plan1.pin_d = _box_impl(plan1.d_bn, nw)
            if not h._box_pro3_ok(plan1.pin_d, plan1):
                pytest.skip(f"the {nw}-wave dgrad of N tile {plan1.d_bn} has no room for the BN prologue")
            plan1.d_grid_m = h._grid_for(plan1.M, plan1.d_Npad, h._box_eff_bn(plan1.pin_d, plan1.d_bn),
                                         2 if nw == 4 else 1)
        _pin_tuned(h)  # the unit's other kernels: the same variants in every arm
        for fuse in (False, True, False):
            h._PRO_FUSE = h._BNBWD_FUSE = fuse
            u = copy.deepcopy(unit)
            xi = x.clone().requires_grad_(True)
            u(xi)  # non-zero running means: the second forward stores shifted pre-BN outputs
            xi.grad = None
            u.zero_grad()
            out = u(xi)
            out.backward(g)
            grads = {n: p.grad.clone() for n, p in u.named_parameters()}
            res[fuse] = (out.detach(), xi.grad.clone(), grads, u.bn1.running_mean.clone(), u.bn2.running_var.clone())
            with torch.no_grad():
                res[(fuse, "ng")] = u(x).clone()
        a, b = res[False], res[True]
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
        for n in a[2]:
            assert torch.equal(a[2][n], b[2][n]), n
        assert torch.equal(a[3], b[3]) and torch.equal(a[4], b[4])
        assert torch.equal(res[(False, "ng")], res[(True, "ng")])
    finally:
        h._PRO_FUSE, h._BNBWD_FUSE = old, old_b
        for pl in h._PLANS.values():  # unpin: later tests tune their own contexts
            pl.pin_f = pl.pin_d = 0


def test_prologue_call_on_plan_without_prologue_room():
    """A plan first tuned on a plain input can hold a 4-wave variant whose 80 KiB has no room for
    the BN prologue's [Cin] constants (impl 17 on a 192-wide N tile fits without them only). A
    prologue ("pro" placeholder) input of the same plan then runs that variant on the materialised
    z, bitwise the unfused path, instead of failing the launch (the two-rank production DP test
    hit exactly this)."""
    import copy
    from mil_nce_howto100m_amd.models.s3dg import STConv3D
    from mil_nce_howto100m_amd.ops import hip_ops as h
    torch.manual_seed(11)
    shape, cin, cmid = (2, 4, 11, 13), 64, 192
    unit = STConv3D(cin, cmid, [3, 3, 3], padding=1, separable=True).cuda().train()
    x = torch.randn(*shape, cin, device=DEV).to(torch.bfloat16)
    g = torch.randn(*shape, cmid, device=DEV).to(torch.bfloat16)
    plan = h.conv_plan(tuple(shape) + (cmid,), (cmid, cmid, 3, 1, 1), (1, 1, 1), (1, 0, 0))
    if plan.bn != 192 or not h._box_ok(plan.bn, cmid, plan.Kpad, 17, h._box_geo(plan)):
        pytest.skip(f"N tile {plan.bn}: no plain-fit 4-wave 192-wide variant")
    assert h._box4_lds(192, plan.k, pro=1, epi=1, cin=cmid) > 80 * 1024
    old = h._PRO_FUSE
    res = {}
    try:
        for fuse in (False, True):  # tune every other plan first
            h._PRO_FUSE = fuse
            copy.deepcopy(unit)(x.clone().requires_grad_(True)).backward(g)
        plan.pin_f = 17
        plan.grid_m = h._grid_for(plan.M, plan.Npad, 192, 2)
        unpin = _pin_tuned(h)  # every other kernel the same in both arms
        for fuse in (False, True):
            h._PRO_FUSE = fuse
            u = copy.deepcopy(unit)
            xi = x.clone().requires_grad_(True)
            out = u(xi)
            out.backward(g)
            res[fuse] = (out.detach(), xi.grad.clone(), {n: p.grad.clone() for n, p in u.named_parameters()})
        a, b = res[False], res[True]
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
        for n in a[2]:
            assert torch.equal(a[2][n], b[2][n]), n
    finally:
        h._PRO_FUSE = old
        for pl in h._PLANS.values():
            pl.pin_f = pl.pin_d = 0


def test_tuned_4wave_dgrad_without_partial_room_runs_8wave_sibling():
    """A dgrad plan tuned without producer-BN partials (EPI 0) can hold impl 17 on a 192-wide
    (3,1,1) tile, which fits 80 KiB only without the partial rows; a later call with partials runs
    the 8-wave sibling (impl 15) on the same grid instead of failing: dX bitwise the 4-wave result,
    partial sums those of impl 15."""
    from mil_nce_howto100m_amd.ops import hip_ops as h
    torch.manual_seed(12)
    shape, c = (2, 4, 11, 13), 192
    plan = h.conv_plan(shape + (c,), (c, c, 3, 1, 1), (1, 1, 1), (1, 0, 0))
    geo = h._box_geo(plan)
    if plan.d_bn != 192 or not (h._box_ok(192, c, plan.d_Kpad, 17, geo) and h._box_ok(192, c, plan.d_Kpad, 15, geo)):
        pytest.skip(f"dgrad N tile {plan.d_bn}: no 192-wide 4-wave / 8-wave pair")
    assert h._box4_lds(192, plan.k, epi=2) > 80 * 1024 >= h._box4_lds(192, plan.k)
    w = torch.randn(c, c, 3, 1, 1, device=DEV) * 0.05
    wd = h._pack(w, plan, 1)
    dy = torch.randn(*shape, c, device=DEV).to(torch.bfloat16)
    x = torch.randn(*shape, c, device=DEV).to(torch.bfloat16)
    ss = torch.cat([torch.randn(c, device=DEV) * 0.1, torch.rand(c, device=DEV) + 0.5,
                    torch.randn(c, device=DEV), torch.randn(c, device=DEV) * 0.2])
    md = plan.B * plan.T * plan.H * plan.W
    try:
        plan.d_grid_m = h._grid_for(md, plan.d_Npad, 192, 2)
        plan.pin_d = 17
        dx4 = h.conv_dgrad(dy, wd, plan)  # no partials: the 4-wave kernel itself
        dx_fb = h.conv_dgrad(dy, wd, plan, (x, ss, c))  # partials: falls back
        p_fb, n_fb, ps = h.take_bn_partials(dx_fb)
        plan.pin_d = 15
        dx8 = h.conv_dgrad(dy, wd, plan, (x, ss, c))
        p8, n8, _ = h.take_bn_partials(dx8)
    finally:
        plan.pin_d = 0
    assert torch.equal(dx_fb, dx4) and torch.equal(dx_fb, dx8)
    assert n_fb == n8
    s_fb = p_fb[:n8 * 2 * ps].view(n8, 2, ps).double().sum(0)
    s8 = p8[:n8 * 2 * ps].view(n8, 2, ps).double().sum(0)
    assert torch.allclose(s_fb, s8, rtol=1e-5, atol=1e-3)


def test_inception_head_prologue_fusion():
    """An Inception block whose head outputs z1a / z2a (channel slices of the fused 1x1 GEMM output,
    row stride = all three branches) are applied by the separable units' box kernels (x_ld != Cin)
    matches the unfused block: output, input gradient and every parameter gradient, up to the
    float-atomic order of the gating sums."""
    import copy
    from mil_nce_howto100m_amd.models.s3dg import InceptionBlock
    from mil_nce_howto100m_amd.ops import hip_ops as h
    torch.manual_seed(7)
    shape = (2, 8, 11, 11)
    blk = InceptionBlock(192, 64, 96, 128, 16, 32, 32).cuda().train()
    x = torch.randn(*shape, 192, device=DEV).to(torch.bfloat16)
    g = torch.randn(*shape, blk.output_dim, device=DEV).to(torch.bfloat16)
    old, old_b = h._PRO_FUSE, h._BNBWD_FUSE
    res = {}
    try:
        for fuse in (False, True):
            h._PRO_FUSE = h._BNBWD_FUSE = fuse
            b = copy.deepcopy(blk)
            xi = x.clone().requires_grad_(True)
            b(xi).sum().backward()  # tune
            # the same running statistics in both arms (the pre-BN storage shift is the running
            # mean, and the tuning pass ran different kernels, i.e. summation orders, per arm)
            if fuse:
                b.load_state_dict(bufs, strict=False)
            else:
                bufs = {n: t.clone() for n, t in b.named_buffers()}
            for cin, cout in ((96, 128), (16, 32)):  # the spatial convs reading z1a / z2a: box-tiled
                plan = h.conv_plan(tuple(shape) + (cin,), (cout, cin, 1, 3, 3), (1, 1, 1), (0, 1, 1))
                plan.pin_f = 15
            _pin_tuned(h)  # the plain-call variants in both arms (each context is tuned on its own)
            xi.grad = None
            b.zero_grad()
            out = b(xi)
            out.backward(g)
            res[fuse] = (out.detach().float(), xi.grad.float(), {n: p.grad.clone() for n, p in b.named_parameters()})
        (o0, x0, g0), (o1, x1, g1) = res[False], res[True]
        assert _rel(o1, o0) < 2e-3 and _rel(x1, x0) < 5e-3
        for n in g0:
            assert _rel(g1[n], g0[n]) < 1e-2, n
    finally:
        h._PRO_FUSE, h._BNBWD_FUSE = old, old_b
        for pl in h._PLANS.values():
            pl.pin_f = pl.pin_d = 0


@pytest.mark.parametrize("impl", [14, 15, 16, 17])
@pytest.mark.parametrize("case", [((4, 4, 8, 8), 176, 64, 96, 128, (1, 3, 3), (0, 1, 1)),
                                  ((8, 8, 25, 25), 128, 0, 128, 128, (1, 3, 3), (0, 1, 1)),
                                  ((8, 8, 25, 25), 192, 0, 192, 192, (3, 1, 1), (1, 0, 0))])
def test_box_cold_cache_deterministic(case, impl):
    """Every launch gives the same bytes whether its operands come from HBM or from L2 / MALL.

    The counted vmcnt waits of the box kernels assume each tap's weight-stage DMA pieces issue
    before its box loads; the scheduler interleaved them, so a wait could leave a DMA piece in
    flight, which only shows when the weights come from HBM slowly enough (2-stage rings, cold
    caches). A flush of L2 and the MALL before every other launch exposes that."""
    from mil_nce_howto100m_amd.ops import hip_ops as h
    from mil_nce_howto100m_amd.ops._lib import call, ptr, stream
    (B, T, H, W), ld, c0, cin, cout, k, p = case
    torch.manual_seed(3)
    plan = h.conv_plan((B, T, H, W, cin), (cout, cin, *k), (1, 1, 1), p)
    if not h._box_ok(plan.bn, cin, plan.Kpad, impl, h._box_geo(plan)):
        pytest.skip("variant does not take this shape")
    wp = h._pack(torch.randn(cout, cin, *k, device=DEV) * 0.05, plan, 0)
    full = torch.randn(B, T, H, W, ld, device=DEV).to(torch.bfloat16)
    ss = torch.cat([torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5,
                    torch.rand(cin, device=DEV) + 0.5, torch.randn(cin, device=DEV) * 0.2])
    flush = torch.empty((384 << 20) // 4, device=DEV)
    grid = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(impl, plan.bn), 2 if impl in h._BOX4_IMPLS else 1)
    outs = []
    for rep in range(8):
        if rep % 2 == 0:
            flush.zero_()
        y = torch.empty((B, T, H, W, cout), dtype=torch.bfloat16, device=DEV)
        z = torch.empty((B, T, H, W, cin), dtype=torch.bfloat16, device=DEV)
        try:
            call("milnce_conv_fwd_pro", ptr(full[..., c0:]), ld, ptr(wp), ptr(y), None, None, ptr(ss), ptr(z),
                 B, T, H, W, cin, cout, *k, *p, plan.Kpad, plan.Npad, cout, plan.bn, grid, impl, stream())
        except h.UnsupportedVariant:
            pytest.skip("variant declines the shape (LDS budget)")
        outs.append((y, z))
    for y, z in outs[1:]:
        assert torch.equal(y, outs[0][0]) and torch.equal(z, outs[0][1])
