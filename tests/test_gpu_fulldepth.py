"""Full-depth S3D-G numerics against an fp32 reference.

Same weights and batch (8 clips of 16 x 112^2, train-mode BN: batch statistics, eps 1e-5,
momentum 0.1, reference ``s3dg.py:107-111``). The fp32 reference is the ATen path computing in
fp32 on the same GPU (``ops.force_aten(keep_dtype=True)``: MIOpen / hipBLASLt fp32).

1. Teacher-forced, block by block: every Inception block of the HIP path gets the fp32
   reference's own block input (rounded to bf16) and a random upstream gradient; its output,
   input gradient and every parameter gradient are compared with the fp32 block on the same
   (bf16-valued) input. This pins the numerics of every fused kernel at depth, at the layer
   shapes of the real network, without the error of earlier blocks.
2. End to end: the embeddings and block outputs of the whole HIP forward against fp32, next to
   the same ATen ops run with bf16 activations (plain MIOpen bf16). At random init this network
   amplifies any perturbation by ~1.4-1.6x per Inception block (shown by perturbing the fp32
   input by 1e-3 relative noise), so both bf16 paths end ~30 % from fp32 at mixed_5c; the HIP
   path must be no less accurate than ATen bf16 at every block.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

BLOCKS = ["mixed_3b", "mixed_3c", "mixed_4b", "mixed_4c", "mixed_4d", "mixed_4e", "mixed_4f", "mixed_5b", "mixed_5c"]


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm()).item()


def _models():
    from mil_nce_howto100m_amd.models import S3D
    torch.manual_seed(0)
    m = S3D(512, vocab_size=2000).cuda().train()
    ref = copy.deepcopy(m).float().train()
    v = torch.randint(0, 256, (8, 3, 16, 112, 112), dtype=torch.uint8, device="cuda")
    t = torch.randint(0, 2000, (16, 20), device="cuda")
    return m, ref, v, t


def _block_io(model, v, t):
    from mil_nce_howto100m_amd import ops
    io = {}
    hooks = [getattr(model, n).register_forward_hook(
        lambda mod, i, o, n=n: io.__setitem__(n, (i[0].detach(), o.detach()))) for n in BLOCKS]
    with torch.no_grad(), ops.force_aten(keep_dtype=True):
        out = model(v, t)
    for h in hooks:
        h.remove()
    return io, out


def test_full_depth_blocks_teacher_forced():
    from mil_nce_howto100m_amd import ops
    m, ref, v, t = _models()
    m_bf = copy.deepcopy(m)
    io, _ = _block_io(copy.deepcopy(ref), v, t)
    torch.manual_seed(1)
    worst = {"out": 0.0, "dx": 0.0, "flat": 0.0, "param": 0.0}
    worst_b = dict(worst)

    def block_run(blk, xin, g, aten, keep):
        x = xin.clone().requires_grad_(True)
        if aten:
            with ops.force_aten(keep_dtype=keep):
                out = blk(x)
                out.backward(g.to(out.dtype))
        else:
            out = blk(x)
            out.backward(g.to(out.dtype))
        grads = {k: p.grad.detach().clone() for k, p in blk.named_parameters() if p.grad is not None}
        for p in blk.parameters():
            p.grad = None
        return out.detach(), x.grad.detach(), grads

    def errs(res, ref_res):
        (o, dx, gp), (o_r, dx_r, gp_r) = res, ref_res
        assert set(gp) == set(gp_r) and gp_r
        per = sorted(((_rel(gp[k], gp_r[k]), k) for k in gp_r), reverse=True)
        flat = _rel(torch.cat([gp[k].reshape(-1) for k in sorted(gp_r)]),
                    torch.cat([gp_r[k].reshape(-1) for k in sorted(gp_r)]))
        return {"out": _rel(o, o_r), "dx": _rel(dx, dx_r), "flat": flat, "param": per[0][0]}, per[0][1]

    for n in BLOCKS:
        x32, _ = io[n]
        xb = x32.to(torch.bfloat16)  # both paths see the same bf16-valued block input
        g = torch.randn(x32.shape[:-1] + (getattr(m, n).output_dim,), device="cuda")
        r_ref = block_run(getattr(ref, n), xb.float(), g, True, True)       # fp32 ATen
        r_hip = block_run(getattr(m, n), xb, g, False, False)               # HIP, bf16 activations
        r_bf = block_run(getattr(m_bf, n), xb, g, True, False)              # ATen, bf16 activations
        e_h, kh = errs(r_hip, r_ref)
        e_b, _ = errs(r_bf, r_ref)
        print(f"{n:9s} hip: out {e_h['out']:.4f} dx {e_h['dx']:.4f} params {e_h['flat']:.4f} "
              f"worst {e_h['param']:.4f} ({kh}) | aten-bf16: out {e_b['out']:.4f} dx {e_b['dx']:.4f} "
              f"params {e_b['flat']:.4f} worst {e_b['param']:.4f}")
        for key in worst:
            worst[key] = max(worst[key], e_h[key])
            worst_b[key] = max(worst_b[key], e_b[key])
    print("worst over blocks: hip", worst, "aten-bf16", worst_b)
    # the block output is pinned to bf16 level; gradients are compared with what plain bf16
    # activations cost on the same ATen ops (bf16 rounding of dz before every BN backward, and
    # max-pool ties among bf16 values routing the gradient)
    assert worst["out"] < 0.02
    for key in ("dx", "flat", "param"):
        assert worst[key] <= 1.25 * worst_b[key] + 0.01, (key, worst[key], worst_b[key])
    # measured worst 0.092 / 0.091 (profiles/r4_fulldepth.md)
    assert worst["dx"] < 0.11 and worst["flat"] < 0.11


def test_full_depth_end_to_end_vs_fp32():
    from mil_nce_howto100m_amd import ops
    m, ref, v, t = _models()
    m_bf = copy.deepcopy(m)
    gv = torch.randn(8, 512, device="cuda", dtype=torch.float64)
    gt = torch.randn(16, 512, device="cuda", dtype=torch.float64)

    def run(model, video):
        acts = {}
        hooks = [getattr(model, n).register_forward_hook(
            lambda mod, i, o, n=n: acts.__setitem__(n, o.detach().double())) for n in BLOCKS]
        ve, te = model(video, t)
        ((ve.double() * gv).sum() + (te.double() * gt).sum()).backward()
        for h in hooks:
            h.remove()
        return ve.detach().double(), te.detach().double(), acts

    ve, te, acts = run(m, v)
    with ops.force_aten(keep_dtype=True):
        vr, tr, acts_r = run(ref, v)
        # sensitivity of the fp32 network itself: the same input with 1e-3 relative noise
        vf = v.float() / 255.0
        vp = (vf * (1 + 1e-3 * torch.randn_like(vf))).clamp(0, 1)
        _, _, acts_p = run(copy.deepcopy(ref), vp)
    with ops.force_aten():  # the same ATen ops with bf16 activations (MIOpen bf16)
        vb, tb, acts_b = run(m_bf, v)
    torch.cuda.synchronize()
    for n in BLOCKS:
        print(f"{n:9s} vs fp32: hip {_rel(acts[n], acts_r[n]):.4f}  aten-bf16 {_rel(acts_b[n], acts_r[n]):.4f}  "
              f"(fp32 with 1e-3 input noise: {_rel(acts_p[n], acts_r[n]):.4f})")
        assert _rel(acts[n], acts_r[n]) <= 1.1 * _rel(acts_b[n], acts_r[n]) + 0.005, n
    ev, eb = _rel(ve, vr), _rel(vb, vr)
    print(f"video embedding vs fp32: hip {ev:.4f} aten-bf16 {eb:.4f}; text: hip {_rel(te, tr):.4f}")
    assert ev <= 1.1 * eb + 0.005 and _rel(te, tr) < 0.02
    assert _rel(acts["mixed_3b"], acts_r["mixed_3b"]) < 0.05
