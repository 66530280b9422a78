"""Per-block S3D-G numerics against fp32, at random init and on trained weights, with the pre-BN
storage shift (MILNCE_BN_SHIFT, ops/hip_ops.py _bn_shift) on and off.

Teacher-forced (as tests/test_gpu_fulldepth.py): every Inception block of the HIP path gets the fp32
reference's own block input (rounded to bf16) and a random upstream gradient; its output, input
gradient and parameter gradients are compared with the fp32 ATen block on the same input, next to
the ATen ops run with bf16 activations. "Trained" weights come from the structured-synthetic
learning run of tests/test_gpu_training.py (Adam, lr 1e-3, bs 32, 8 x 112^2), after which the
conv outputs' channel means dwarf their spread in many layers (printed as |mean| / std).

    python tools/fulldepth_numerics.py [--steps 400] [--out profiles/r4_fulldepth.md]
"""
import argparse
import copy
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BLOCKS = ["mixed_3b", "mixed_3c", "mixed_4b", "mixed_4c", "mixed_4d", "mixed_4e", "mixed_4f", "mixed_5b", "mixed_5c"]


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm()).item()


def _trained_model(steps):
    import math
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    b = 32
    args = get_args(argv=["--word2vec_path", "", "--vocab_size", "4000", "--batch_size", str(b), "--num_frames", "8",
                          "--video_size", "112", "--num_candidates", "2", "--lr", "1e-3", "--warmup_steps", "10"])
    ctx = pdist.DistContext(device=torch.device("cuda", 0))
    pdist.set_context(ctx)
    seed_everything(1, 0)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 1000)
    data = SyntheticClips(b, 8, 112, 2, args.max_words, args.vocab_size, num_classes=16, device=torch.device("cuda"))
    t0 = time.time()
    losses = []
    for i in range(steps):
        losses.append(float(tr.train_step(data.batch(i))))
        if i % 50 == 0:
            print(f"  train step {i} loss {losses[-1]:.3f} ({time.time() - t0:.0f} s)", flush=True)
    print(f"trained {steps} steps: first20 {sum(losses[:20]) / 20:.3f} last20 {sum(losses[-20:]) / 20:.3f} "
          f"(zero-logit level {math.log(2 * b):.3f})")
    return tr.model, data


def _mean_over_std(model, v, t):
    """|running mean| / sqrt(running var), median over channels, per BN of each block."""
    out = {}
    for n in BLOCKS:
        r = []
        for mod in getattr(model, n).modules():
            if isinstance(mod, torch.nn.BatchNorm3d):
                r.append((mod.running_mean.abs() / mod.running_var.clamp_min(1e-12).sqrt()).median().item())
        out[n] = (min(r), max(r)) if r else (0.0, 0.0)
    return out


def _block_errors(m, v, t, shift):
    from mil_nce_howto100m_amd import ops
    from mil_nce_howto100m_amd.ops import hip_ops
    hip_ops._BN_SHIFT = shift
    ref = copy.deepcopy(m).float().train()
    m_h = copy.deepcopy(m).train()
    m_bf = copy.deepcopy(m).train()
    io = {}
    hooks = [getattr(ref, n).register_forward_hook(
        lambda mod, i, o, n=n: io.__setitem__(n, i[0].detach())) for n in BLOCKS]
    with torch.no_grad(), ops.force_aten(keep_dtype=True):
        copy.deepcopy(ref)(v, t)  # (a copy, so ref's running statistics stay the trained ones; it carries the hooks)
    for h in hooks:
        h.remove()

    def block_run(blk, xin, g, aten, keep):
        x = xin.clone().requires_grad_(True)
        if aten:
            with ops.force_aten(keep_dtype=keep):
                o = blk(x)
                o.backward(g.to(o.dtype))
        else:
            o = blk(x)
            o.backward(g.to(o.dtype))
        grads = {k: p.grad.detach().clone() for k, p in blk.named_parameters() if p.grad is not None}
        for p in blk.parameters():
            p.grad = None
        return o.detach(), x.grad.detach(), grads

    def errs(res, rr):
        (o, dx, gp), (o_r, dx_r, gp_r) = res, rr
        flat = _rel(torch.cat([gp[k].reshape(-1) for k in sorted(gp_r)]),
                    torch.cat([gp_r[k].reshape(-1) for k in sorted(gp_r)]))
        worst = max(_rel(gp[k], gp_r[k]) for k in gp_r)
        return {"out": _rel(o, o_r), "dx": _rel(dx, dx_r), "flat": flat, "param": worst}

    torch.manual_seed(1)
    rows = {}
    for n in BLOCKS:
        x32 = io[n]
        xb = x32.to(torch.bfloat16)
        g = torch.randn(x32.shape[:-1] + (getattr(m, n).output_dim,), device="cuda")
        # fresh copies per block so the running statistics every path starts from are the trained ones
        r_ref = block_run(copy.deepcopy(getattr(ref, n)), xb.float(), g, True, True)
        r_hip = block_run(copy.deepcopy(getattr(m_h, n)), xb, g, False, False)
        r_bf = block_run(copy.deepcopy(getattr(m_bf, n)), xb, g, True, False)
        rows[n] = (errs(r_hip, r_ref), errs(r_bf, r_ref))
    hip_ops._BN_SHIFT = True
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from mil_nce_howto100m_amd.models import S3D
    torch.manual_seed(0)
    init = S3D(512, vocab_size=2000).cuda().train()
    trained, data = _trained_model(a.steps)
    # evaluation batch: 16 clips of the training distribution (a batch index never trained on)
    v = data.batch(10 ** 6)["video"][:16]
    t = torch.randint(0, 2000, (16, 20), device="cuda")
    lines = ["# S3D-G per-block numerics vs fp32 (teacher-forced), pre-BN shift on / off", "",
             "Generated by `tools/fulldepth_numerics.py` on one MI355X. Each Inception block gets the fp32",
             "ATen reference's own block input (bf16-rounded) and a random upstream gradient; relative L2",
             "errors against the fp32 block: `out` block output, `dx` input gradient, `flat` all parameter",
             "gradients concatenated, `param` the worst single parameter gradient. `aten-bf16` = the same",
             "ATen ops with bf16 activations (MIOpen bf16). 16 clips x 8 x 112^2 of the training distribution,",
             "train-mode BN (batch statistics; running statistics as trained).", ""]
    for label, model, txt in (("random init", init, t), (f"trained ({a.steps} Adam steps, structured synthetic)",
                                                          trained, t)):
        ms = _mean_over_std(model, v, txt)
        res = {s: _block_errors(model, v, txt, s) for s in (True, False)}
        lines += [f"## {label}", "",
                  "| block | BN median \\|rm\\|/std (min..max over BNs) | shift: out | dx | flat | param "
                  "| no shift: out | dx | flat | param | aten-bf16: out | dx | flat | param |",
                  "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
        worst = {s: {k: 0.0 for k in ("out", "dx", "flat", "param")} for s in ("shift", "plain", "aten")}
        for n in BLOCKS:
            (hs, bs), (hp, _) = res[True][n], res[False][n]
            lo, hi = ms[n]
            lines.append(f"| {n} | {lo:.2f}..{hi:.2f} | " + " | ".join(
                f"{d[k]:.4f}" for d in (hs, hp, bs) for k in ("out", "dx", "flat", "param")) + " |")
            for key, d in (("shift", hs), ("plain", hp), ("aten", bs)):
                for k in d:
                    worst[key][k] = max(worst[key][k], d[k])
        lines += ["", "worst over blocks: " + "; ".join(
            f"{key}: " + ", ".join(f"{k} {v_:.4f}" for k, v_ in w.items()) for key, w in worst.items()), ""]
        print("\n".join(lines[-(len(BLOCKS) + 5):]), flush=True)
    text = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main()
