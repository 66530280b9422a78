#!/usr/bin/env python3
"""Per-layer conv kernel timing for the flagship config (run on the GPU box).

Runs one training step to populate the conv plan cache, then times the forward (with BN
statistics epilogue), dgrad and wgrad kernels of every distinct conv shape in isolation and
prints achieved TFLOP/s. Usage: python tools/conv_bench.py [--batch 256] [--frames 16] [--size 200]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--size", type=int, default=200)
    o = ap.parse_args()
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.ops import hip_ops
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model

    ctx = pdist.init_distributed("nccl", "auto")
    args = get_args(argv=["--batch_size", str(o.batch), "--num_frames", str(o.frames), "--video_size", str(o.size),
                          "--word2vec_path", ""])
    data = SyntheticClips(o.batch, o.frames, o.size, 4, args.max_words, args.vocab_size, device=ctx.device)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 100)
    tr.train_step(data.batch(0))
    torch.cuda.synchronize()
    print("plans as tuned inside the training step:")
    for key, plan in sorted(hip_ops._PLANS.items(), key=lambda kv: -kv[1].M * kv[1].Cout * kv[1].Ktot):
        print(f"  {key[0]}->{plan.Cout} k{plan.k}: fwd impl {plan.impl} dgrad {plan.d_impl} wgrad {plan.w_impl} "
              f"(tn {plan.w_tn})", flush=True)
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    flops_tot = 0.0
    print(f"{'shape (B,T,H,W,Cin)->Cout k s':58s} {'GFLOP':>7s} {'fwd ms':>7s} {'TF/s':>6s} {'dgr ms':>7s} "
          f"{'TF/s':>6s} {'wgr ms':>7s} {'TF/s':>6s}")
    for key, plan in sorted(hip_ops._PLANS.items(), key=lambda kv: -kv[1].M * kv[1].Cout * kv[1].Ktot):
        plan.pin_f = plan.pin_d = plan.w_impl = 0
    plan.ctx.clear()  # re-tune on these operands
        xs, ws, s, p, _wo = key
        u8 = plan.Cin % 8 != 0
        x = (torch.randint(0, 255, xs, dtype=torch.uint8, device="cuda") if u8
             else torch.randn(xs, device="cuda").to(torch.bfloat16))
        w = torch.randn(ws, device="cuda") * 0.05
        wp = hip_ops._pack(w, plan, 0)
        stats = torch.empty((hip_ops._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), dtype=torch.float32, device="cuda")
        fl = 2.0 * plan.M * plan.Cout * plan.k[0] * plan.k[1] * plan.k[2] * plan.Cin_p
        t_f = timeit(lambda: hip_ops.conv_forward_raw(x, wp, plan, stats))
        dy = torch.randn((plan.B, plan.To, plan.Ho, plan.Wo, plan.Cout), device="cuda").to(torch.bfloat16)
        t_d = float("nan")
        if plan.s == (1, 1, 1):
            wd = hip_ops._pack(w, plan, 1)
            t_d = timeit(lambda: hip_ops.conv_dgrad(dy, wd, plan))
        t_w = timeit(lambda: hip_ops.conv_wgrad(dy, x, plan))
        tot["fwd"] += t_f
        tot["dgrad"] += 0 if t_d != t_d else t_d
        tot["wgrad"] += t_w
        flops_tot += fl
        desc = f"{xs}->{plan.Cout} k{plan.k} s{plan.s[1]}"
        print(f"{desc:58s} {fl / 1e9:7.1f} {t_f:7.3f} {fl / t_f / 1e9:6.0f} {t_d:7.3f} {fl / t_d / 1e9:6.0f} "
              f"{t_w:7.3f} {fl / t_w / 1e9:6.0f}  impl f{plan.impl} d{plan.d_impl} w{plan.w_impl}", flush=True)
    print(f"TOTAL fwd {tot['fwd']:.2f} ms  dgrad {tot['dgrad']:.2f} ms  wgrad {tot['wgrad']:.2f} ms  "
          f"(fwd FLOP {flops_tot / 1e12:.2f} T -> {flops_tot / tot['fwd'] / 1e9:.0f} TF/s)")


if __name__ == "__main__":
    main()
