#!/usr/bin/env python3
"""Per-layer conv timing of the flagship step: run the bench configuration for two training
steps (so every conv plan is autotuned exactly as in bench.py), then time each plan's forward,
dgrad and wgrad in isolation with the tuned kernel choices and print a table sorted by total
time -- which layers to attack next, and at what TF/s they run.

    python tools/conv_layers.py [--batch 256 --frames 16 --size 200]
"""
import argparse
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--size", type=int, default=200)
    o = ap.parse_args()
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.ops import hip_ops as h
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    ctx = pdist.init_distributed("nccl", "cuda")
    args = get_args(argv=["--batch_size", str(o.batch), "--num_frames", str(o.frames), "--video_size", str(o.size),
                          "--num_candidates", "4", "--word2vec_path", "", "--warmup_steps", "10000"])
    seed_everything(args.seed, 0)
    data = SyntheticClips(o.batch, o.frames, o.size, 4, args.max_words, args.vocab_size, device=ctx.device)
    tr = Trainer(args, build_model(args, ctx.device), ctx, len(data))
    for step in range(2):
        tr.train_step(data.batch(step))
    torch.cuda.synchronize()
    del tr, data
    gc.collect()
    torch.cuda.empty_cache()

    rows = []
    for key, plan in list(h._PLANS.items()):
        x_shape, w_shape, stride, pad, wo = key
        if plan.impl == 0 and plan.w_impl == 0:
            continue
        fl = 2.0 * plan.M * plan.Cout * plan.Ktot
        x = torch.randn(x_shape, device="cuda").to(torch.bfloat16)
        dy = torch.randn(plan.B, plan.To, plan.Ho, plan.Wo, plan.Cout, device="cuda").to(torch.bfloat16)
        w = torch.randn(w_shape, device="cuda") * 0.05
        tf = td = tw = 0.0
        stem = h._is_paired_stem(plan)
        if plan.impl and not stem:
            wp = h._pack(w, plan, 0)
            stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device="cuda")
            tf = timeit(lambda: h.conv_forward_raw(x, wp, plan, stats))
        if plan.d_impl and not stem and stride == (1, 1, 1):
            wd = h._pack(w, plan, 1)
            td = timeit(lambda: h.conv_dgrad(dy, wd, plan))
        if plan.w_impl:
            tw = timeit(lambda: h.conv_wgrad(dy, x, plan))
        rows.append((tf + td + tw, x_shape, w_shape, stride, fl, tf, td, tw,
                     f"f{plan.impl}/{plan.bn} d{plan.d_impl}/{plan.d_bn} w{plan.w_impl}/{plan.w_tn}x{plan.w_tk}"
                     f"/o{plan.w_occ}"))
        del x, dy, w
        torch.cuda.empty_cache()
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)

    def tfs(ms, fl):
        return f"{ms:6.3f} {fl / ms / 1e9:5.0f}" if ms else "     -     -"
    print(f"{len(rows)} conv plans, {tot:.2f} ms total (fwd + dgrad + wgrad in isolation)")
    print(f"{'x shape':>26s} {'w shape':>22s} {'GFLOP':>6s}  {'fwd ms TF/s':>12s} {'dgrad ms TF/s':>12s} "
          f"{'wgrad ms TF/s':>12s}  choice")
    for t, xs, ws, st, fl, tf, td, tw, ch in rows:
        print(f"{str(tuple(xs)):>26s} {str(tuple(ws)) + ('' if st == (1, 1, 1) else '/s' + ''.join(map(str, st))):>22s} "
              f"{fl / 1e9:6.0f}  {tfs(tf, fl)} {tfs(td, fl)} {tfs(tw, fl)}  {ch}", flush=True)
    pdist.destroy()


if __name__ == "__main__":
    main()
