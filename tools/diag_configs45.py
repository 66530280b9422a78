#!/usr/bin/env python3
"""Loss of BASELINE configs 4/5 at their bench shapes: HIP path vs ATen/MIOpen path on the same
weights and batch (train-mode BN, forward only), and the spread of the random-init loss over
weight seeds. Explains the final_loss values bench.py prints for these configs (they are the
random-init loss: with the 10k-step LR warmup the few timed Adam steps barely move the weights).

    python tools/diag_configs45.py [--seeds 3] [--c5_batch 64]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=3)
    ap.add_argument("--c5_batch", type=int, default=64)
    o = ap.parse_args()
    from mil_nce_howto100m_amd import ops
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips, SyntheticSequences
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    ctx = pdist.init_distributed("nccl", "cuda")
    dev = ctx.device
    cfgs = {
        "config4 sdtw_3 128 clips 16x200^2": (["--batch_size", "128", "--num_frames", "16", "--video_size", "200",
                                                "--num_candidates", "4", "--loss", "sdtw_3", "--seq_len", "8"],
                                               lambda a: SyntheticSequences(16, 8, SyntheticClips(
                                                   128, 16, 200, 4, a.max_words, a.vocab_size, device=dev)).batch(0), 0),
        f"config5 milnce {o.c5_batch} clips 32x200^2 gradcache 4": (
            ["--batch_size", str(o.c5_batch), "--num_frames", "32", "--video_size", "200", "--num_candidates", "4",
             "--grad_cache_chunks", "4"],
            lambda a: SyntheticClips(o.c5_batch, 32, 200, 4, a.max_words, a.vocab_size, device=dev).batch(0), 4),
    }
    for name, (extra, mk, chunks) in cfgs.items():
        for seed in range(1, o.seeds + 1):
            vals = []
            for aten in (False, True):
                args = get_args(argv=["--word2vec_path", "", "--warmup_steps", "10000", *extra])
                seed_everything(seed, 0)
                tr = Trainer(args, build_model(args, dev), ctx, 100)
                batch = mk(args)
                tr.model.train()
                with torch.no_grad(), (ops.force_aten() if aten else torch.enable_grad()):
                    if chunks > 1:
                        b = batch["video"].shape[0]
                        vs, ts = [], []
                        for i in range(chunks):
                            s, e = i * b // chunks, (i + 1) * b // chunks
                            v, t = tr.model(batch["video"][s:e], batch["text"][s:e].reshape(-1, batch["text"].shape[-1]))
                            vs.append(v)
                            ts.append(t)
                        loss = tr._loss(batch, torch.cat(vs).float(), torch.cat(ts).float())
                        vn = torch.cat(vs).float().norm(dim=1).mean()
                    else:
                        loss = tr.forward_loss(batch)
                        vn = torch.tensor(float("nan"))
                torch.cuda.synchronize()
                vals.append((float(loss), float(vn)))
                del tr
                torch.cuda.empty_cache()
            print(f"{name} seed {seed}: loss hip {vals[0][0]:.4f} aten {vals[1][0]:.4f} "
                  f"(|v| hip {vals[0][1]:.2f} aten {vals[1][1]:.2f})", flush=True)


if __name__ == "__main__":
    main()
