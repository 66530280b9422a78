#!/usr/bin/env python3
"""Flagship benchmark: S3D-G + word2vec text tower, MIL-NCE, synthetic 16f x 200 x 200 clips,
num_candidates=4, bf16, 256 clips per GPU (BASELINE.json configs 2 and 3).

    python bench.py --gpus N --steps K --warmup W
    (or under python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

With WORLD_SIZE unset and N > 1 the script is its own launcher (reference
``main_distributed.py:57-60``): before anything touches HIP it starts N fresh child processes,
one per GPU, with the torchrun environment on 127.0.0.1 (``parallel/launch.py``). Every rank
checks that the process group it joined has exactly N ranks, and the JSON reports the world
size observed through ``torch.distributed``.

Each timed step is the full training step: on-device synthetic batch generation, forward of
both towers, cross-GPU all-gather of embeddings, MIL-NCE on the global batch, backward with
bucketed RCCL gradient all-reduce, fused Adam, LR schedule. Rank 0 prints ONE JSON line; the
value is the whole-job aggregate video-text pairs/s (max step time over ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _native_lib() -> str:
    """File name of the HIP kernel library this process loaded (there is no fallback path)."""
    from mil_nce_howto100m_amd.ops import _lib
    return os.path.basename(_lib.LIB_PATH)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch_per_gpu", type=int, default=256)
    ap.add_argument("--num_frames", type=int, default=16)
    ap.add_argument("--size", type=int, default=200)
    ap.add_argument("--num_candidates", type=int, default=4)
    ap.add_argument("--device", type=str, default="auto")
    ap.add_argument("--blocks", type=str, default="")
    ap.add_argument("--profile_steps", type=int, default=0, help="extra steps under torch profiler")
    ap.add_argument("--loss", type=str, default="milnce",
                    help="milnce (configs 2/3) | cdtw | sdtw_cidm | sdtw_negative | sdtw_3 (config 4)")
    ap.add_argument("--seq_len", type=int, default=8, help="clips per sequence for the soft-DTW losses")
    ap.add_argument("--grad_cache_chunks", type=int, default=-1,
                    help="GradCache micro-batches per GPU (config 5: 32f, 1024 clips/GPU)")
    ap.add_argument("--prefetch", type=int, default=0,
                    help="generate the next step's synthetic batch on a side stream during the current step "
                         "(same-box A/B: 4592 vs 4677 pairs/s without, profiles/r5_launch_merge.md)")
    ap.add_argument("--save_plan", type=str, default="",
                    help="write this run's kernel-plan decisions as a plan table (ops/tune_sync.py)")
    opts = ap.parse_args()

    if opts.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from mil_nce_howto100m_amd.parallel.launch import launch_local
        return launch_local(os.path.abspath(__file__), sys.argv[1:], opts.gpus)

    import torch
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything

    ctx = pdist.init_distributed("nccl", opts.device)
    observed = pdist.observed_world_size()
    if observed != opts.gpus or ctx.world_size != opts.gpus:
        print(f"error: --gpus {opts.gpus} but the process group has {observed} rank(s)", file=sys.stderr)
        pdist.destroy()
        return 2
    b = opts.batch_per_gpu
    args = get_args(argv=["--batch_size", str(b * ctx.world_size), "--num_frames", str(opts.num_frames),
                          "--video_size", str(opts.size), "--num_candidates", str(opts.num_candidates),
                          "--warmup_steps", "10000", "--lr", "0.001", "--epochs", "150",
                          "--word2vec_path", "", "--blocks", opts.blocks, "--loss", opts.loss,
                          "--seq_len", str(opts.seq_len), "--grad_cache_chunks", str(opts.grad_cache_chunks)])
    seed_everything(args.seed, ctx.rank)
    data = SyntheticClips(b, opts.num_frames, opts.size, opts.num_candidates, args.max_words, args.vocab_size,
                          seed=args.seed, device=ctx.device, rank=ctx.rank, world_size=ctx.world_size)
    if opts.loss != "milnce":
        from mil_nce_howto100m_amd.data.synthetic import SyntheticSequences
        assert b % opts.seq_len == 0, "batch_per_gpu must be a multiple of seq_len"
        data = SyntheticSequences(b // opts.seq_len, opts.seq_len, data)
    model = build_model(args, ctx.device)
    trainer = Trainer(args, model, ctx, len(data))
    cuda = ctx.device.type == "cuda"
    if cuda and opts.prefetch:
        # the next step's batch is generated on a side stream during the current step
        # (data/loader.py PrefetchedBatches; each timed step still generates one batch)
        from mil_nce_howto100m_amd.data.loader import PrefetchedBatches
        data = PrefetchedBatches(data, ctx.device)

    def sync():
        if cuda:
            torch.cuda.synchronize()

    # the steps run on a high-priority stream, as in the trainer's loop (utils/streams.py
    # MainStream; MILNCE_MAIN_PRIO=0 keeps the default stream)
    from mil_nce_howto100m_amd.utils import MainStream
    main_stream = MainStream(ctx.device)
    main_stream.__enter__()

    step = 0
    if opts.warmup == 0 and cuda:
        # setup, not a training step: one forward/backward so per-shape conv autotuning
        # (first use of each conv plan) does not land inside the timed region
        trainer.model.train()
        with trainer.tune_region():
            trainer.forward_loss(data.batch(0)).backward()
        trainer.bucketer.finish()
        trainer.bucketer.zero()
    for _ in range(opts.warmup):
        loss = trainer.train_step(data.batch(step))
        step += 1
    sync()
    pdist.barrier()
    sync()
    t0 = time.perf_counter()
    losses = []
    for _ in range(opts.steps):
        losses.append(trainer.train_step(data.batch(step)))
        step += 1
    sync()
    pdist.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt = pdist.all_reduce_max(dt)
    final_loss = float(losses[-1].item()) if losses else float("nan")
    # kernel plan of every rank (ops/tune_sync: rank 0 tunes, the others launch its choices)
    from mil_nce_howto100m_amd.ops import tune_sync
    hashes = [tune_sync.plan_hash()]
    if ctx.world_size > 1:
        hashes = [None] * ctx.world_size
        torch.distributed.all_gather_object(hashes, tune_sync.plan_hash())
    comm = None
    if ctx.world_size > 1:
        # after the timed region: the step's collectives alone at the step's sizes (xGMI record)
        from mil_nce_howto100m_amd.parallel.comm_probe import probe
        net = trainer.model.module if hasattr(trainer.model, "module") else trainer.model
        # packed [b video + b*K text] fp32 rows of the embedding width (models/s3dg.py fc)
        comm = probe(trainer.bucketer.flat.numel(), trainer.bucketer.buckets, b * (1 + opts.num_candidates),
                     net.fc.out_features, net.fc.weight.dtype, ctx.device)
    if opts.profile_steps and cuda:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
            for _ in range(opts.profile_steps):
                trainer.train_step(data.batch(step))
                step += 1
            sync()
        if ctx.is_main:
            os.makedirs("gpurun_out", exist_ok=True)
            with open("gpurun_out/torch_profile.txt", "w") as f:
                f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=80))
            # where the small ATen ops (adds, fills, reductions) come from
            with open("gpurun_out/torch_profile_stacks.txt", "w") as f:
                for e in prof.key_averages(group_by_stack_n=8):
                    if e.key.startswith(("aten::add", "aten::fill", "aten::zero", "aten::sum", "aten::copy",
                                         "aten::mul", "aten::mm", "aten::addmm", "aten::sub", "aten::div")):
                        f.write(f"{e.key} count={e.count} cuda_us={e.device_time_total:.0f}\n")
                        for fr in e.stack:
                            f.write(f"    {fr}\n")
    ms = 1000.0 * dt / max(1, opts.steps)
    pairs = b * ctx.world_size * opts.steps / dt
    if ctx.is_main:
        peak = torch.cuda.max_memory_allocated() / 2 ** 30 if cuda else 0.0
        out = {
            "metric": "video-text pairs/sec/node (S3D-G MIL-NCE train step)",
            "value": round(pairs, 2),
            "unit": "pairs/s",
            "n_gpus": observed,
            "steps": opts.steps,
            "warmup": opts.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if cuda else "fp32",
            "data": "synthetic (on-device generator, random-init weights)",
            "config": {"model": "S3D-G + word2vec text tower, " + ("MIL-NCE" if opts.loss == "milnce"
                                                                    else f"{opts.loss} (soft-DTW)"),
                       "global_batch": b * ctx.world_size,
                       # no token sequence in the MIL-NCE step; soft-DTW: clips per sequence
                       "seq_len": opts.seq_len if opts.loss != "milnce" else None,
                       "frames": opts.num_frames, "resolution": opts.size,
                       "num_candidates": opts.num_candidates,
                       "parallelism": f"dp{observed}",
                       "backend": ctx.backend,
                       "grad_cache_chunks": trainer.grad_cache_chunks()},
            "final_loss": round(final_loss, 4),
            "peak_mem_gib": round(peak, 2),
            "peak_reserved_gib": round(torch.cuda.max_memory_reserved() / 2 ** 30, 2) if cuda else 0.0,
        }
        out["plan_hash"] = hashes[0] if len(set(hashes)) == 1 else hashes
        # where the kernel plan came from: the shipped plan table (ops/plans/gfx950.json, valid for
        # these kernel sources) or first-use timing on this box
        out["plan"] = tune_sync.table_info()
        if cuda:
            from mil_nce_howto100m_amd.ops import hip_ops
            # launches whose tuned variant could not run in the call (0: every forward / dgrad call
            # context was tuned on its own) and the side-stream memory rule's per-step decisions
            out["plan"].update(hip_ops.plan_events())
            out["side_stream"] = dict(hip_ops._HEADROOM_STATS)
        if opts.save_plan:
            out["plan"]["saved"] = tune_sync.save_table(opts.save_plan)
        if comm is not None:
            out["comm"] = comm
            if getattr(trainer, "comm_plan", None) is not None:  # --bucket_mb auto (parallel/bucket_plan.py)
                out["comm"]["bucket_plan"] = trainer.comm_plan.as_dict()
        if cuda:
            out["kernel_lib"] = _native_lib()
            out["main_stream_priority"] = main_stream.priority
        print(json.dumps(out), flush=True)
    main_stream.__exit__(None, None, None)
    pdist.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
