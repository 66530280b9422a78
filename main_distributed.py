#!/usr/bin/env python3
"""MIL-NCE pretraining entry point, CLI-compatible with the reference ``main_distributed.py``.

    python main_distributed.py --batch_size 256 --num_frames 16 --video_size 200 \
        --num_candidates 4 --lr 0.001 --warmup_steps 10000 --epochs 150 --checkpoint_dir run1

Process model (replaces ``main_distributed.py:35-62`` / ``mp.spawn`` + UDP IP probe):
  * under ``torchrun``/``torch.distributed.run`` (``WORLD_SIZE`` set): one rank per process;
  * otherwise: one fresh process per visible GPU, started here with a 127.0.0.1 rendezvous
    before anything touches HIP (``parallel/launch.py``; the reference forces
    ``--multiprocessing-distributed`` the same way, ``:48``);
  * no GPU: single CPU process on gloo (the plumbing configuration).
``--batch_size`` is global per node and divided across ranks (``:88``). Data is the on-device
synthetic generator unless ``--synthetic 0`` (which needs ffmpeg + the HowTo100M files).
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def run(argv):
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import run_training

    args = get_args(argv=argv)
    if args.verbose and int(os.environ.get("RANK", "0")) == 0:
        print(args, flush=True)
    ctx = pdist.init_distributed(args.dist_backend, args.device, args.dist_timeout_s)
    args.rank, args.world_size = ctx.rank, ctx.world_size
    try:
        run_training(args, ctx)  # -e/--evaluate: HMDB probe every max(1, total_bs // 512) epochs
    finally:
        pdist.destroy()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if "WORLD_SIZE" in os.environ:
        return run(argv)
    # count GPUs without initialising HIP in this (parent) process, then start one fresh
    # child per GPU (parallel/launch.py) -- the parent never touches the device
    from mil_nce_howto100m_amd.parallel.launch import count_gpus_no_init, launch_local
    n = count_gpus_no_init()
    if n <= 1:
        return run(argv)
    return launch_local(os.path.abspath(__file__), argv, n)


if __name__ == "__main__":
    sys.exit(main() or 0)
