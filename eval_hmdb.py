#!/usr/bin/env python3
"""HMDB-51 linear probe (reference ``eval_hmdb.py``); same CLI flags as training (config.py).

    python eval_hmdb.py --pretrain_cnn_path checkpoint/run1/epoch0150.pth.tar \\
        --eval_video_root <videos> --num_windows_test 10 --num_frames 32 --video_size 224

Process model: one rank per visible GPU (self-launched like ``main_distributed.py``, or under
torchrun); the feature extraction is sharded over the ranks and rank 0 reports. The CSV
defaults to the copy shipped in ``csv/`` next to this script (as the reference resolves it,
``eval_hmdb.py:40``). Real videos need ffmpeg and ``--eval_video_root``; without them the run
warns loudly and evaluates a synthetic labelled set.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def run(argv=None):
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.evaluation import eval_hmdb

    args = get_args(argv=argv)
    ctx = pdist.init_distributed(args.dist_backend, args.device)
    try:
        return eval_hmdb(args, ctx.device, ctx=ctx)
    finally:
        pdist.destroy()


def main(argv=None):
    from mil_nce_howto100m_amd.parallel.launch import run_per_gpu
    argv = sys.argv[1:] if argv is None else argv
    rc = run_per_gpu(__file__, argv, run)
    return rc if isinstance(rc, int) else 0


if __name__ == "__main__":
    sys.exit(main() or 0)
