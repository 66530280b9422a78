#!/usr/bin/env python3
"""MSR-VTT zero-shot retrieval (reference ``eval_msrvtt.py``).

    python eval_msrvtt.py --pretrain_cnn_path s3d_howto100m.pth --eval_video_root <videos> \\
        --num_windows_test 10 --num_frames 32 --video_size 224

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
    from mil_nce_howto100m_amd.train.evaluation import eval_retrieval

    args = get_args(argv=argv)
    ctx = pdist.init_distributed(args.dist_backend, args.device)
    try:
        return eval_retrieval(args, ctx.device, "msrvtt", ctx=ctx)
    finally:
        pdist.destroy()


def main(argv=None):
    from mil_nce_howto100m_amd.parallel.launch import run_per_gpu
    argv = sys.argv[1:] if argv is None else argv
    rc = run_per_gpu(__file__, argv, run)
    return rc if isinstance(rc, int) else 0


if __name__ == "__main__":
    sys.exit(main() or 0)
