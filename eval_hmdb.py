#!/usr/bin/env python3
"""HMDB-51 linear probe (eval_hmdb.py); same CLI flags as training (config.py).

    python eval_hmdb.py --pretrain_cnn_path checkpoint/run1/epoch0150.pth.tar \
        --eval_video_root <videos> --num_windows_test 10 --num_frames 32 --video_size 224

Uses the real CSV + videos when ffmpeg and the files exist; otherwise it warns loudly and evaluates
a synthetic labelled set (an explicit --eval_csv that does not exist is an error).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.evaluation import eval_hmdb

    args = get_args(argv=argv)
    ctx = pdist.init_distributed(args.dist_backend, args.device)
    return eval_hmdb(args, ctx.device, ctx=ctx)


if __name__ == "__main__":
    main()
