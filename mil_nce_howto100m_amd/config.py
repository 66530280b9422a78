"""Command-line configuration.

One parser replaces the reference's two copied files (``args.py:3-52`` and
``args_small.py:3-52``). Every one of the reference's 45 flags is accepted with the same
name, default and ``dest`` (including the ``--momemtum`` typo, ``args.py:20``), so an
existing ``python main_distributed.py ...`` command line keeps working. New flags for
the MI355X build (dtype, synthetic data, loss family, distributed knobs) are grouped
separately. ``--preset small`` reproduces ``args_small.py``'s defaults.
"""
from __future__ import annotations

import argparse
from typing import Optional, Sequence

# args_small.py differs from args.py only in these defaults (args_small.py:5,17,21,28,34,36).
SMALL_PRESET = dict(
    train_csv="csv/small_videos.csv",
    batch_size=12,
    n_display=100,
    warmup_steps=1000,
    epochs=100,
    lr=0.001,
)


def _bucket_mb(v):
    """--bucket_mb: a size in MiB, or "auto" (parallel/bucket_plan.py)."""
    if str(v).lower() == "auto":
        return "auto"
    f = float(v)
    if f <= 0:
        raise argparse.ArgumentTypeError("--bucket_mb must be > 0 or auto")
    return f


def build_parser(description: str = "MILNCE") -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=description)
    # ---- reference flags (args.py:5-49), same names/defaults/dests ----
    p.add_argument("--train_csv", type=str, default="../HowTo100M/csv/new_videos.csv", help="train csv")
    p.add_argument("--video_path", type=str, default="../HowTo100M/videos", help="video_path")
    p.add_argument("--caption_root", type=str, default="../HowTo100M/caption_json", help="caption json root")
    p.add_argument("--checkpoint_root", type=str, default="checkpoint", help="checkpoint dir root")
    p.add_argument("--log_root", type=str, default="log", help="log dir root")
    p.add_argument("--eval_video_root", type=str, default="../HowTo100M/downstream", help="eval video root")
    p.add_argument("--checkpoint_dir", type=str, default="", help="checkpoint model folder")
    p.add_argument("--optimizer", type=str, default="adam", help="adam | sgd")
    p.add_argument("--weight_init", type=str, default="uniform", help="uniform | kaiming_normal")
    p.add_argument("--num_thread_reader", type=int, default=20, help="data loader workers (global)")
    p.add_argument("--num_class", type=int, default=512, help="embedding dim")
    p.add_argument("--num_candidates", type=int, default=5, help="num candidates for MILNCE loss")
    p.add_argument("--batch_size", type=int, default=128, help="batch size (global, per node)")
    p.add_argument("--num_windows_test", type=int, default=4, help="number of testing windows")
    p.add_argument("--batch_size_val", type=int, default=32, help="batch size eval")
    p.add_argument("--momemtum", type=float, default=0.9, help="SGD momentum (sic, args.py:20)")
    p.add_argument("--n_display", type=int, default=400, help="Information display frequency")
    p.add_argument("--num_frames", type=int, default=32, help="frames per clip")
    p.add_argument("--video_size", type=int, default=224, help="clip height/width")
    p.add_argument("--crop_only", type=int, default=1, help="random crop without resize")
    p.add_argument("--centercrop", type=int, default=0, help="center crop")
    p.add_argument("--random_flip", type=int, default=1, help="random horizontal flip")
    p.add_argument("--verbose", type=int, default=1, help="")
    p.add_argument("--warmup_steps", type=int, default=50000, help="")
    p.add_argument("--min_time", type=float, default=5.0, help="")
    p.add_argument("--pretrain_cnn_path", type=str, default="", help="plain S3D state_dict to init from")
    p.add_argument("--word2vec_path", type=str, default="../HowTo100M/data/word2vec.pth", help="")
    p.add_argument("--fps", type=int, default=10, help="")
    p.add_argument("--cudnn_benchmark", type=int, default=0, help="accepted for CLI compatibility")
    p.add_argument("--epochs", default=300, type=int, metavar="N", help="number of total epochs to run")
    p.add_argument("--start-epoch", default=0, type=int, metavar="N", help="manual epoch number")
    p.add_argument("--lr", "--learning-rate", default=0.001, type=float, metavar="LR", dest="lr")
    p.add_argument("--momentum", default=0.9, type=float, metavar="M", help="unused (see --momemtum)")
    p.add_argument("--resume", dest="resume", action="store_true", help="resume from last checkpoint")
    p.add_argument("-e", "--evaluate", dest="evaluate", action="store_true", help="evaluate (HMDB linear probe)")
    p.add_argument("--pretrained", dest="pretrained", action="store_true", help="unused")
    p.add_argument("--pin_memory", dest="pin_memory", action="store_true", help="use pin_memory")
    p.add_argument("--world-size", default=-1, type=int, help="number of nodes")
    p.add_argument("--rank", default=-1, type=int, help="node rank")
    p.add_argument("--dist-file", default="dist-file", type=str, help="unused")
    p.add_argument("--dist-url", default="env://", type=str, help="rendezvous url (env:// or tcp://host:port)")
    p.add_argument("--dist-backend", default="nccl", type=str, help="nccl (=RCCL on ROCm) | gloo")
    p.add_argument("--seed", default=1, type=int, help="seed (propagated to every rank)")
    p.add_argument("--gpu", default=None, type=int, help="GPU id to use")
    p.add_argument("--multiprocessing-distributed", action="store_true", help="spawn one process per GPU")

    # ---- MI355X-native additions ----
    g = p.add_argument_group("mi355x")
    g.add_argument("--preset", type=str, default="", help="'' | small (args_small.py defaults)")
    g.add_argument("--device", type=str, default="auto", help="auto | cuda | cpu")
    g.add_argument("--dtype", type=str, default="bf16", help="activation/compute dtype on GPU: bf16")
    g.add_argument("--synthetic", type=int, default=1, help="1: on-device synthetic clips (no ffmpeg)")
    g.add_argument("--synthetic_len", type=int, default=1238911, help="samples per synthetic epoch (README.md:64)")
    g.add_argument("--steps_per_epoch", type=int, default=0, help="cap steps per epoch (0: full epoch)")
    g.add_argument("--max_words", type=int, default=20, help="words per caption (video_loader.py:28)")
    g.add_argument("--vocab_size", type=int, default=66250, help="word2vec vocabulary (s3dg.py:153)")
    g.add_argument("--token_to_word_path", type=str, default="", help="dict.npy (optional)")
    g.add_argument("--loss", type=str, default="milnce", help="milnce | cdtw | sdtw_cidm | sdtw_negative | sdtw_3")
    g.add_argument("--seq_len", type=int, default=8, help="clips per sequence for soft-DTW losses")
    g.add_argument("--grad_scale", type=str, default="reference",
                   help="reference: reproduce the 1/world_size gradient scale (utils.py:19-24 + DDP mean); "
                        "exact: full-batch gradient")
    g.add_argument("--bucket_mb", type=_bucket_mb, default="auto",
                   help="gradient all-reduce bucket size (MiB), or auto: sized from the all-reduce cost "
                        "measured on the process group at start-up (parallel/bucket_plan.py)")
    g.add_argument("--grad_comm_dtype", type=str, default="fp32", choices=("fp32", "bf16"),
                   help="gradient all-reduce wire dtype (bf16 halves the bytes, sums in bf16)")
    g.add_argument("--emb_gather", type=str, default="rccl", choices=("rccl", "peer"),
                   help="MIL-NCE negatives all-gather: RCCL ring, or one-shot xGMI peer writes (same node)")
    g.add_argument("--broadcast_buffers", type=int, default=1, help="broadcast BN buffers from rank 0 each step")
    g.add_argument("--blocks", type=str, default="", help="comma list of inception blocks to keep (plumbing)")
    g.add_argument("--log_jsonl", type=str, default="", help="also write metrics as JSON lines here")
    g.add_argument("--dist_timeout_s", type=int, default=1800, help="collective watchdog timeout")
    g.add_argument("--ckpt_every_steps", type=int, default=0, help="extra mid-epoch checkpoint interval")
    g.add_argument("--eval_csv", type=str, default="", help="eval CSV (csv/hmdb51.csv, msrvtt_test.csv, ...)")
    g.add_argument("--synthetic_eval_videos", type=int, default=96, help="videos in the synthetic eval set")
    g.add_argument("--stop_epoch", type=int, default=0,
                   help="end this run after this epoch (simulated interruption for resume tests)")
    g.add_argument("--hip_graph", type=int, default=1,
                   help="replay evaluation forwards from captured HIP graphs (launch-bound at small batch)")
    g.add_argument("--grad_cache_chunks", type=int, default=-1,
                   help="GradCache-style step in this many micro-batches per GPU: exact global-negative "
                        "MIL-NCE with bounded activation memory; 0/1: off (the reference's one-shot step); "
                        "-1 (default): one-shot whenever the step's activations fit the GPU's memory "
                        "(BASELINE config 5, 1024 x 32f clips, fits 288 GB one-shot), else the fewest chunks that fit")
    g.add_argument("--watchdog_s", type=float, default=0.0,
                   help="abort a rank (exit 3, stacks dumped) after this many seconds without a finished step")
    g.add_argument("--phase_timers", type=int, default=0,
                   help="HIP-event timers per step phase, reported in the JSONL metrics")
    g.add_argument("--fault_at_step", type=int, default=-1,
                   help="fault injection: raise on this global step (tests kill-and-resume)")
    g.add_argument("--verify_buckets", type=int, default=0,
                   help="debug: check every gradient bucket is unchanged between its all-reduce launch and "
                        "the end of backward (comm/compute ordering verifier; 2 extra gradient copies)")
    return p


def get_args(description: str = "MILNCE", argv: Optional[Sequence[str]] = None) -> argparse.Namespace:
    """Parse the CLI. Mirrors ``args.py:get_args`` (``args.py:3``)."""
    parser = build_parser(description)
    args = parser.parse_args(argv)
    if args.preset == "small":
        # Apply args_small.py defaults only where the user did not pass a value.
        defaults = parser.parse_args([])
        for k, v in SMALL_PRESET.items():
            if getattr(args, k) == getattr(defaults, k):
                setattr(args, k, v)
    return args
