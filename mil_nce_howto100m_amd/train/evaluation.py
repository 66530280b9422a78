"""Evaluation drivers shared by ``eval_hmdb.py``, ``eval_msrvtt.py``, ``eval_youcook.py`` and the
in-training HMDB probe (``main_distributed.py:188-189, 243-287`` — dead code in the reference
because ``test_loader`` is undefined; wired up here).

Model loading follows ``eval_hmdb.py:21-36``: a training checkpoint (``{"state_dict": ...}``,
``module.``-prefixed) builds the standard model; a plain dict (the public S3D_HowTo100M
weights) builds the space-to-depth variant. The checkpoint path comes from
``--pretrain_cnn_path`` (the reference hard-codes ``./checkpoint/epoch0089.pth.tar`` and
``./checkpoint/s3d_howto100m.pth``, §2.10 item 10). Data: the real CSV-driven datasets when
ffmpeg and the videos exist, else the synthetic labelled set (pipeline validation only).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..data.datasets import HMDBDataset, Tokenizer, WindowedClipDataset, ffmpeg_available, to_model_layout
from ..data.synthetic import SyntheticEvalSet
from ..eval import extract_features, format_metrics, linear_probe
from ..eval.retrieval import evaluate_retrieval
from ..models import S3D
from . import checkpoint as ckpt


def load_eval_model(args, device) -> S3D:
    path = args.pretrain_cnn_path
    sd = ckpt.load_checkpoint(path) if path else None
    if sd is not None and "state_dict" not in sd:
        model = S3D(args.num_class, space_to_depth=True, word2vec_path="", vocab_size=args.vocab_size)
        ckpt.load_model_weights(model, sd, strict=True)
    else:
        model = S3D(args.num_class, space_to_depth=False, word2vec_path="", vocab_size=args.vocab_size)
        if sd is not None:
            ckpt.load_model_weights(model, sd["state_dict"], strict=True)
    return model.to(device).eval()


def _native(b):
    b = dict(b)
    b["video"] = to_model_layout(b["video"])
    return b


def _sharded_batches(ds, batch_size, workers, rank, world):
    """Only this rank's batches are ever decoded (eval/sharding.py sharded_loader)."""
    from ..eval.sharding import sharded_loader
    return sharded_loader(ds, batch_size, workers, rank, world, convert=_native)


# the eval CSVs shipped with the repository (csv/, from the reference's csv/): the default when
# --eval_csv is not given, resolved next to the package rather than against the cwd
CSV_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "csv")


def default_csv(name: str) -> str:
    return os.path.join(CSV_DIR, name)


def _use_real(csv: str, root: str) -> bool:
    return bool(csv) and os.path.isfile(csv) and os.path.isdir(root) and ffmpeg_available()


def _synthetic_fallback(args, csv: str, what: str) -> None:
    """No CSV / videos / ffmpeg: an explicitly requested eval CSV is an error; otherwise the
    synthetic labelled set runs (pipeline check only) with a loud warning."""
    missing = [m for m, ok in (("CSV " + repr(csv), bool(csv) and os.path.isfile(csv)),
                               ("video root " + repr(args.eval_video_root), os.path.isdir(args.eval_video_root)),
                               ("ffmpeg", ffmpeg_available())) if not ok]
    if getattr(args, "eval_csv", ""):
        raise FileNotFoundError(f"{what} eval: --eval_csv given but missing: {', '.join(missing)}")
    import warnings
    msg = (f"{what} eval is running on SYNTHETIC clips (missing: {', '.join(missing)}); the numbers only check "
           f"the pipeline, they are not {what} results")
    warnings.warn(msg, RuntimeWarning, stacklevel=3)
    print("WARNING: " + msg, flush=True)


def _graph_env(args) -> None:
    os.environ["MILNCE_EVAL_GRAPHS"] = "1" if getattr(args, "hip_graph", 1) else "0"


def _rank_world(ctx):
    return (ctx.rank, ctx.world_size) if ctx is not None else (0, 1)


def eval_hmdb(args, device, model: Optional[S3D] = None, ctx=None) -> dict:
    """HMDB linear probe; with a multi-rank ``ctx`` the feature extraction is sharded over the
    ranks (one process per GPU) and rank 0 reports."""
    model = model or load_eval_model(args, device)
    rank, world = _rank_world(ctx)
    _graph_env(args)
    csv = getattr(args, "eval_csv", "") or default_csv("hmdb51.csv")
    if _use_real(csv, args.eval_video_root):
        ds = HMDBDataset(csv, args.eval_video_root, args.num_windows_test, args.num_frames, args.video_size)
        batches = _sharded_batches(ds, args.batch_size_val, max(0, args.num_thread_reader), rank, world)
    else:
        _synthetic_fallback(args, csv, "HMDB")
        batches = SyntheticEvalSet(getattr(args, "synthetic_eval_videos", 96), args.num_windows_test,
                                   args.num_frames, args.video_size, device=device).batches(args.batch_size_val)
    feats, labels, splits = extract_features(model, batches, device, rank, world)
    res = linear_probe(feats, labels, splits, C=100.0) if rank == 0 else {}
    for k in (1, 2, 3):
        if f"split{k}" in res:
            print("Top 1 accuracy split {} and C {} : {}".format(k, 100.0, res[f"split{k}"]), flush=True)
    return res


def eval_retrieval(args, device, kind: str, model: Optional[S3D] = None, ctx=None) -> dict:
    model = model or load_eval_model(args, device)
    rank, world = _rank_world(ctx)
    _graph_env(args)
    csv = getattr(args, "eval_csv", "") or default_csv("msrvtt_test.csv" if kind == "msrvtt"
                                                       else "validation_youcook.csv")
    tok = Tokenizer(args.token_to_word_path, max_words=30)
    if _use_real(csv, args.eval_video_root):
        ds = WindowedClipDataset(csv, args.eval_video_root, tok, args.num_windows_test, args.fps, args.num_frames,
                                 args.video_size, kind)
        batches = _sharded_batches(ds, args.batch_size_val, max(0, args.num_thread_reader), rank, world)
    else:
        _synthetic_fallback(args, csv, kind)
        batches = SyntheticEvalSet(getattr(args, "synthetic_eval_videos", 96), args.num_windows_test,
                                   args.num_frames, args.video_size, device=device).batches(args.batch_size_val)
    m = evaluate_retrieval(model, batches, device, rank, world)
    if rank == 0:
        print(format_metrics(m), flush=True)
    return m


def evaluate_hmdb_during_training(args, ctx, model: Optional[S3D] = None) -> Optional[dict]:
    """HMDB probe of the model being trained (``main_distributed.py:188-189``, run every
    ``max(1, total_bs // 512)`` epochs before the epoch's training). Feature extraction is
    sharded over all ranks; rank 0 fits the probe. The model is left in eval mode; the next
    training step switches it back."""
    res = eval_hmdb(args, ctx.device, model=model, ctx=ctx)
    return res if ctx.is_main else None
