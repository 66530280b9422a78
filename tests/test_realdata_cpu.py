"""Real-data pipeline on CPU: HowTo100M feed with a fake decoder, the
rank sampler, the reference's eval CSVs, and CDTW with several sequences per rank.

ffmpeg is not in this image, so ``decode_clip`` is replaced (inside each rank process) by a
deterministic function of (path, seek, flip); everything else -- CSV, caption JSON, nearest-
candidate captions, tokenizer, sampler, DataLoader, device layout, trainer, checkpoints -- is the
production path.
"""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REF_CSV = "/root/reference/csv"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_decode(path, size, fps=None, start=None, duration=None, crop_only=False, center_crop=True, hflip=False,
                 rng=None):
    h = (sum(map(ord, os.path.basename(path))) * 31 + int(start or 0) * 7 + int(hflip)) % 251
    n = int(round((duration or 1.0) * (fps or 10)))
    t = np.arange(n, dtype=np.int64).reshape(n, 1, 1, 1)
    y = np.arange(size, dtype=np.int64).reshape(1, size, 1, 1)
    c = np.arange(3, dtype=np.int64).reshape(1, 1, 1, 3)
    return ((h + t * 5 + y * 3 + c * 40) % 256).astype(np.uint8) * np.ones((1, 1, size, 1), np.uint8)


def _fixture(d, n_videos=5):
    os.makedirs(os.path.join(d, "videos"))
    os.makedirs(os.path.join(d, "captions"))
    words = ["cut", "the", "onion", "add", "salt", "stir", "pan", "oil", "heat", "serve"]
    rows = []
    for v in range(n_videos):
        name = f"vid{v}.mp4"
        open(os.path.join(d, "videos", name), "wb").close()
        k = 6 + v
        cap = {"start": [2.0 * i for i in range(k)], "end": [2.0 * i + 1.5 for i in range(k)],
               "text": [" ".join(words[(v + i + j) % len(words)] for j in range(4)) for i in range(k)]}
        with open(os.path.join(d, "captions", f"vid{v}.json"), "w") as f:
            json.dump(cap, f)
        rows.append(name)
    with open(os.path.join(d, "train.csv"), "w") as f:
        f.write("video_path\n" + "\n".join(rows) + "\n")
    np.save(os.path.join(d, "dict.npy"), np.array(words))
    return d


def _args(d, ck, extra=()):
    from mil_nce_howto100m_amd.config import get_args
    return get_args(argv=["--synthetic", "0", "--train_csv", os.path.join(d, "train.csv"),
                          "--video_path", os.path.join(d, "videos"), "--caption_root", os.path.join(d, "captions"),
                          "--token_to_word_path", os.path.join(d, "dict.npy"), "--batch_size", "2",
                          "--num_frames", "4", "--video_size", "32", "--fps", "4", "--num_candidates", "2",
                          "--blocks", "mixed_3b", "--warmup_steps", "1", "--word2vec_path", "", "--vocab_size", "50",
                          "--num_thread_reader", "0", "--checkpoint_root", ck, "--checkpoint_dir", "run",
                          "--log_root", ck, "--n_display", "1", "--verbose", "0", "--epochs", "2", *extra])


def _worker(rank, world, port, d, ck, extra):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from mil_nce_howto100m_amd.data import datasets
    datasets.decode_clip = _fake_decode
    datasets.ffmpeg_available = lambda: True
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import run_training
    ctx = pdist.init_distributed("gloo", "cpu")
    try:
        run_training(_args(d, ck, extra), ctx)
    finally:
        dist.destroy_process_group()


def test_real_data_training_two_ranks_and_resume():
    """2 gloo ranks, 2 epochs over a 5-video HowTo100M fixture (per-rank batch 1, 3 steps per
    epoch); a run stopped after epoch 1 and resumed lands on the uninterrupted run's state."""
    from mil_nce_howto100m_amd.train import checkpoint as ck
    with tempfile.TemporaryDirectory() as d, tempfile.TemporaryDirectory() as c1, \
            tempfile.TemporaryDirectory() as c2:
        _fixture(d)
        mp.spawn(_worker, args=(2, _port(), d, c1, ()), nprocs=2)
        mp.spawn(_worker, args=(2, _port(), d, c2, ("--stop_epoch", "1")), nprocs=2)
        assert os.path.isfile(os.path.join(c2, "run", "epoch0001.pth.tar"))
        mp.spawn(_worker, args=(2, _port(), d, c2, ("--resume",)), nprocs=2)
        a = ck.load_checkpoint(os.path.join(c1, "run", "epoch0002.pth.tar"))
        b = ck.load_checkpoint(os.path.join(c2, "run", "epoch0002.pth.tar"))
        assert a["scheduler"]["last_epoch"] == b["scheduler"]["last_epoch"] == 6
        for k in a["state_dict"]:
            assert torch.allclose(a["state_dict"][k].float(), b["state_dict"][k].float(), atol=1e-6), k


def test_real_data_mid_epoch_resume_skips_seen_batches():
    """Mid-epoch step checkpoint + resume continues at the next unseen batch of the same epoch."""
    from mil_nce_howto100m_amd.train import checkpoint as ck
    with tempfile.TemporaryDirectory() as d, tempfile.TemporaryDirectory() as c1, \
            tempfile.TemporaryDirectory() as c2:
        _fixture(d)
        mp.spawn(_worker, args=(2, _port(), d, c1, ()), nprocs=2)
        with pytest.raises(Exception):
            mp.spawn(_worker, args=(2, _port(), d, c2, ("--ckpt_every_steps", "1", "--fault_at_step", "4")), nprocs=2)
        mid = ck.load_checkpoint(ck.get_last_checkpoint(os.path.join(c2, "run")))
        assert mid["epoch"] == 1 and mid["step_in_epoch"] == 1
        mp.spawn(_worker, args=(2, _port(), d, c2, ("--resume",)), nprocs=2)
        a = ck.load_checkpoint(os.path.join(c1, "run", "epoch0002.pth.tar"))
        b = ck.load_checkpoint(os.path.join(c2, "run", "epoch0002.pth.tar"))
        for k in a["state_dict"]:
            assert torch.allclose(a["state_dict"][k].float(), b["state_dict"][k].float(), atol=1e-6), k


def test_epoch_rank_sampler_shards():
    from mil_nce_howto100m_amd.data.loader import EpochRankSampler
    n, world = 12, 3
    shards = [list(EpochRankSampler(n, r, world, seed=7)) for r in range(world)]
    assert sorted(i for s in shards for i in s) == list(range(n))  # disjoint and complete
    s = EpochRankSampler(n, 1, world, seed=7)
    e0 = list(s)
    s.set_epoch(1)
    assert list(s) != e0 and sorted(s) == sorted(set(s))  # reshuffled per epoch
    s.set_start(2)
    assert list(s) == s.indices()[2:] and len(s) == 2
    padded = [list(EpochRankSampler(10, r, 4)) for r in range(4)]
    assert all(len(p) == 3 for p in padded)  # DistributedSampler padding: ceil(10 / 4)


def test_howto100m_items_deterministic_per_epoch_and_index(monkeypatch):
    from mil_nce_howto100m_amd.data import datasets
    monkeypatch.setattr(datasets, "decode_clip", _fake_decode)
    with tempfile.TemporaryDirectory() as d:
        _fixture(d)
        tok = datasets.Tokenizer(os.path.join(d, "dict.npy"), max_words=20)
        ds = datasets.HowTo100MDataset(os.path.join(d, "train.csv"), os.path.join(d, "videos"),
                                       os.path.join(d, "captions"), tok, num_frames=4, size=32, fps=4,
                                       num_candidates=3, seed=3)
        a, b = ds[2], ds[2]
        assert torch.equal(a["video"], b["video"]) and torch.equal(a["text"], b["text"])
        assert a["video"].shape == (4, 32, 32, 3) and a["text"].shape == (3, 20)
        assert (a["text"][:, 0] > 0).all()  # every candidate caption tokenised
        ds.set_epoch(1)
        draws = {(int(ds[i]["video"].float().sum()), tuple(ds[i]["text"][0].tolist())) for i in range(5)}
        assert len(draws) > 1


@pytest.mark.skipif(not os.path.isdir(REF_CSV), reason="reference CSVs not present")
def test_reference_eval_csvs_parse():
    """The reference's own eval CSVs through our datasets."""
    from mil_nce_howto100m_amd.data.datasets import HMDBDataset, Tokenizer, WindowedClipDataset
    hm = HMDBDataset(os.path.join(REF_CSV, "hmdb51.csv"), "/nonexistent")
    assert len(hm) == 6766
    meta = [hm.meta(i) for i in range(len(hm))]
    labels = {m[0] for m in meta}
    assert len(labels) == 51 and not any(lab.endswith("_test") for lab in labels)
    s1 = [m[1] for m in meta]
    assert (s1.count(1), s1.count(2), s1.count(0)) == (3570, 1530, 1666)
    tok = Tokenizer(words=["the", "a"], max_words=30)
    yc = WindowedClipDataset(os.path.join(REF_CSV, "validation_youcook.csv"), "/nonexistent", tok, kind="youcook")
    assert len(yc) == 3350
    assert {"end", "start", "task", "text", "video_id"} <= set(yc.data.columns)
    mv = WindowedClipDataset(os.path.join(REF_CSV, "msrvtt_test.csv"), "/nonexistent", tok, kind="msrvtt")
    assert len(mv) == 1000
    assert {"key", "vid_key", "video_id", "sentence"} <= set(mv.data.columns)


def test_eval_csv_given_but_videos_missing_is_an_error(tmp_path):
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.train import evaluation
    args = get_args(argv=["--eval_csv", str(tmp_path / "hmdb51.csv"), "--eval_video_root", str(tmp_path / "none"),
                          "--word2vec_path", ""])
    with pytest.raises(FileNotFoundError):
        evaluation._synthetic_fallback(args, args.eval_csv, "HMDB")
    args.eval_csv = ""
    with pytest.warns(RuntimeWarning):
        evaluation._synthetic_fallback(args, "csv/hmdb51.csv", "HMDB")


def _worker_cdtw(rank, world, port, outdir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.losses.sdtw import CDTW
    from mil_nce_howto100m_amd.parallel import dist as pdist
    ctx = pdist.init_distributed("gloo", "cpu")
    args = get_args(argv=[])
    args.rank, args.world_size = ctx.rank, ctx.world_size
    torch.manual_seed(10 + rank)
    v = torch.randn(2, 4, 8, requires_grad=True)  # b = 2 local sequences
    t = torch.randn(2, 4, 8, requires_grad=True)
    gv, gt = pdist.all_gather_embeddings(v.view(2, -1), t.view(2, -1), ctx)
    loss = CDTW(args)(gv.view(-1, 4, 8), gt.view(-1, 4, 8))
    loss.backward()
    torch.save({"grad": v.grad, "loss": float(loss)}, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_cdtw_every_local_sequence_gets_gradient():
    """with b > 1 sequences per rank every local video sequence -- the only rows the
    gather's local-slice backward keeps -- must get a gradient on every rank."""
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_cdtw, args=(2, _port(), out), nprocs=2)
        for r in range(2):
            g = torch.load(os.path.join(out, f"r{r}.pt"))["grad"]
            assert torch.isfinite(g).all()
            assert (g.flatten(1).norm(dim=1) > 0).all(), r
