"""Eval entry points on the shipped CSVs: the defaults resolve to ``csv/``
next to the package (reference ``eval_hmdb.py:40``), and ``eval_hmdb.run`` sharded over two
gloo ranks (the one-process-per-GPU replacement of the reference's DataParallel eval,
``eval_hmdb.py:27,32``) reports what one rank reports.

ffmpeg is not in this image: ``decode_clip`` is replaced by a deterministic function of the
video path (class-dependent, so the probe has something to learn); everything else -- the
shipped CSV rows, the HMDB dataset, the sharded loader, the feature all-gather and the
LinearSVC probe -- is the production path.
"""
import json
import os
import socket
import sys
import tempfile

import numpy as np
import pandas as pd
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_decode(path, size, fps=None, start=None, duration=None, crop_only=False, center_crop=True, hflip=False,
                 rng=None):
    label = os.path.basename(os.path.dirname(path))
    cls = sum(map(ord, label)) % 7
    vid = sum(map(ord, os.path.basename(path))) % 13
    n = 6
    t = np.arange(n).reshape(n, 1, 1, 1)
    y = np.arange(size).reshape(1, size, 1, 1)
    x = np.arange(size).reshape(1, 1, size, 1)
    c = np.arange(3).reshape(1, 1, 1, 3)
    v = (cls * 37 + vid + t * 3 + (y * (cls + 1)) % 29 + x * (c + 1) * (cls % 3 + 1)) % 256
    return v.astype(np.uint8)


def _patch(dump):
    from mil_nce_howto100m_amd.data import datasets
    from mil_nce_howto100m_amd.train import evaluation
    datasets.decode_clip = _fake_decode
    evaluation.ffmpeg_available = lambda: True
    probe = evaluation.linear_probe

    def recording_probe(feats, labels, splits, C=100.0):
        # the features rank 0 fits on: compared across world sizes (the SVC fit on a random-init
        # model's features is too ill-conditioned to compare accuracies)
        np.savez(dump, feats=feats, labels=np.asarray(labels), splits=np.stack(splits))
        return probe(feats, labels, splits, C=C)

    evaluation.linear_probe = recording_probe


def _argv(d):
    return ["--device", "cpu", "--num_frames", "4", "--video_size", "32",
            "--num_windows_test", "2", "--batch_size_val", "4", "--num_thread_reader", "0",
            "--eval_csv", os.path.join(d, "hmdb_subset.csv"), "--eval_video_root", os.path.join(d, "videos"),
            "--pretrain_cnn_path", os.path.join(d, "ckpt.pth.tar"), "--word2vec_path", "", "--vocab_size", "100"]


def _worker(rank, world, port, d):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    _patch(os.path.join(d, f"feats_w{world}.npz"))
    import eval_hmdb
    res = eval_hmdb.run(_argv(d))
    if rank == 0:
        with open(os.path.join(d, f"res_w{world}.json"), "w") as f:
            json.dump(res, f)


def test_default_eval_csvs_shipped():
    from mil_nce_howto100m_amd.train.evaluation import CSV_DIR, default_csv
    assert os.path.dirname(CSV_DIR) == ROOT
    hm = pd.read_csv(default_csv("hmdb51.csv"))
    assert len(hm) == 6766 and list(hm.columns) == ["video_id", "label", "split1", "split2", "split3"]
    assert hm["label"].str.replace("_test$", "", regex=True).nunique() == 51
    assert (hm["split1"] == 1).sum() == 3570 and (hm["split1"] == 2).sum() == 1530
    yc = pd.read_csv(default_csv("validation_youcook.csv"))
    assert len(yc) == 3350 and list(yc.columns) == ["end", "start", "task", "text", "video_id"]
    ms = pd.read_csv(default_csv("msrvtt_test.csv"))
    assert len(ms) == 1000 and list(ms.columns) == ["key", "vid_key", "video_id", "sentence"]


def test_eval_hmdb_two_ranks_match_one_rank():
    from mil_nce_howto100m_amd.models import S3D
    from mil_nce_howto100m_amd.train.evaluation import default_csv
    with tempfile.TemporaryDirectory() as d:
        hm = pd.read_csv(default_csv("hmdb51.csv"))
        # 4 classes of the shipped CSV, the split-1 train/test rows of each (16 + 6 per class)
        classes = sorted(hm["label"].unique())[:4]
        parts = []
        for c in classes:
            rows = hm[hm["label"] == c]
            parts += [rows[rows["split1"] == 1].head(16), rows[rows["split1"] == 2].head(6)]
        sub = pd.concat(parts)
        sub.to_csv(os.path.join(d, "hmdb_subset.csv"), index=False)
        os.makedirs(os.path.join(d, "videos"))
        torch.manual_seed(0)
        model = S3D(512, word2vec_path="", vocab_size=100)
        torch.save({"epoch": 1, "state_dict": {"module." + k: v for k, v in model.state_dict().items()}},
                   os.path.join(d, "ckpt.pth.tar"))
        # one rank in this process (no process group), then two gloo ranks
        _patch(os.path.join(d, "feats_w1.npz"))
        import eval_hmdb
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            os.environ.pop(k, None)
        res1 = eval_hmdb.run(_argv(d))
        mp.spawn(_worker, args=(2, _port(), d), nprocs=2)
        with open(os.path.join(d, "res_w2.json")) as f:
            res2 = json.load(f)
        f1, f2 = np.load(os.path.join(d, "feats_w1.npz")), np.load(os.path.join(d, "feats_w2.npz"))
        assert set(res1) == set(res2) and "split1" in res1
        assert f1["feats"].shape == (len(sub), 2, 1024)
        assert (f1["labels"] == f2["labels"]).all() and (f1["splits"] == f2["splits"]).all()
        assert sorted(set(f1["labels"])) == sorted(c[:-5] if c.endswith("_test") else c for c in classes)
        err = np.abs(f1["feats"] - f2["feats"]).max() / np.abs(f1["feats"]).max()
        assert err < 1e-4, err
