"""Retrieval metrics, linear probe, eval pipelines on synthetic data, the synthetic generator,
the tokenizer / candidate sampling, the CLI."""
import numpy as np
import torch

from mil_nce_howto100m_amd.config import get_args
from mil_nce_howto100m_amd.data.datasets import HowTo100MDataset, Tokenizer
from mil_nce_howto100m_amd.data.synthetic import SyntheticClips, SyntheticEvalSet, SyntheticSequences
from mil_nce_howto100m_amd.eval import compute_metrics, extract_features, linear_probe
from mil_nce_howto100m_amd.eval.retrieval import evaluate_retrieval
from mil_nce_howto100m_amd.models import S3D


def test_compute_metrics_reference_semantics():
    x = np.array([[3.0, 1.0, 0.0], [0.0, 1.0, 5.0], [2.0, 2.0, 2.0]])
    m = compute_metrics(x)
    # row0 rank 0; row1 rank 1; row2 ties with all 3 -> contributes 3 entries 0,1,2
    assert m["R1"] == 2 / 5 and m["R5"] == 1.0 and m["MR"] == 2.0


def test_linear_probe_separable_features():
    rng = np.random.default_rng(0)
    n, nw, d, ncls = 60, 2, 16, 3
    labels = [f"c{i % ncls}" for i in range(n)]
    centers = rng.normal(size=(ncls, d)) * 5
    feats = np.stack([[centers[i % ncls] + rng.normal(size=d) for _ in range(nw)] for i in range(n)])
    splits = [np.array([1 if i % 3 else 2 for i in range(n)])] * 3
    res = linear_probe(feats.astype(np.float32), labels, splits)
    assert res["split1"] > 0.9 and "mean" in res


def test_eval_pipelines_on_synthetic():
    torch.manual_seed(0)
    m = S3D(512, blocks=["mixed_3b"], vocab_size=500)
    ds = SyntheticEvalSet(8, num_clip=2, num_frames=4, size=32, num_classes=2, vocab_size=500)
    f, labels, splits = extract_features(m, ds.batches(4), torch.device("cpu"))
    assert f.shape == (8, 2, m.feature_dim) and len(labels) == 8 and len(splits) == 3
    r = evaluate_retrieval(m, ds.batches(4), torch.device("cpu"))
    assert set(r) == {"R1", "R5", "R10", "MR"}


def test_synthetic_clips_deterministic_and_sharded():
    a = SyntheticClips(3, 4, 16, 2, 10, 1000, rank=0, world_size=2)
    b = SyntheticClips(3, 4, 16, 2, 10, 1000, rank=1, world_size=2)
    a0, a0b, b0 = a.batch(5), a.batch(5), b.batch(5)
    assert torch.equal(a0["video"], a0b["video"]) and not torch.equal(a0["video"], b0["video"])
    assert a0["video"].shape == (3, 4, 16, 16, 4) and a0["video"].dtype == torch.uint8
    assert int(a0["video"][..., 3].abs().sum()) == 0
    assert a0["text"].shape == (3, 2, 10)
    # class words are shared by the K candidates of a clip
    assert torch.equal(a0["text"][:, 0, :4], a0["text"][:, 1, :4])
    assert set(a.sample_ids(5).tolist()).isdisjoint(set(b.sample_ids(5).tolist()))
    ref = SyntheticClips(2, 4, 16, layout="reference").batch(0)["video"]
    assert ref.shape == (2, 3, 4, 16, 16)
    seq = SyntheticSequences(2, 3, a).batch(0)
    assert seq["video"].shape[0] == 6 and seq["start"].shape == (2, 3)


def test_tokenizer_and_nearest_candidates():
    tok = Tokenizer(words=["hello", "world", "it's"], max_words=5)
    ids = tok("Hello world, it's a world!")
    assert ids.tolist() == [2, 3, 2, 0, 0]  # 'Hello' unknown (case-sensitive), ids = index + 1
    starts = [0, 10, 12, 30, 31]
    ends = [5, 11, 20, 31, 40]
    # video_loader.py:119-133 semantics
    assert HowTo100MDataset.nearest_candidates(starts, ends, 2, 3) == 0
    assert HowTo100MDataset.nearest_candidates(starts, ends, 3, 2) == 3
    assert HowTo100MDataset.nearest_candidates(starts, ends, 0, 3) == 0
    assert HowTo100MDataset.nearest_candidates(starts, ends, 4, 3) == 2


def test_cli_has_all_reference_flags_with_reference_defaults():
    a = get_args(argv=[])
    expect = dict(train_csv="../HowTo100M/csv/new_videos.csv", video_path="../HowTo100M/videos",
                  caption_root="../HowTo100M/caption_json", checkpoint_root="checkpoint", log_root="log",
                  eval_video_root="../HowTo100M/downstream", checkpoint_dir="", optimizer="adam",
                  weight_init="uniform", num_thread_reader=20, num_class=512, num_candidates=5, batch_size=128,
                  num_windows_test=4, batch_size_val=32, momemtum=0.9, n_display=400, num_frames=32,
                  video_size=224, crop_only=1, centercrop=0, random_flip=1, verbose=1, warmup_steps=50000,
                  min_time=5.0, pretrain_cnn_path="", word2vec_path="../HowTo100M/data/word2vec.pth", fps=10,
                  cudnn_benchmark=0, epochs=300, start_epoch=0, lr=0.001, momentum=0.9, resume=False,
                  evaluate=False, pretrained=False, pin_memory=False, world_size=-1, rank=-1,
                  dist_file="dist-file", dist_backend="nccl", seed=1, gpu=None,
                  multiprocessing_distributed=False)
    for k, v in expect.items():
        assert getattr(a, k) == v, k
    assert hasattr(a, "dist_url")
    assert len(expect) + 1 == 45
    s = get_args(argv=["--preset", "small"])
    assert s.batch_size == 12 and s.warmup_steps == 1000 and s.epochs == 100 and s.n_display == 100
