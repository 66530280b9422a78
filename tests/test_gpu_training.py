"""Training-level GPU checks (VERDICT r1 "next round" item 3).

* the full S3D-G + text tower actually learns on the class-structured synthetic data: the mean
  MIL-NCE loss over the last 20 of 150 Adam steps is well below the first 20 and below the
  zero-logit level log(2B) (SURVEY.md §7.3 exit criterion 1);
* the soft-DTW SDTW_3 loss (BASELINE config 4) and the GradCache micro-batched MIL-NCE loss
  (config 5): the HIP path equals the ATen/MIOpen path on the same weights and batch in
  train-mode BN (embeddings, loss, loss gradient w.r.t. the embeddings, step loss);
* the same comparison at the flagship layer shapes (16 x 200^2, K = 4; 64 clips).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(extra, seed=1):
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    args = get_args(argv=["--word2vec_path", "", "--vocab_size", "4000", *extra])
    ctx = pdist.DistContext(device=torch.device("cuda", 0))
    pdist.set_context(ctx)
    seed_everything(seed, 0)
    return Trainer(args, build_model(args, ctx.device), ctx, 1000), args


STEPS = 400


def test_full_model_learns_on_structured_synthetic_data():
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    b = 32
    tr, args = _trainer(["--batch_size", str(b), "--num_frames", "8", "--video_size", "112", "--num_candidates", "2",
                         "--lr", "1e-3", "--warmup_steps", "10"])
    data = SyntheticClips(b, 8, 112, 2, args.max_words, args.vocab_size, num_classes=16, device=torch.device("cuda"))
    losses = [tr.train_step(data.batch(i)) for i in range(STEPS)]
    losses = torch.stack(losses).float().cpu()
    first, last = float(losses[:20].mean()), float(losses[-20:].mean())
    chance = math.log(2 * b)
    curve = " ".join(f"{float(losses[i:i + 25].mean()):.2f}" for i in range(0, STEPS, 25))
    print(f"first20 {first:.3f} last20 {last:.3f} zero-logit level {chance:.3f}; per-25-step means: {curve}")
    assert torch.isfinite(losses).all()
    assert last < first - 1.0, (first, last)
    # below the zero-logit (chance) level; the trajectory is not bit-reproducible across boxes (the
    # autotuner's variant picks and float atomics change the roundings), and runs have ended 0.2-0.6
    # below chance, so the margin here is kept small
    assert last < chance - 0.1, (last, chance)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _soften(tr, f=0.05):
    """Scale the two output projections down so the logits are O(1): at the random-init O(10-30)
    logits the softmax is nearly one-hot and bf16 rounding of the embeddings decides the loss."""
    with torch.no_grad():
        tr.model.fc.weight.mul_(f)
        tr.model.text_module.fc2.weight.mul_(f)


def _embed(tr, batch, chunks, aten):
    """Train-mode embeddings of the batch (in ``chunks`` micro-batches, as the GradCache step's
    first pass computes them)."""
    from mil_nce_howto100m_amd import ops
    video, text = batch["video"], batch["text"]
    b = video.shape[0]
    vs, ts = [], []
    with torch.no_grad(), (ops.force_aten() if aten else _Null()):
        tr.model.train()
        for i in range(max(1, chunks)):
            s, e = i * b // max(1, chunks), (i + 1) * b // max(1, chunks)
            v, t = tr.model(video[s:e], text[s:e].reshape(-1, text.shape[-1]))
            vs.append(v.float())
            ts.append(t.float())
    return torch.cat(vs), torch.cat(ts)


def _loss_grad(tr, batch, v, t, aten):
    from mil_nce_howto100m_amd import ops
    v = v.clone().requires_grad_(True)
    t = t.clone().requires_grad_(True)
    with (ops.force_aten() if aten else _Null()):
        loss = tr._loss(batch, v, t)
        loss.backward()
    return float(loss), v.grad, t.grad


def _compare(extra, make_batch, chunks=0, video_tol=0.15):
    """Same weights, same batch: (1) the HIP towers' embeddings equal the ATen/MIOpen ones to bf16
    accuracy; (2) on the SAME embeddings the loss and its gradient w.r.t. the embeddings (the HIP
    soft-DTW / MIL-NCE kernels vs the ATen formulas) agree to fp32 accuracy; (3) the whole
    step (GradCache or one-shot) gives the same loss on both paths.

    Parameter gradients are deliberately not compared here: near the zero-logit level the loss
    gradient is almost the same for every sample, train-mode BN backward subtracts that common
    part, and what is left is below bf16 resolution on BOTH bf16 paths (each is ~uncorrelated
    with a CPU fp32 reference at this point; tools/debug/grad_ab.py). Layer-level gradient
    accuracy is covered by test_gpu_model.py with random upstream gradients."""
    tr, args = _trainer(extra, seed=5)
    tr_a, _ = _trainer(extra, seed=5)  # same seed: identical weights
    _soften(tr)
    _soften(tr_a)
    batch = make_batch(args)
    rel = lambda x, y: ((x - y).norm() / y.norm()).item()  # noqa: E731
    vh, th = _embed(tr, batch, chunks, aten=False)
    va, ta = _embed(tr_a, batch, chunks, aten=True)
    print(f"embeddings rel diff: video {rel(vh, va):.4f} text {rel(th, ta):.4f}")
    # bf16 conv outputs stored before train-mode BN lose precision where |mean| >> std; both bf16
    # paths carry that (each is 5-9 % from a CPU fp32 forward at these shapes, tools/debug/grad_ab.py;
    # HIP vs ATen measured 0.053 at the flagship shapes, 0.088 / 0.098 at the 96^2 ones). The
    # per-block fp32 bounds are in tests/test_gpu_fulldepth.py.
    assert rel(vh, va) < video_tol and rel(th, ta) < 0.02
    lh, gvh, gth = _loss_grad(tr, batch, vh, th, aten=False)
    la, gva, gta = _loss_grad(tr, batch, vh, th, aten=True)
    print(f"loss on the same embeddings: hip {lh:.6f} aten {la:.6f}; d/dv {rel(gvh, gva):.2e} d/dt {rel(gth, gta):.2e}")
    assert abs(lh - la) <= 1e-4 * max(1.0, abs(la))
    assert rel(gvh, gva) < 1e-3 and rel(gth, gta) < 1e-3
    steps = []
    for trainer, aten in ((tr, False), (tr_a, True)):
        from mil_nce_howto100m_amd import ops
        with (ops.force_aten() if aten else _Null()):
            trainer.model.train()
            trainer.bucketer.zero()
            if chunks > 1:
                loss = trainer._grad_cache_backward(batch, chunks)
            else:
                loss = trainer.forward_loss(batch)
                loss.backward()
        steps.append(float(loss))
        assert torch.isfinite(trainer.bucketer.flat).all()
    print(f"step loss hip {steps[0]:.5f} aten {steps[1]:.5f}")
    assert abs(steps[0] - steps[1]) <= 0.01 * max(1.0, abs(steps[1]))


def test_sdtw3_loss_hip_matches_aten():
    """BASELINE config 4's loss at a reduced shape: 8 sequences x 8 clips, 8 x 112^2."""
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips, SyntheticSequences

    def mk(args):
        clips = SyntheticClips(64, 8, 112, 1, args.max_words, args.vocab_size, device=torch.device("cuda"))
        return SyntheticSequences(8, 8, clips).batch(0)

    _compare(["--batch_size", "64", "--num_frames", "8", "--video_size", "112", "--num_candidates", "1",
              "--loss", "sdtw_3", "--seq_len", "8"], mk)


def test_gradcache_loss_hip_matches_aten():
    """BASELINE config 5's step (GradCache, 4 micro-batches, train-mode BN) at 32 clips x 16 frames."""
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips

    def mk(args):
        return SyntheticClips(32, 16, 96, 4, args.max_words, args.vocab_size, device=torch.device("cuda")).batch(0)

    _compare(["--batch_size", "32", "--num_frames", "16", "--video_size", "96", "--num_candidates", "4",
              "--grad_cache_chunks", "4"], mk, chunks=4)


def test_flagship_shapes_hip_matches_aten():
    """The BASELINE config-2 layer shapes (16 x 200^2 clips, K = 4 captions; 64 clips instead of 256
    to keep the ATen/MIOpen reference quick): every conv / pool / gate runs at its production
    spatial size and channel count with the kernel variants the autotuner picks for it, and the
    whole HIP step equals the ATen one (embeddings to bf16 accuracy, loss and embedding gradient
    to fp32 accuracy, step loss)."""
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips

    def mk(args):
        return SyntheticClips(64, 16, 200, 4, args.max_words, args.vocab_size, device=torch.device("cuda")).batch(0)

    _compare(["--batch_size", "64", "--num_frames", "16", "--video_size", "200", "--num_candidates", "4"], mk,
             video_tol=0.08)
