"""Gradient-bucket readiness on the HIP path (VERDICT r1 "next round" item 1, step 3).

One GPU, but the bucketer is built for world_size=2 with its all-reduce replaced by a stream-
ordered snapshot of the bucket's flat slice. The HIP kernels write weight / BN gradients
straight into the flat buffer and report through ``ops.grad_sink``; autograd-accumulated
parameters report through post-accumulate hooks. After a full training step of the whole
S3D-G + text tower (one-shot and GradCache with 2 micro-batches) every parameter must have
reported (a parameter written in place reports twice: kernel + autograd's post-accumulate
hook, and the bucketer must count it once -- found by this test), every bucket must have been issued exactly once before ``finish()``,
and each snapshot must equal the final gradient slice (nothing landed after the issue).
"""
import pytest
import torch

from bucket_recorder import BucketRecorder

pytestmark = pytest.mark.gpu


class _Done:
    def wait(self):
        pass


@pytest.mark.parametrize("chunks", [0, 2])
def test_bucket_issue_after_last_direct_write(chunks):
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.ops import _lib
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.parallel.ddp import GradBucketer
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    _lib.lib()
    ctx = pdist.init_distributed("nccl", "cuda")
    args = get_args(argv=["--batch_size", "4", "--num_frames", "8", "--video_size", "64", "--num_candidates", "2",
                          "--word2vec_path", "", "--warmup_steps", "1", "--grad_cache_chunks", str(chunks)])
    seed_everything(3, 0)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 10)
    bk = GradBucketer(list(tr.model.parameters()), world_size=2, bucket_bytes=2 << 20)
    assert len(bk.buckets) >= 8
    bk._launch = lambda i: bk._handles.__setitem__(i, _Done())
    rec = BucketRecorder(bk)
    tr.bucketer = bk
    tr.optimizer.bind_flat_grad(bk.flat, bk.offsets)
    data = SyntheticClips(4, 8, 64, 2, args.max_words, args.vocab_size, device=ctx.device)
    try:
        for step in range(2):
            rec.snaps.clear()
            rec.notes.clear()
            tr.train_step(data.batch(step))
            torch.cuda.synchronize()
            snaps = rec.check()
            for i, (s, e) in enumerate(bk.buckets):
                assert torch.equal(snaps[i], bk.flat[s:e]), f"bucket {i} changed after it was issued"
            assert float(bk.flat.abs().sum()) > 0
    finally:
        from mil_nce_howto100m_amd.ops import grad_sink
        grad_sink.set_sink(None)
