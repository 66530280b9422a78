"""One rank of the on-GPU data-parallel check (tests/test_gpu_dp.py); not a test module.

    python tests/dp_worker.py OUTDIR CHUNKS [BUCKET_MB]   (env: RANK, WORLD_SIZE, MASTER_*, MILNCE_DEVICE_INDEX)

Runs the production Trainer on cuda (HIP kernels, direct flat-buffer gradient writes, the
GradBucketer's async all-reduces, the embedding all-gather) with the ranks sharing one device
over a gloo process group, and saves what the test compares:
  * eval-mode BN (per-sample independent, so W ranks see exactly the single-process batch):
    the loss and the reduced flat gradient of one forward/backward (GradCache CHUNKS > 1 or not);
  * train mode with --verify_buckets 1: two full train_steps (bucket order verifier, fused Adam),
    then the flat parameters, which must be identical on every rank;
  * at W > 1 the comm probe (parallel/comm_probe.py) on the step's sizes, and the buckets (with
    BUCKET_MB auto: the start-up plan measured on the process group, parallel/bucket_plan.py).
World size 1 gets the concatenation of the W=2 shards as its batch (the reference run).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    out, chunks = sys.argv[1], int(sys.argv[2])
    bucket_mb = sys.argv[3] if len(sys.argv) > 3 else "1"
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.ops import _lib, hip_ops
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    _lib.lib()
    ctx = pdist.init_distributed("gloo", "cuda")
    W, r = ctx.world_size, ctx.rank
    b_local = 4
    args = get_args(argv=["--batch_size", str(b_local * W), "--num_frames", "8", "--video_size", "64",
                          "--num_candidates", "2", "--word2vec_path", "", "--warmup_steps", "1",
                          "--grad_cache_chunks", str(chunks), "--verify_buckets", "1", "--bucket_mb", bucket_mb])
    seed_everything(7, r)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 10)

    def shard(step, rank):
        return SyntheticClips(b_local, 8, 64, 2, args.max_words, args.vocab_size, device=ctx.device,
                              rank=rank, world_size=2).batch(step)

    def batch(step):
        if W == 2:
            return shard(step, r)
        parts = [shard(step, q) for q in range(2)]
        return {k: torch.cat([p[k] for p in parts]) for k in parts[0]}

    # 1. eval-mode BN forward/backward, reduced flat gradient
    tr.model.eval()
    tr.bucketer.zero()
    hip_ops.zero_arena_begin(ctx.device)
    try:
        with tr.tune_region():  # kernel choices: rank 0's, on every rank
            if chunks > 1:
                loss = tr._grad_cache_backward(batch(0), chunks)
            else:
                loss = tr.forward_loss(batch(0))
                loss.backward()
    finally:
        hip_ops.zero_arena_end()
    tr.bucketer.finish()
    torch.cuda.synchronize()
    res = {"loss": float(loss.detach()), "world": W, "rank": r}
    torch.save(tr.bucketer.flat.detach().cpu(), os.path.join(out, f"grad_w{W}_r{r}.pt"))
    # 2. two real train steps (train-mode BN, bucket verifier, optimizer)
    for step in range(1, 3):
        res[f"train_loss{step}"] = float(tr.train_step(batch(step)))
    torch.cuda.synchronize()
    flat_p = torch.cat([p.detach().reshape(-1).float().cpu() for p in tr.model.parameters()])
    torch.save(flat_p, os.path.join(out, f"param_w{W}_r{r}.pt"))
    # BN buffers through the flat BufferBroadcaster: the train steps (GradCache micro-batches when
    # CHUNKS > 1) updated them in place through its views; one more broadcast (the next step's
    # first action) makes every rank hold rank 0's statistics
    bc = tr.buffers
    if bc is not None:
        bc()
        torch.cuda.synchronize()
        res["bcast"] = {"flats": len(bc.flats), "intact": bool(bc.views_intact()) if bc.flats else True,
                        "reflattens": bc.reflattens}
    bufs = torch.cat([b.detach().reshape(-1).double().cpu() for b in tr.model.buffers()])
    torch.save(bufs, os.path.join(out, f"bufs_w{W}_r{r}.pt"))
    from mil_nce_howto100m_amd.ops import tune_sync
    res["plan_hash"] = tune_sync.plan_hash()
    res["tune_decisions"] = tune_sync.decisions()
    res["buckets"] = [list(b) for b in tr.bucketer.buckets]
    res["bucket_plan"] = tr.comm_plan.as_dict() if tr.comm_plan is not None else None
    if W > 1:
        from mil_nce_howto100m_amd.parallel.comm_probe import probe
        res["comm"] = probe(tr.bucketer.flat.numel(), tr.bucketer.buckets, b_local * 3, 512, torch.float32,
                            ctx.device, reps=3)
    with open(os.path.join(out, f"res_w{W}_r{r}.json"), "w") as f:
        json.dump(res, f)
    pdist.destroy()


if __name__ == "__main__":
    main()
