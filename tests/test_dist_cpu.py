"""Distributed semantics on CPU/gloo with real multi-process rendezvous (127.0.0.1).

* the embedding all-gather: rank-major order, local-slice backward (utils.py:8-24);
* the reference gradient scale: world_size=2 DP gradient == full-batch gradient / 2
  (SURVEY.md §2.10 item 2), and ``--grad_scale exact`` gives the full-batch gradient;
* bucketed all-reduce + BN buffer broadcast keep replicas identical after steps;
* checkpoint save on rank 0 + resume on both ranks reproduces the uninterrupted run.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _put(outdir, rank, obj):
    torch.save(obj, os.path.join(outdir, f"rank{rank}.pt"))


def _collect(outdir, world):
    return [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=False) for r in range(world)]


def _init(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from mil_nce_howto100m_amd.parallel import dist as pdist
    return pdist.init_distributed("gloo", "cpu")


def _args(extra=()):
    from mil_nce_howto100m_amd.config import get_args
    return get_args(argv=["--batch_size", "4", "--num_frames", "4", "--video_size", "32", "--num_candidates", "2",
                          "--blocks", "mixed_3b", "--warmup_steps", "1", "--word2vec_path", "", "--vocab_size", "500",
                          "--lr", "1e-3", *extra])


def _worker_gather(rank, world, port, outdir, mode="rccl"):
    ctx = _init(rank, world, port)
    from mil_nce_howto100m_amd.parallel.dist import all_gather_embeddings, set_emb_gather
    set_emb_gather(mode)
    if mode == "peer":  # the peer path's host fallback (CPU tensors) keeps the rank-major layout
        from mil_nce_howto100m_amd.parallel.peer import PeerAllGather, same_node
        assert same_node()  # every rank of this group on one host (the IPC path's precondition)
        got = PeerAllGather().gather(torch.full((3, 2), float(rank)))
        assert torch.equal(got[:, 0], torch.tensor([0.0] * 3 + [1.0] * 3))
    v = torch.full((2, 3), float(rank), requires_grad=True)
    t = torch.full((4, 3), 10.0 + rank, requires_grad=True)
    gv, gt = all_gather_embeddings(v, t, ctx)
    (gv.sum() * 2 + gt.sum() * 3).backward()
    _put(outdir, rank, (rank, gv.detach(), gt.detach(), v.grad, t.grad))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["rccl", "peer"])
def test_allgather_semantics(mode):
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_gather, args=(world, port, out, mode), nprocs=world)
        res = _collect(out, world)
    for rank, gv, gt, vg, tg in res:
        assert torch.equal(gv[:, 0], torch.tensor([0.0, 0.0, 1.0, 1.0]))
        assert torch.equal(gt[:, 0], torch.tensor([10.0] * 4 + [11.0] * 4))
        assert torch.equal(vg, torch.full((2, 3), 2.0))  # local slice only, no reduction
        assert torch.equal(tg, torch.full((4, 3), 3.0))


def _worker_negatives(rank, world, port, outdir, mode, b, K):
    """Each rank's b video rows carry global id rank*b + j, its b*K text rows the id of their clip
    (candidate k in the fractional part): after the gather, text rows i*K..i*K+K-1 belong to
    video row i of the global batch (loss.py:12, the MIL-NCE positive block)."""
    ctx = _init(rank, world, port)
    from mil_nce_howto100m_amd.parallel.dist import all_gather_embeddings, set_emb_gather
    set_emb_gather(mode)
    vid = torch.arange(b, dtype=torch.float32) + rank * b
    v = vid[:, None].repeat(1, 4).requires_grad_(True)
    t = (vid[:, None] + torch.arange(K, dtype=torch.float32)[None] / 10).reshape(b * K, 1).repeat(1, 4)
    t.requires_grad_(True)
    gv, gt = all_gather_embeddings(v, t, ctx)
    # a loss that weights every global row by its index: the local-slice backward keeps this
    # rank's rows only
    w_v = torch.arange(world * b, dtype=torch.float32)[:, None]
    w_t = torch.arange(world * b * K, dtype=torch.float32)[:, None]
    ((gv * w_v).sum() + (gt * w_t).sum()).backward()
    _put(outdir, rank, (rank, gv.detach(), gt.detach(), v.grad, t.grad))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["rccl", "peer"])
def test_negatives_rank_major_w8(mode):
    world, b, K = 8, 3, 4
    port = _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_negatives, args=(world, port, out, mode, b, K), nprocs=world)
        res = _collect(out, world)
    for rank, gv, gt, vg, tg in res:
        assert gv.shape == (world * b, 4) and gt.shape == (world * b * K, 4)
        i = torch.arange(world * b, dtype=torch.float32)
        assert torch.equal(gv[:, 0], i)  # video row i = global clip i, rank-major
        # text rows i*K .. i*K+K-1 are clip i's K candidates, in order
        exp_t = (i[:, None] + torch.arange(K, dtype=torch.float32)[None] / 10).reshape(-1)
        assert torch.allclose(gt[:, 0], exp_t)
        # local-slice backward: this rank's rows' weights, no cross-rank reduction
        assert torch.equal(vg[:, 0], torch.arange(rank * b, (rank + 1) * b, dtype=torch.float32))
        assert torch.equal(tg[:, 0], torch.arange(rank * b * K, (rank + 1) * b * K, dtype=torch.float32))


def _worker_grad(rank, world, port, outdir, mode):
    ctx = _init(rank, world, port)
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    args = _args(["--grad_scale", mode])
    seed_everything(1, rank)
    model = build_model(args, ctx.device)
    tr = Trainer(args, model, ctx, 10)
    data = SyntheticClips(2, 4, 32, 2, 20, 500, device=ctx.device, rank=rank, world_size=world)
    tr.model.eval()  # BN on running stats: per-rank forward == its slice of the full-batch forward
    tr.bucketer.zero()
    tr.buffers()
    loss = tr.forward_loss(data.batch(0))
    loss.backward()
    tr.bucketer.finish()
    _put(outdir, rank, (rank, tr.bucketer.flat * tr.optimizer.grad_scale, float(loss)))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,world", [("reference", 2), ("exact", 2), ("reference", 4), ("reference", 8)])
def test_dp_gradient_scale(mode, world):
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    ratio = 1.0 / world if mode == "reference" else 1.0
    port = _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_grad, args=(world, port, out, mode), nprocs=world)
        res = _collect(out, world)
    g0 = res[0][1]
    for r in range(1, world):
        assert torch.allclose(g0, res[r][1], atol=1e-6)
    # single process, full global batch (both ranks' samples, rank-major)
    ctx = pdist.DistContext()
    pdist.set_context(ctx)
    args = _args()
    seed_everything(1, 0)
    model = build_model(args, ctx.device)
    tr = Trainer(args, model, ctx, 10)
    ds = [SyntheticClips(2, 4, 32, 2, 20, 500, rank=r, world_size=world).batch(0) for r in range(world)]
    batch = {k: torch.cat([d[k] for d in ds]) for k in ("video", "text")}
    tr.model.eval()
    tr.bucketer.zero()
    loss = tr.forward_loss(batch)
    loss.backward()
    full = tr.bucketer.flat
    assert abs(float(loss) - res[0][2]) < 1e-4
    assert torch.allclose(g0, full * ratio, rtol=1e-3, atol=1e-7)


def _worker_train(rank, world, port, ckdir, stop, resume):
    ctx = _init(rank, world, port)
    from mil_nce_howto100m_amd.train.engine import run_training
    args = _args(["--checkpoint_root", ckdir, "--checkpoint_dir", "run", "--epochs", "2", "--stop_epoch", str(stop),
                  "--steps_per_epoch", "2", "--n_display", "1", "--verbose", "0", "--log_root", ckdir]
                 + (["--resume"] if resume else []))
    args.rank, args.world_size = ctx.rank, ctx.world_size
    run_training(args, ctx)
    dist.destroy_process_group()


def test_checkpoint_resume_equivalence():
    from mil_nce_howto100m_amd.train import checkpoint as ck
    world = 2
    with tempfile.TemporaryDirectory() as d1, tempfile.TemporaryDirectory() as d2:
        mp.spawn(_worker_train, args=(world, _port(), d1, 2, False), nprocs=world)  # 2 epochs straight
        mp.spawn(_worker_train, args=(world, _port(), d2, 1, False), nprocs=world)  # 1 epoch
        mp.spawn(_worker_train, args=(world, _port(), d2, 2, True), nprocs=world)   # resume -> 2
        a = ck.load_checkpoint(os.path.join(d1, "run", "epoch0002.pth.tar"))
        b = ck.load_checkpoint(os.path.join(d2, "run", "epoch0002.pth.tar"))
        assert a["epoch"] == b["epoch"] == 2
        assert a["scheduler"]["last_epoch"] == b["scheduler"]["last_epoch"] == 4
        for k in a["state_dict"]:
            assert torch.allclose(a["state_dict"][k].float(), b["state_dict"][k].float(), atol=1e-6), k
        sa, sb = a["optimizer"]["state"], b["optimizer"]["state"]
        assert sa.keys() == sb.keys()
        for k in sa:
            assert torch.allclose(sa[k]["exp_avg"], sb[k]["exp_avg"], atol=1e-7)


def _worker_fault(rank, world, port, ckdir, extra):
    ctx = _init(rank, world, port)
    from mil_nce_howto100m_amd.train.engine import run_training
    args = _args(["--checkpoint_root", ckdir, "--checkpoint_dir", "run", "--epochs", "2",
                  "--steps_per_epoch", "3", "--n_display", "1", "--verbose", "0", "--log_root", ckdir, *extra])
    args.rank, args.world_size = ctx.rank, ctx.world_size
    try:
        run_training(args, ctx)
    finally:
        dist.destroy_process_group()


def test_fault_injection_mid_epoch_resume():
    """Kill both ranks mid-epoch (injected fault), --resume from the step checkpoint, and land on
    exactly the state of an uninterrupted run."""
    from mil_nce_howto100m_amd.train import checkpoint as ck
    world = 2
    with tempfile.TemporaryDirectory() as d1, tempfile.TemporaryDirectory() as d2:
        mp.spawn(_worker_fault, args=(world, _port(), d1, []), nprocs=world)
        with pytest.raises(Exception):
            mp.spawn(_worker_fault, args=(world, _port(), d2, ["--ckpt_every_steps", "1", "--fault_at_step", "5"]),
                     nprocs=world)
        mid = ck.load_checkpoint(ck.get_last_checkpoint(os.path.join(d2, "run")))
        assert mid["epoch"] == 1 and mid["step_in_epoch"] == 2  # global step 5 = epoch 1, step 2
        mp.spawn(_worker_fault, args=(world, _port(), d2, ["--resume"]), nprocs=world)
        a = ck.load_checkpoint(os.path.join(d1, "run", "epoch0002.pth.tar"))
        b = ck.load_checkpoint(os.path.join(d2, "run", "epoch0002.pth.tar"))
        assert a["scheduler"]["last_epoch"] == b["scheduler"]["last_epoch"] == 6
        for k in a["state_dict"]:
            assert torch.allclose(a["state_dict"][k].float(), b["state_dict"][k].float(), atol=1e-6), k


def test_watchdog_fires_without_progress():
    import time
    from mil_nce_howto100m_amd.utils import Watchdog
    with tempfile.TemporaryDirectory() as d:
        wd = Watchdog(0.3, rank=0, dump_dir=d, abort=False, poll_s=0.05).start()
        for _ in range(8):  # steady progress: silent
            time.sleep(0.1)
            wd.beat(1)
        assert not wd.fired.is_set()
        assert wd.fired.wait(3.0)
        wd.stop()
        assert "no training progress" in open(os.path.join(d, "watchdog_rank0.txt")).read()


def test_phase_timers_cpu():
    from mil_nce_howto100m_amd.utils import StepTimer
    t = StepTimer(True, torch.device("cpu"))
    for _ in range(3):
        with t.phase("forward"):
            sum(range(1000))
    s = t.summary()
    assert set(s) == {"forward"} and s["forward"] >= 0.0


def _worker_eval(rank, world, port, outdir):
    ctx = _init(rank, world, port)
    from mil_nce_howto100m_amd.data.synthetic import SyntheticEvalSet
    from mil_nce_howto100m_amd.eval import embed_retrieval, extract_features
    from mil_nce_howto100m_amd.train.engine import build_model, seed_everything
    args = _args()
    seed_everything(5, 0)
    model = build_model(args, ctx.device)
    ev = SyntheticEvalSet(10, 2, 4, 32, vocab_size=500)
    f, lab, spl = extract_features(model, ev.batches(3), ctx.device, ctx.rank, ctx.world_size)
    t, v = embed_retrieval(model, ev.batches(3), ctx.device, ctx.rank, ctx.world_size)
    _put(outdir, rank, (f, lab, spl, t, v))
    dist.destroy_process_group()


def test_sharded_eval_matches_single_process():
    """One process per GPU replaces nn.DataParallel in the evals: 2-rank sharded features and
    embeddings == the single-process ones, in the same order, on every rank."""
    import numpy as np
    from mil_nce_howto100m_amd.data.synthetic import SyntheticEvalSet
    from mil_nce_howto100m_amd.eval import embed_retrieval, extract_features
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import build_model, seed_everything
    world = 2
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_eval, args=(world, _port(), out), nprocs=world)
        res = _collect(out, world)
    pdist.set_context(pdist.DistContext())
    seed_everything(5, 0)
    model = build_model(_args(), torch.device("cpu"))
    ev = SyntheticEvalSet(10, 2, 4, 32, vocab_size=500)
    f, lab, spl = extract_features(model, ev.batches(3), "cpu")
    t, v = embed_retrieval(model, ev.batches(3), "cpu")
    for rf, rlab, rspl, rt, rv in res:
        assert np.allclose(rf, f, atol=1e-5) and list(rlab) == list(lab)
        assert all(np.array_equal(a, b) for a, b in zip(rspl, spl))
        assert np.allclose(rt, t, atol=1e-5) and np.allclose(rv, v, atol=1e-5)


def test_bench_contract_two_ranks_cpu():
    """bench.py under torch.distributed.run (the driver's N>1 launch, gloo on CPU here): exactly
    one JSON line from rank 0 with the whole-job aggregate and the documented keys."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--num_frames", "4", "--size", "32", "--batch_per_gpu", "2", "--blocks", "mixed_3b"]
    out = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in r, k
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["warmup"] == 1
    assert r["config"]["global_batch"] == 4 and r["config"]["parallelism"] == "dp2"
    assert abs(r["value"] - 4 * 1000.0 / r["ms_per_step"]) / r["value"] < 1e-2


def _worker_verify(rank, world, port, outdir, late_write):
    _init(rank, world, port)
    from mil_nce_howto100m_amd.parallel.ddp import BucketOrderError, GradBucketer
    torch.manual_seed(0)
    lin = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 4))
    bk = GradBucketer(list(lin.parameters()), world, bucket_bytes=64, verify=True)
    bk.zero()
    x = torch.full((3, 8), 1.0 + rank)
    lin(x).sum().backward()  # every bucket launches from its post-accumulate hooks
    if late_write:
        lin[0].weight.grad.add_(1.0)  # a write after the bucket was issued: lost in normal mode
    err = None
    try:
        bk.finish()
    except BucketOrderError as e:
        err = str(e)
    _put(outdir, rank, (err, bk.flat.clone()))
    dist.destroy_process_group()


@pytest.mark.parametrize("late_write", [False, True])
def test_bucket_order_verifier(late_write):
    """GradBucketer(verify=True): clean steps pass and still all-reduce; a gradient written after
    its bucket launched is reported (parallel/ddp.py BucketOrderError)."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker_verify, args=(world, _port(), d, late_write), nprocs=world, join=True)
        res = _collect(d, world)
    for err, flat in res:
        if late_write:
            assert err is not None and "bucket" in err
        else:
            assert err is None
    assert torch.equal(res[0][1], res[1][1])  # the reduced gradient was installed on both ranks


def _worker_bf16_wire(rank, world, port, outdir):
    _init(rank, world, port)
    from mil_nce_howto100m_amd.parallel.ddp import GradBucketer
    torch.manual_seed(0)
    lin = torch.nn.Sequential(torch.nn.Linear(16, 16), torch.nn.Linear(16, 4))
    res = []
    for dt in (torch.float32, torch.bfloat16):
        bk = GradBucketer(list(lin.parameters()), world, bucket_bytes=256, comm_dtype=dt)
        bk.zero()
        x = torch.linspace(-1, 1, 48).view(3, 16) * (1.0 + rank)
        lin(x).pow(2).sum().backward()
        bk.finish()
        assert bk.flat.dtype == torch.float32 and len(bk.buckets) > 1
        res.append(bk.flat.clone())
    _put(outdir, rank, res)
    dist.destroy_process_group()


def test_bucket_bf16_wire():
    """--grad_comm_dtype bf16: every bucket is reduced as bf16 and written back into the fp32
    flat buffer; the sum matches the fp32 wire to bf16 accuracy on every rank."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker_bf16_wire, args=(world, _port(), d), nprocs=world, join=True)
        res = _collect(d, world)
    f32, b16 = res[0]
    assert torch.equal(b16, res[1][1]) and torch.equal(f32, res[1][0])
    assert not torch.equal(f32, b16)  # really went through bf16
    assert ((f32 - b16).norm() / f32.norm()).item() < 1e-2


def _worker_buffers(rank, world, port, outdir):
    _init(rank, world, port)
    from mil_nce_howto100m_amd.parallel.ddp import BufferBroadcaster
    torch.manual_seed(rank)  # different buffers per rank
    m = torch.nn.Sequential(torch.nn.BatchNorm3d(5), torch.nn.Linear(3, 3), torch.nn.BatchNorm3d(7))
    for b in m.buffers():
        if b.is_floating_point():
            b.copy_(torch.randn_like(b))
        else:
            b.fill_(rank + 3)
    keys = list(m.state_dict())
    bb = BufferBroadcaster(m, world)
    views = [(b.data_ptr(), b.dtype) for b in m.buffers()]
    flat_ptrs = [(f.data_ptr(), f.data_ptr() + f.numel() * f.element_size(), f.dtype) for f in bb.flats]
    # every buffer is a view into its dtype's flat tensor; names / shapes unchanged
    inside = all(any(lo <= p < hi and fd == d for lo, hi, fd in flat_ptrs) for p, d in views)
    bb()
    after = {k: v.clone() for k, v in m.state_dict().items() if "running" in k or "num_batches" in k}
    # in-place updates (what the BN kernels do) land in the flat tensor; a load copies into the views
    m[0].running_mean.add_(1.0)
    m.load_state_dict({k: v.clone() for k, v in m.state_dict().items()})
    still = all(b.data_ptr() == p for b, (p, _) in zip(m.buffers(), views))
    _put(outdir, rank, (len(bb.flats), inside, keys == list(m.state_dict()), after, still,
                        m[0].running_mean.clone(), bb.flats[0].clone()))
    dist.destroy_process_group()


def test_buffer_broadcaster_flat_views():
    """BufferBroadcaster at N > 1: the BN buffers become views of one flat tensor per dtype (no
    per-step pack / unpack), the broadcast makes every rank's buffers rank 0's, in-place updates and
    state-dict loads keep writing through the views."""
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_buffers, args=(world, port, out), nprocs=world)
        res = _collect(out, world)
    for nflat, inside, same_keys, _, still, rm, flat in res:
        assert nflat == 2  # float32 stats, int64 counters
        assert inside and same_keys and still
        assert torch.equal(flat[:rm.numel()], rm)  # the first BN's running mean leads the float flat
    a, b = res[0][3], res[1][3]
    assert a.keys() == b.keys() and all(torch.equal(a[k], b[k]) for k in a)
    assert all(int(v.reshape(-1)[0]) == 3 for k, v in a.items() if "num_batches" in k)  # rank 0's


def _worker_bcast(rank, world, port, outdir):
    _init(rank, world, port)
    from mil_nce_howto100m_amd.parallel.ddp import BufferBroadcaster
    m = torch.nn.Sequential(torch.nn.BatchNorm1d(3), torch.nn.BatchNorm1d(5))
    for b in m.buffers():
        b.fill_(float(rank + 1))
    bc = BufferBroadcaster(m, world)
    bc()
    first = [b.clone() for b in m.buffers()]
    # replace a buffer tensor (what load_state_dict(assign=True) or .to() does): it leaves the flat
    m[1].running_mean = torch.full((5,), 10.0 + rank)
    assert not bc.views_intact()
    bc()  # re-flattens, then broadcasts rank 0's values into the new buffer too
    _put(outdir, rank, (first, [b.clone() for b in m.buffers()], bc.reflattens, bc.views_intact()))
    dist.destroy_process_group()


def test_buffer_broadcaster_reflattens_replaced_buffers():
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_bcast, args=(world, port, out), nprocs=world)
        res = _collect(out, world)
    for first, after, refl, intact in res:
        assert all(torch.all(b == 1.0) for b in first)  # rank 0's values everywhere
        assert refl == 1 and intact
        assert torch.all(after[3] == 10.0)  # the replaced running_mean: rank 0's new value


def test_bucket_plan_model():
    """The link model's plan: buckets at 4x the latency knee within [4, 64] MiB and at most half the
    gradient, the last bucket at the knee (>= 1 MiB); more ranks -> larger latency term."""
    from mil_nce_howto100m_amd.parallel import bucket_plan as bp
    MIB = bp.MIB
    m2, m8 = bp.xgmi_model(2), bp.xgmi_model(8)
    assert m8.a_s > m2.a_s and m8.knee_bytes > 0
    for w in (2, 4, 8):
        p = bp.plan_buckets(45 * MIB, w)
        assert 1 * MIB <= p.tail_bytes <= p.bucket_bytes <= max(22.5 * MIB, 4 * MIB)
        assert p.source == "xgmi-model" and p.busbw_gbps > 0
    # a measured latency-free link: minimum sizes; a slow-latency link: capped at half the gradient
    fast = bp.LinkModel(0.0, 1e-11, "measured")
    p = bp.plan_buckets(45 * MIB, 8, fast)
    assert p.bucket_bytes == 4 * MIB and p.tail_bytes == 1 * MIB
    slow = bp.LinkModel(1e-3, 1e-11, "measured")
    p = bp.plan_buckets(45 * MIB, 8, slow)
    assert p.bucket_bytes == 45 * MIB // 2 and p.tail_bytes == p.bucket_bytes


def test_bucketer_tail_bucket():
    """tail_bytes: the first-registered parameters (backward's last gradients) form the last
    bucket, at most tail_bytes (at least one parameter); the rest keep the greedy buckets."""
    from mil_nce_howto100m_amd.parallel.ddp import GradBucketer
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in (10, 20, 30, 40, 50)]
    bk = GradBucketer(ps, 1, bucket_bytes=4 * 60, tail_bytes=4 * 35)
    # backward order 50, 40, 30, 20, 10: greedy 60-element buckets [50], [40], then the tail
    # [20 + 10] split off at its start even though [30] alone would have room for 20 more
    assert bk.buckets == [[0, 50], [50, 90], [90, 120], [120, 150]]
    bk1 = GradBucketer(ps, 1, bucket_bytes=4 * 60, tail_bytes=4)  # tail smaller than any param
    assert bk1.buckets[-1] == [140, 150]  # the first parameter alone
    bk2 = GradBucketer(ps, 1, bucket_bytes=4 * 60)
    assert bk2.buckets == [[0, 50], [50, 90], [90, 150]]


def _worker_autoplan(rank, world, port, outdir):
    ctx = _init(rank, world, port)
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    args = _args()
    assert args.bucket_mb == "auto"
    seed_everything(1, rank)
    model = build_model(args, ctx.device)
    tr = Trainer(args, model, ctx, 10)
    _put(outdir, rank, (tr.comm_plan.as_dict(), [list(b) for b in tr.bucketer.buckets]))
    dist.destroy_process_group()


def test_auto_bucket_plan_same_on_every_rank():
    """--bucket_mb auto at W = 4 on gloo: the all-reduce is timed on the process group, and every
    rank builds the same buckets (a mismatch would pair different slices in the all-reduce)."""
    world, port = 4, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_autoplan, args=(world, port, out), nprocs=world)
        res = _collect(out, world)
    plan0, buckets0 = res[0]
    assert plan0["source"] == "measured" and plan0["world_size"] == world
    assert plan0["tail_bytes"] <= plan0["bucket_bytes"]
    for plan, buckets in res[1:]:
        assert buckets == buckets0
        assert (plan["bucket_bytes"], plan["tail_bytes"]) == (plan0["bucket_bytes"], plan0["tail_bytes"])
