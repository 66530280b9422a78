"""Rank-consistent decisions under data parallelism (CPU / gloo, 2 real rank processes).

* ops/tune_sync: inside a synced region every rank uses rank 0's kernel-variant choice (the other
  ranks do not time anything), the plan hash is identical on every rank, and a rank that asks for
  a different problem than rank 0 tuned raises instead of using the wrong kernel;
* the Trainer's ``--grad_cache_chunks -1`` decision is collective (largest count any rank needs),
  and a budget below one clip raises instead of silently running the one-shot step.
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


def _init(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from mil_nce_howto100m_amd.parallel import dist as pdist
    return pdist.init_distributed("gloo", "cpu")


def _worker_tune(rank, world, port, outdir):
    _init(rank, world, port)
    from mil_nce_howto100m_amd.ops import tune_sync
    assert tune_sync.configure_from_process_group()
    timed = []

    def tuner(value):
        def f():
            timed.append(value)
            return value
        return f

    # outside a region: local decisions
    local = tune_sync.decide("probe", tuner(100 + rank))
    with tune_sync.region():
        a = tune_sync.decide("fwd|B4|64>192", tuner(10 + rank))
        b = tune_sync.decide("wgrad|B4|64>192", tuner(20 + 3 * rank))
        mismatch = None
        try:
            tune_sync.decide(f"dgrad|rank{rank}", tuner(1))
        except RuntimeError as e:
            mismatch = str(e)
    torch.save({"local": local, "a": a, "b": b, "timed": timed, "mismatch": mismatch,
                "hash": tune_sync.plan_hash()}, os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_rank0_decides_inside_region():
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_tune, args=(world, port, out), nprocs=world)
        r0, r1 = (torch.load(os.path.join(out, f"r{r}.pt")) for r in range(world))
    assert (r0["local"], r1["local"]) == (100, 101)  # no sync outside the region
    assert (r0["a"], r0["b"]) == (r1["a"], r1["b"]) == (10, 20)
    # rank 1 timed nothing inside the region (only its local probe)
    assert r1["timed"] == [101] and r0["timed"][:3] == [100, 10, 20]
    assert r0["mismatch"] is None and "rank 0 tuned" in r1["mismatch"]


def _worker_chunks(rank, world, port, outdir, budgets):
    ctx = _init(rank, world, port)
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    args = get_args(argv=["--batch_size", "8", "--num_frames", "4", "--video_size", "32", "--num_candidates", "2",
                          "--blocks", "mixed_3b", "--warmup_steps", "1", "--word2vec_path", "",
                          "--vocab_size", "500", "--grad_cache_chunks", "-1"])
    seed_everything(1, rank)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 10)
    video = torch.zeros((4, 3, 32, 200, 200), dtype=torch.uint8)  # 4 clips of 32 x 200^2 per rank
    per_clip = Trainer.GIB_PER_CLIP_32F200 * 2 ** 30
    tr._memory_budget = lambda: budgets[rank] * per_clip
    res = {}
    try:
        res["chunks"] = tr.grad_cache_chunks(video_batch=video)
    except RuntimeError as e:
        res["error"] = str(e)
    torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    from mil_nce_howto100m_amd.parallel import dist as pdist
    pdist.destroy()


@pytest.mark.parametrize("budgets,expect", [((10.0, 10.0), 0), ((10.0, 2.5), 2), ((1.5, 10.0), 3)])
def test_grad_cache_auto_is_collective(budgets, expect):
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_chunks, args=(world, port, out, budgets), nprocs=world)
        res = [torch.load(os.path.join(out, f"r{r}.pt")) for r in range(world)]
    assert [r["chunks"] for r in res] == [expect, expect]


def test_grad_cache_auto_raises_below_one_clip():
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_chunks, args=(1, port, out, (0.5,)), nprocs=1)
        res = torch.load(os.path.join(out, "r0.pt"))
    assert "less than one clip" in res["error"]


def test_grad_cache_auto_raises_on_every_rank():
    # only rank 1 is short of memory: both ranks raise (after the collective), neither hangs
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_chunks, args=(world, port, out, (10.0, 0.5)), nprocs=world)
        res = [torch.load(os.path.join(out, f"r{r}.pt")) for r in range(world)]
    assert all("less than one clip" in r.get("error", "") for r in res), res


def _worker_tune_fail(rank, world, port, outdir):
    _init(rank, world, port)
    from mil_nce_howto100m_amd.ops import tune_sync
    assert tune_sync.configure_from_process_group()

    def bad():
        raise ValueError("no kernel variant supports this shape")

    err = None
    with tune_sync.region():
        try:
            tune_sync.decide("fwd|unsupported", bad)
        except Exception as e:  # rank 0: its own error; rank 1: the published one (no hang)
            err = f"{type(e).__name__}: {e}"
    torch.save({"err": err}, os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_rank0_tune_error_reaches_every_rank():
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_tune_fail, args=(world, port, out), nprocs=world)
        r0, r1 = (torch.load(os.path.join(out, f"r{r}.pt")) for r in range(world))
    assert r0["err"].startswith("ValueError")
    assert "rank 0 failed to tune" in r1["err"] and "no kernel variant" in r1["err"]


def test_plan_table_hit_miss_and_staleness(tmp_path, monkeypatch):
    from mil_nce_howto100m_amd.ops import tune_sync as ts
    path = str(tmp_path / "plan.json")
    monkeypatch.setenv("MILNCE_PLAN_TABLE", path)

    def reset():
        ts._TABLE.update(entries=None, status="", hits=0, timed=0, path="")
        ts._MADE.clear()

    reset()
    timed = []
    assert ts.decide("fwd|a", lambda: timed.append("a") or 7) == 7  # no table: timed
    assert ts.table_info()["table_status"] == "absent" and ts.plan_source() == "tuned"
    ts.save_table(path)
    reset()
    assert ts.decide("fwd|a", lambda: timed.append("a2") or 9) == 7  # from the table, nothing timed
    assert timed == ["a"] and ts.plan_source() == "table"
    assert ts.decide("fwd|b", lambda: 3) == 3 and ts.plan_source() == "mixed"
    # a table recorded for other kernel sources is ignored
    import json
    with open(path) as f:
        t = json.load(f)
    t["src_sha"] = "0" * 16
    with open(path, "w") as f:
        json.dump(t, f)
    reset()
    assert ts.decide("fwd|a", lambda: 11) == 11 and ts.table_info()["table_status"].startswith("stale")
    reset()
