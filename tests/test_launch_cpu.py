"""Launcher and gradient-bucket readiness on CPU (gloo, real multi-process rendezvous).

* ``bench.py --gpus N`` with WORLD_SIZE unset starts N ranks itself (reference
  ``main_distributed.py:57-60``) and reports the world size torch.distributed observed;
* a world-size mismatch is an error, never a silent 1-rank measurement;
* GPU counting for the launcher never initialises HIP (env lists / KFD topology);
* ``GradBucketer``: every trainable parameter reports ready each step, every bucket
  is issued exactly once, and no gradient lands in a bucket after it was issued (the
  all-reduce would have read an incomplete slice), at W=2, 4 and 8, one-shot and GradCache.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bucket_recorder import BucketRecorder as _Recorder

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--device", "cpu", "--batch_per_gpu", "2", "--num_frames", "4", "--size", "32", "--blocks", "mixed_3b"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _clean_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("world", [2, 8])
def test_bench_self_launches_n_ranks(world):
    """bench.py --gpus N as its own launcher: N ranks, one JSON line, the world size observed by
    torch.distributed; W = 8 is the driver's scaling-run shape (rehearsed on gloo here)."""
    cmd = [sys.executable, "bench.py", "--gpus", str(world), "--steps", "1", "--warmup", "1", *TINY]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900, env=_clean_env())
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    r = json.loads(lines[0])
    assert r["n_gpus"] == world and r["config"]["parallelism"] == f"dp{world}"
    assert r["config"]["backend"] == "gloo" and r["config"]["global_batch"] == 2 * world
    # the step's collectives timed after the timed region (parallel/comm_probe.py)
    c = r["comm"]
    assert c["world_size"] == world and c["buckets"] >= 1 and c["grad_mib"] > 0
    assert c["allreduce_ms"] > 0 and c["bucketed_allreduce_ms"] > 0 and c["allgather_ms"] > 0
    assert c["allreduce_bf16_ms"] > 0
    # the link-aware bucket plan measured at start-up (--bucket_mb auto, parallel/bucket_plan.py)
    bp = c["bucket_plan"]
    assert bp["source"] == "measured" and bp["world_size"] == world
    assert 0 < bp["tail_bytes"] <= bp["bucket_bytes"]
    assert c["allgather_kib"] == world * 2 * (1 + 4) * 512 * 4 / 1024  # W * b(1+K) rows * 512 fp32


def test_bench_world_size_mismatch_fails():
    env = _clean_env()
    env["WORLD_SIZE"] = "1"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", *TINY]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 2
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_count_gpus_no_init(monkeypatch):
    from mil_nce_howto100m_amd.parallel import launch
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    assert launch.count_gpus_no_init() == 4
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert launch.count_gpus_no_init() == 0
    env = launch.rank_env(3, 8, 1234)
    assert env["RANK"] == "3" and env["WORLD_SIZE"] == "8" and env["MASTER_ADDR"] == "127.0.0.1"


def test_launch_local_propagates_failure():
    from mil_nce_howto100m_amd.parallel.launch import launch_local
    with tempfile.TemporaryDirectory() as d:
        script = os.path.join(d, "w.py")
        with open(script, "w") as f:
            f.write("import os, sys, time\n"
                    "r = int(os.environ['RANK'])\n"
                    "sys.exit(7) if r == 1 else time.sleep(60)\n")
        assert launch_local(script, [], 3) == 7  # rank 1 fails, the sleeping ranks are terminated


# --------------------------------------------------------------------------------------
def _worker_buckets(rank, world, port, outdir, chunks):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    ctx = pdist.init_distributed("gloo", "cpu")
    args = get_args(argv=["--batch_size", str(4 * world), "--num_frames", "4", "--video_size", "32",
                          "--num_candidates", "2", "--blocks", "mixed_3b", "--warmup_steps", "1",
                          "--word2vec_path", "", "--vocab_size", "500", "--bucket_mb", "0.25",
                          "--grad_cache_chunks", str(chunks)])
    seed_everything(1, rank)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 10)
    assert len(tr.bucketer.buckets) > 4
    rec = _Recorder(tr.bucketer)
    data = SyntheticClips(4, 4, 32, 2, 20, 500, device=ctx.device, rank=rank, world_size=world)
    for step in range(2):
        rec.snaps.clear()
        rec.notes.clear()
        orig_finish = tr.bucketer.finish

        def finish_and_check():
            orig_finish()
            snaps = rec.check()  # every param ready once, every bucket issued once, from the hooks
            torch.save(snaps, os.path.join(outdir, f"snap{rank}_{step}.pt"))

        tr.bucketer.finish = finish_and_check
        tr.train_step(data.batch(step))
        tr.bucketer.finish = orig_finish
    torch.save(tr.bucketer.flat.clone(), os.path.join(outdir, f"flat{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(2, 0), (4, 0), (2, 2), (8, 0)])
def test_bucket_readiness_multirank(world, chunks):
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_worker_buckets, args=(world, _port(), out, chunks), nprocs=world)
        snaps = [torch.load(os.path.join(out, f"snap{r}_1.pt")) for r in range(world)]
        flats = [torch.load(os.path.join(out, f"flat{r}.pt")) for r in range(world)]
    # the reduced flat buffer (identical on every rank) is exactly the sum of the slices each
    # rank issued: nothing was added to a bucket after its all-reduce started
    for r in range(1, world):
        assert torch.equal(flats[r], flats[0])
    s0 = torch.cat([sum(s[i] for s in snaps) for i in sorted(snaps[0])])
    assert torch.allclose(s0, flats[0], rtol=1e-5, atol=1e-7)


def test_count_gpus_intersects_visibility(monkeypatch):
    from mil_nce_howto100m_amd.parallel import launch
    monkeypatch.setattr(launch, "_kfd_gpu_count", lambda: 8)
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert launch.count_gpus_no_init() == 8
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")  # indexes into the 4 ROCr left
    assert launch.count_gpus_no_init() == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3,4,5")
    assert launch.count_gpus_no_init() == 4
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setattr(launch, "_kfd_gpu_count", lambda: 2)
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "0,1,2,3")  # lists more than the topology has
    assert launch.count_gpus_no_init() == 2


@pytest.mark.parametrize("sig", ["TERM", "HUP"])
def test_launch_local_forwards_signals(sig):
    """A SIGTERM / SIGHUP to the launcher reaches every rank: none survives it."""
    import signal
    import time
    with tempfile.TemporaryDirectory() as d:
        script = os.path.join(d, "w.py")
        with open(script, "w") as f:
            f.write("import os, time\n"
                    "open(os.path.join(%r, 'pid%%s' %% os.environ['RANK']), 'w').write(str(os.getpid()))\n"
                    "time.sleep(120)\n" % d)
        parent = os.path.join(d, "p.py")
        with open(parent, "w") as f:
            f.write("import sys\nsys.path.insert(0, %r)\n"
                    "from mil_nce_howto100m_amd.parallel.launch import launch_local\n"
                    "sys.exit(launch_local(%r, [], 3, grace_s=5))\n" % (ROOT, script))
        p = subprocess.Popen([sys.executable, parent], env=_clean_env())
        t0 = time.time()
        while len([n for n in os.listdir(d) if n.startswith("pid")]) < 3:
            assert time.time() - t0 < 60 and p.poll() is None
            time.sleep(0.1)
        time.sleep(0.3)
        pids = [int(open(os.path.join(d, f"pid{r}")).read()) for r in range(3)]
        p.send_signal(getattr(signal, "SIG" + sig))
        assert p.wait(timeout=30) == 128 + getattr(signal, "SIG" + sig)
        for pid in pids:
            try:
                os.kill(pid, 0)
                alive = os.path.exists(f"/proc/{pid}") and "zombie" not in open(f"/proc/{pid}/status").read()
            except ProcessLookupError:
                alive = False
            assert not alive, f"rank pid {pid} survived the launcher's SIG{sig}"


def test_launch_local_ranks_die_with_killed_parent():
    """A SIGKILLed launcher (no handler runs) still takes its ranks down (PR_SET_PDEATHSIG)."""
    import signal
    import time
    with tempfile.TemporaryDirectory() as d:
        script = os.path.join(d, "w.py")
        with open(script, "w") as f:
            f.write("import os, time\n"
                    "open(os.path.join(%r, 'pid%%s' %% os.environ['RANK']), 'w').write(str(os.getpid()))\n"
                    "time.sleep(120)\n" % d)
        parent = os.path.join(d, "p.py")
        with open(parent, "w") as f:
            f.write("import sys\nsys.path.insert(0, %r)\n"
                    "from mil_nce_howto100m_amd.parallel.launch import launch_local\n"
                    "sys.exit(launch_local(%r, [], 2))\n" % (ROOT, script))
        p = subprocess.Popen([sys.executable, parent], env=_clean_env())
        t0 = time.time()
        while len([n for n in os.listdir(d) if n.startswith("pid")]) < 2:
            assert time.time() - t0 < 60 and p.poll() is None
            time.sleep(0.1)
        time.sleep(0.3)
        pids = [int(open(os.path.join(d, f"pid{r}")).read()) for r in range(2)]
        p.send_signal(signal.SIGKILL)
        p.wait(timeout=10)
        deadline = time.time() + 15
        for pid in pids:
            while time.time() < deadline:
                if not os.path.exists(f"/proc/{pid}") or "zombie" in open(f"/proc/{pid}/status").read().lower():
                    break
                time.sleep(0.1)
            else:
                raise AssertionError(f"rank pid {pid} outlived its killed launcher")
