"""Data parallelism with real collectives next to the HIP kernels on a GPU.

Two fresh rank processes share the box's one MI355X over a gloo process group (RCCL refuses two
ranks on one device; ``MILNCE_DEVICE_INDEX`` pins both to cuda:0). They run the production
Trainer (tests/dp_worker.py): HIP kernels writing weight / BN gradients straight into the flat
buffer, the GradBucketer's async all-reduces issued as buckets fill during backward (ordering
verifier on), the packed embedding all-gather with local-slice backward, fused Adam. Checks:

* the reduced flat gradient at W=2 equals the single-process gradient of the concatenated batch
  (the sum of the ranks' local-slice gradients; the optimizer applies the reference's 1/W, SURVEY
  §2.10 item 2), one-shot and GradCache, with eval-mode BN so both runs see the same batch;
* the loss is bitwise identical on both ranks (computed redundantly on the gathered batch);
* after two train steps every rank holds bitwise identical parameters;
* the comm probe runs at W=2 on the step's sizes.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dp_worker.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(out, world, chunks, production=False):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world), "LOCAL_WORLD_SIZE": str(world),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "MILNCE_DEVICE_INDEX": "0",
                    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                    # one conv kernel family whatever the batch split: the v3 / v4 variants sum in
                    # the same order (bitwise equal), the box-tiled ones (csrc/conv_box.hip) in
                    # another, and at random init the network amplifies bf16-level differences
                    # between the W=1 and W=2 kernel choices to several % of the gradient
                    "MILNCE_BOX": "0"})
        if production:  # the bench's kernel set (box-tiled variants included)
            env.pop("MILNCE_BOX")
        argv = [out, str(chunks)] + (["auto"] if production else [])  # production: the default bucket plan
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, *argv], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o)
    for p, o in zip(procs, logs):
        assert p.returncode == 0, o[-3000:]


def _load(out, world, r):
    with open(os.path.join(out, f"res_w{world}_r{r}.json")) as f:
        res = json.load(f)
    res["bufs"] = torch.load(os.path.join(out, f"bufs_w{world}_r{r}.pt"))
    return (res, torch.load(os.path.join(out, f"grad_w{world}_r{r}.pt")),
            torch.load(os.path.join(out, f"param_w{world}_r{r}.pt")))


@pytest.mark.parametrize("chunks", [0, 2])
def test_two_ranks_on_gpu_match_single_process(chunks):
    with tempfile.TemporaryDirectory() as out:
        _run(out, 1, chunks)
        _run(out, 2, chunks)
        ref, g1, _ = _load(out, 1, 0)
        (r0, g20, p20), (r1, g21, p21) = _load(out, 2, 0), _load(out, 2, 1)
    # every rank holds the same reduced gradient, the loss was computed on the same gathered batch
    assert torch.equal(g20, g21)
    assert r0["loss"] == r1["loss"]
    assert abs(r0["loss"] - ref["loss"]) < 1e-3 * max(1.0, abs(ref["loss"]))
    # sum of the ranks' local-slice gradients == the single-process gradient of the whole batch
    rel = ((g20 - g1).norm() / g1.norm()).item()
    assert torch.isfinite(g20).all() and rel < 2e-2, rel
    cos = torch.nn.functional.cosine_similarity(g20, g1, dim=0).item()
    assert cos > 0.999, cos
    # identical updates on both ranks after real train steps (bucket verifier on)
    assert torch.equal(p20, p21)
    # the flat BN-buffer broadcast (parallel/ddp.py BufferBroadcaster) through one-shot and GradCache
    # train steps: the buffers stayed views of its flats and every rank holds rank 0's statistics
    assert torch.equal(r0["bufs"], r1["bufs"])
    assert r0["bcast"]["flats"] >= 1 and r0["bcast"]["intact"] and r0["bcast"]["reflattens"] == 0
    assert r1["bcast"] == r0["bcast"]
    for k in ("train_loss1", "train_loss2"):
        assert r0[k] == r1[k]
    c = r0["comm"]
    assert c["world_size"] == 2 and c["buckets"] >= 2 and c["allreduce_ms"] > 0 and c["allgather_ms"] > 0


def test_two_ranks_production_kernels_rank_consistent():
    """Production defaults (box-tiled kernels in the tuner, the measured bucket plan, as in
    bench.py): rank 0 tunes and every rank launches its choices (ops/tune_sync), so both ranks hold
    the same plan and, after two real train steps, bitwise identical parameters and losses
    (VERDICT r3 item 5)."""
    with tempfile.TemporaryDirectory() as out:
        _run(out, 2, 0, production=True)
        (r0, g0, p0), (r1, g1, p1) = _load(out, 2, 0), _load(out, 2, 1)
    assert r0["plan_hash"] is not None and r0["plan_hash"] == r1["plan_hash"]
    assert r0["tune_decisions"] == r1["tune_decisions"] > 0
    assert torch.equal(g0, g1)
    assert r0["loss"] == r1["loss"]
    for k in ("train_loss1", "train_loss2"):
        assert r0[k] == r1[k]
    assert torch.equal(p0, p1)
    # --bucket_mb auto: the plan measured on the process group at start-up, the same buckets on both
    assert r0["bucket_plan"]["source"] == "measured" and r0["buckets"] == r1["buckets"]
    assert r0["bucket_plan"]["bucket_bytes"] == r1["bucket_plan"]["bucket_bytes"]
