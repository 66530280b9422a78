"""One-shot xGMI peer-write all-gather (parallel/peer.py) between two rank processes sharing the
box's one MI355X: receive buffers exported / mapped by IPC handle, each rank's slice written by
the native scatter kernel, gloo fence. Checks the rank-major result over both alternating receive
buffers and three shapes / dtypes, the local-slice backward of all_gather_embeddings on that path,
and that the comm probe reports both gather paths at W = 2 on one device."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_peer_allgather_two_processes_one_device():
    world, port = 2, _port()
    with tempfile.TemporaryDirectory() as out:
        procs = []
        for r in range(world):
            env = dict(os.environ)
            env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world),
                        "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                        "MILNCE_DEVICE_INDEX": "0", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "peer_worker.py"), out],
                                          env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
        logs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=180)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            logs.append(o)
        for p, o in zip(procs, logs):
            assert p.returncode == 0, o[-3000:]
        res = [json.load(open(os.path.join(out, f"peer_r{r}.json"))) for r in range(world)]
    for r in res:
        assert r["checks"] == 9
        c = r["comm"]
        print(json.dumps(c))
        assert c["peer_allgather_matches"] is True and c["peer_allgather_ms"] > 0 and c["allgather_ms"] > 0
