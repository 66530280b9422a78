"""Single-node launcher: one fresh process per GPU, started before anything touches HIP.

Replaces the reference's ``mp.spawn(main_worker, nprocs=torch.cuda.device_count())``
(``main_distributed.py:57-60``). The parent never initialises the GPU runtime: it counts the
visible devices from the environment / the KFD topology in sysfs, picks a free 127.0.0.1 port
and starts ``sys.executable <script> <argv>`` children with the torchrun environment
(``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``LOCAL_WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT``).
Children are plain subprocesses (fork+exec of a fresh interpreter from a process that holds no
GPU state), so every rank owns exactly one device and RCCL sees W independent processes.
"""
from __future__ import annotations

import glob
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _visible_list(var: str) -> Optional[int]:
    v = os.environ.get(var)
    if v is None:
        return None
    v = v.strip()
    return 0 if v in ("", "-1") else len([x for x in v.split(",") if x.strip()])


def count_gpus_no_init() -> int:
    """Visible GPU count without initialising HIP (no ``hipGetDeviceCount``).

    Order: ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` if set,
    else the KFD topology nodes with SIMDs (GPU agents).
    """
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        n = _visible_list(var)
        if n is not None:
            return n
    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(props) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
        except OSError:
            continue
    return n


def rank_env(rank: int, world: int, port: int, addr: str = "127.0.0.1") -> dict:
    env = dict(os.environ)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                "MASTER_ADDR": addr, "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL peer buffers
    return env


def launch_local(script: str, argv: Sequence[str], nprocs: int, poll_s: float = 0.2) -> int:
    """Run ``script argv`` as ``nprocs`` ranks; return the first non-zero exit code (or 0).

    If any rank fails, the others are terminated (a collective would otherwise hang until the
    process-group timeout).
    """
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(nprocs):
        procs.append(subprocess.Popen([sys.executable, "-u", script, *argv], env=rank_env(r, nprocs, port)))
    rc = 0
    try:
        alive = set(range(nprocs))
        while alive:
            for r in list(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    for o in alive:
                        procs[o].send_signal(signal.SIGTERM)
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        rc = 130
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc if rc >= 0 else 128 - rc
