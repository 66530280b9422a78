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


def _visible_list(var: str) -> Optional[List[str]]:
    v = os.environ.get(var)
    if v is None:
        return None
    v = v.strip()
    return [] if v in ("", "-1") else [x.strip() for x in v.split(",") if x.strip()]


def _kfd_gpu_count() -> int:
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


def count_gpus_no_init() -> int:
    """Visible GPU count without initialising HIP (no ``hipGetDeviceCount``).

    The visibility variables filter in layers: ``ROCR_VISIBLE_DEVICES`` selects from the KFD
    agents, then ``HIP_VISIBLE_DEVICES`` (or ``CUDA_VISIBLE_DEVICES``) indexes into what ROCr
    left. So the count is the most restrictive of every list that is set, capped by the KFD
    GPU agents when the topology is readable. Children still check ``local_rank`` against
    ``torch.cuda.device_count()`` (``check_local_rank``), since a container can list agents it
    cannot open.
    """
    counts = []
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        lst = _visible_list(var)
        if lst is not None:
            counts.append(len(lst))
    kfd = _kfd_gpu_count()
    if kfd > 0:
        counts.append(kfd)
    return min(counts) if counts else 0


def check_local_rank(local_rank: int) -> None:
    """Fail with a clear message when a rank has no device of its own (more ranks were started
    than this process can open)."""
    import torch
    n = torch.cuda.device_count()
    if local_rank >= n:
        raise SystemExit(f"local rank {local_rank} has no GPU: this process sees {n} device(s); "
                         f"start at most {n} ranks per node (check *_VISIBLE_DEVICES)")


def rank_env(rank: int, world: int, port: int, addr: str = "127.0.0.1") -> dict:
    env = dict(os.environ)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                "MASTER_ADDR": addr, "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL peer buffers
    return env


def _die_with_parent() -> None:
    """preexec_fn of every rank: SIGTERM the child when the launcher dies (PR_SET_PDEATHSIG),
    so a SIGKILLed launcher cannot leave ranks blocked in a collective holding their GPU."""
    try:
        import ctypes
        libc = ctypes.CDLL("libc.so.6", use_errno=True)
        libc.prctl(1, signal.SIGTERM, 0, 0, 0)  # PR_SET_PDEATHSIG = 1
    except OSError:
        pass


def _terminate(procs: List[subprocess.Popen], sig: int = signal.SIGTERM) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(sig)
            except ProcessLookupError:
                pass


def launch_local(script: str, argv: Sequence[str], nprocs: int, poll_s: float = 0.2,
                 grace_s: float = 30.0) -> int:
    """Run ``script argv`` as ``nprocs`` ranks; return the first non-zero exit code (or 0).

    If any rank fails, the others are terminated (a collective would otherwise hang until the
    process-group timeout). SIGINT / SIGTERM / SIGHUP sent to the launcher are forwarded to every
    rank, which then gets ``grace_s`` to exit before SIGKILL; ranks also carry
    PR_SET_PDEATHSIG, so they die with a launcher that was killed outright.
    """
    port = free_port()
    procs: List[subprocess.Popen] = []
    received: List[int] = []

    def on_signal(signum, frame):  # noqa: ARG001
        received.append(signum)
        _terminate(procs, signal.SIGTERM)

    old = {}
    for sig in (signal.SIGINT, signal.SIGTERM, signal.SIGHUP):
        try:
            old[sig] = signal.signal(sig, on_signal)
        except ValueError:  # not the main thread: no handlers, PDEATHSIG still applies
            pass
    rc = 0
    try:
        for r in range(nprocs):
            procs.append(subprocess.Popen([sys.executable, "-u", script, *argv], env=rank_env(r, nprocs, port),
                                          preexec_fn=_die_with_parent))
            if received:
                break
        alive = set(range(len(procs)))
        while alive:
            for r in list(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    _terminate([procs[o] for o in alive])
            if received:
                break
            time.sleep(poll_s)
    finally:
        if received:
            _terminate(procs)
        deadline = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for sig, h in old.items():
            signal.signal(sig, h)
    if received:
        return 128 + received[0]
    return rc if rc >= 0 else 128 - rc


def _device_flag(argv: Sequence[str]) -> str:
    """--device as argparse reads it (``--device cpu``, ``--device=cpu``, unambiguous prefixes)."""
    import argparse
    ap = argparse.ArgumentParser(add_help=False, allow_abbrev=True)
    ap.add_argument("--device", default="auto")
    known, _ = ap.parse_known_args(list(argv))
    return known.device


def run_per_gpu(script: str, argv: Sequence[str], run) -> int:
    """Entry-point process model shared by ``main_distributed.py`` and the ``eval_*.py`` scripts:
    under torchrun (``WORLD_SIZE`` set) or on CPU run this process as one rank; otherwise start
    one fresh rank per visible GPU (counted without initialising HIP) and wait for them. This is
    the reference's DataParallel eval (``eval_hmdb.py:27,32``) done as one process per GPU."""
    argv = list(argv)
    if "WORLD_SIZE" in os.environ:
        return run(argv)
    if _device_flag(argv) == "cpu":
        return run(argv)
    n = count_gpus_no_init()
    if n <= 1:
        return run(argv)
    return launch_local(os.path.abspath(script), argv, n)
