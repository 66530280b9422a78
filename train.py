#!/usr/bin/env python3
"""Multi-node MIL-NCE training (the reference's ``train.py`` with its hard-coded 10-node IP list,
``train.py:48-63``), using standard env rendezvous instead:

    # on every node (N nodes x G GPUs):
    python -m torch.distributed.run --nnodes N --nproc-per-node G --node-rank <i> \
        --master-addr <node0-ip> --master-port 23456 train.py --batch_size <per-node> ...

Each process reads RANK/LOCAL_RANK/WORLD_SIZE from the environment; collectives run on RCCL
(intra-node xGMI, inter-node over the fabric). ``--batch_size`` is per node (divided over the
node's GPUs), as in the reference.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from main_distributed import run  # noqa: E402

if __name__ == "__main__":
    if "WORLD_SIZE" not in os.environ:
        print("train.py expects a torchrun launch (see module docstring); running single-process", file=sys.stderr)
    run(sys.argv[1:])
