"""Rank-consistent kernel autotuning for data parallelism.

Every conv shape / direction picks its kernel variant and persistent grid by timing the
candidates on first use (``hip_ops._tune``). Timed independently on each rank, 8 GPUs could pick
different kernels for the same layer: a straggler for the max-over-ranks step time, and a
rank-dependent summation order (the box-tiled and the v3 / v4 kernel families accumulate in
different orders). Inside ``region()`` (entered by the Trainer around every training step when
the world size is > 1) rank 0 alone times the candidates and publishes each decision through the
process group's c10d store; the other ranks take it from there and launch the same variant.

Decisions are keyed by a running counter plus the caller's problem signature: every rank makes
the same sequence of tuning calls in a DP step (same model, same per-rank batch shape), and a
rank whose signature differs from rank 0's raises instead of silently using a kernel tuned for
another shape. ``plan_hash()`` digests the decisions this process made (bench.py reports it per
rank). The reference has no autotuning; cuDNN's benchmark mode (``--cudnn_benchmark``,
``main_distributed.py:177-178``) is per process, which is what this replaces for the HIP kernels.

Plan table. Timing on first use makes the kernel plan a property of the run (two runs on two
boxes could pick different variants for a near-tie). ``ops/plans/gfx950.json`` holds decisions
recorded on an MI355X, keyed by the same problem signatures, and is valid only for the kernel
sources it was recorded with (``src_sha``: a digest of ``csrc/*.hip`` / ``*.h``) and the arch.
``decide()`` takes a valid table's entry without timing anything (every rank reads the same file,
so no store traffic either) and times only signatures the table lacks. ``plan_source()`` says
where this process's decisions came from; ``save_table()`` (bench.py ``--save_plan``) writes the
decisions of a run. ``MILNCE_PLAN_TABLE``: another table file, or ``0`` to ignore the table.
"""
from __future__ import annotations

import contextlib
import glob
import hashlib
import json
import os
from typing import Callable, Dict, Optional

_STATE = {"store": None, "rank": 0, "world": 1, "active": 0, "n": 0, "prefix": "milnce_tune", "checked": False}
_HASH = hashlib.sha1()
_COUNT = [0]
_ARCH = "gfx950"
_HERE = os.path.dirname(os.path.abspath(__file__))
_CSRC = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "csrc")
DEFAULT_TABLE = os.path.join(_HERE, "plans", _ARCH + ".json")
# table state: entries (None until loaded), why it is unusable, hits / timed decisions, all decisions
_TABLE = {"entries": None, "status": "", "hits": 0, "timed": 0, "path": ""}
_MADE: Dict[str, int] = {}


def source_sha() -> str:
    """Digest of the kernel sources (csrc/*.hip, csrc/*.h) the plan table is valid for."""
    h = hashlib.sha1()
    for f in sorted(glob.glob(os.path.join(_CSRC, "*.hip")) + glob.glob(os.path.join(_CSRC, "*.h"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _table_path() -> str:
    v = os.environ.get("MILNCE_PLAN_TABLE", "")
    return "" if v == "0" else (v or DEFAULT_TABLE)


def _load_table() -> Dict[str, int]:
    if _TABLE["entries"] is not None:
        return _TABLE["entries"]
    path = _table_path()
    _TABLE.update(entries={}, path=path)
    if not path:
        _TABLE["status"] = "disabled"
    elif not os.path.isfile(path):
        _TABLE["status"] = "absent"
    else:
        with open(path) as f:
            t = json.load(f)
        if t.get("arch") != _ARCH:
            _TABLE["status"] = f"arch {t.get('arch')}"
        elif t.get("src_sha") != source_sha():
            _TABLE["status"] = "stale (kernel sources changed since it was recorded)"
        else:
            _TABLE.update(entries={str(k): int(v) for k, v in t.get("entries", {}).items()}, status="valid")
    return _TABLE["entries"]


def plan_source() -> str:
    """'table' (every decision from the plan table), 'tuned' (none), 'mixed', or 'none'."""
    hits, timed = _TABLE["hits"], _TABLE["timed"]
    if hits and not timed:
        return "table"
    if timed and not hits:
        return "tuned"
    return "mixed" if hits else "none"


def table_info() -> dict:
    _load_table()
    return {"source": plan_source(), "table_hits": _TABLE["hits"], "timed": _TABLE["timed"],
            "table": os.path.relpath(_TABLE["path"], os.path.dirname(_CSRC)) if _TABLE["path"] else "",
            "table_status": _TABLE["status"]}


def save_table(path: str = "") -> str:
    """Write this process's decisions (merged over a valid table's entries) as a plan table."""
    path = path or DEFAULT_TABLE
    entries = dict(_load_table())
    entries.update(_MADE)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump({"version": 1, "arch": _ARCH, "src_sha": source_sha(), "entries": dict(sorted(entries.items()))},
                  f, indent=0, sort_keys=False)
        f.write("\n")
    os.replace(tmp, path)
    return path


def configure(store, rank: int, world: int, prefix: str = "milnce_tune") -> None:
    """Use ``store`` (a c10d Store shared by every rank) for decisions inside ``region()``."""
    _STATE.update(store=store if world > 1 else None, rank=rank, world=world, prefix=prefix, checked=False)


def configure_from_process_group() -> bool:
    """configure() from the default torch.distributed group (no-op without one)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() <= 1:
        return False
    from torch.distributed import distributed_c10d as c10d
    configure(c10d._get_default_store(), dist.get_rank(), dist.get_world_size())
    return True


@contextlib.contextmanager
def region(enabled: bool = True):
    """Tuning decisions made inside are rank 0's (when configured and ``enabled``)."""
    if not enabled:
        yield
        return
    _STATE["active"] += 1
    try:
        yield
    finally:
        _STATE["active"] -= 1


def synced() -> bool:
    return _STATE["store"] is not None and _STATE["active"] > 0


def _table_digest() -> str:
    t = _load_table()
    h = hashlib.sha1(json.dumps(sorted(t.items())).encode()).hexdigest()[:16]
    return f"{_TABLE['status']}|{h}"


def _check_table_consistent() -> None:
    """Synced tuning numbers its store keys by a counter that only table misses advance, so every
    rank must see the same table: rank 0 publishes its table status and entry digest, the others
    compare before their first decision (a different MILNCE_PLAN_TABLE per rank, or a checkout
    whose csrc/ differs, would otherwise desynchronise the keys: wrong decisions or a hang)."""
    _STATE["checked"] = True
    store, key = _STATE["store"], f"{_STATE['prefix']}/table"
    mine = _table_digest()
    if _STATE["rank"] == 0:
        store.set(key, mine)
        return
    theirs = store.get(key).decode()
    if theirs != mine:
        raise RuntimeError(f"rank {_STATE['rank']}: kernel-plan table {mine!r} differs from rank 0's {theirs!r} "
                           "(MILNCE_PLAN_TABLE / csrc sources must match on every rank)")


def decide(sig: str, tune: Callable[[], int]) -> int:
    """The variant code for problem ``sig``: the plan table's entry, else ``tune()`` here, or rank
    0's choice when synced. A rank-0 ``tune()`` that raises publishes the error, so the other ranks
    raise too instead of waiting for a decision that never comes."""
    if synced() and not _STATE["checked"]:
        _check_table_consistent()
    table = _load_table()
    if sig in table:
        value = table[sig]
        _TABLE["hits"] += 1
    elif synced():
        _TABLE["timed"] += 1
        _STATE["n"] += 1
        key = f"{_STATE['prefix']}/{_STATE['n']}"
        store = _STATE["store"]
        if _STATE["rank"] == 0:
            try:
                value = int(tune())
            except BaseException as e:
                store.set(key, json.dumps([sig, None, f"{type(e).__name__}: {e}"]))
                raise
            store.set(key, json.dumps([sig, value]))
        else:
            got = json.loads(store.get(key).decode())
            sig0, value = got[0], got[1]
            if value is None:
                raise RuntimeError(f"rank {_STATE['rank']}: rank 0 failed to tune {sig0!r}: {got[2]}")
            if sig0 != sig:
                raise RuntimeError(f"rank {_STATE['rank']}: tuning call {_STATE['n']} is for {sig!r}, rank 0 tuned "
                                   f"{sig0!r}: the ranks ran different shapes inside a synced tuning region")
    else:
        _TABLE["timed"] += 1
        value = int(tune())
    _MADE[sig] = value
    _HASH.update(f"{sig}={value};".encode())
    _COUNT[0] += 1
    return value


def plan_hash() -> Optional[str]:
    """Digest of every tuning decision of this process (None before the first)."""
    return _HASH.hexdigest()[:16] if _COUNT[0] else None


def decisions() -> int:
    return _COUNT[0]
