"""Autograd Functions over the HIP kernels (GPU path). Activations are bf16 NDHWC.

Every forward and backward here is a call into ``libmilnce_hip.so``; the only library GEMMs
are the tiny, plain ones (text tower fc1/fc2, video fc, the MIL-NCE logits, the gating fc of
the stem) which go to hipBLASLt through ``torch.mm``. Shapes are planned once per
(layer geometry, input shape) and cached.
"""
from __future__ import annotations

import collections
import ctypes
import os
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import aten, grad_sink, tune_sync
from ._lib import UnsupportedVariant, call, lib, ptr, stream

BF16 = torch.bfloat16
F32 = torch.float32


class _ZeroArena:
    """Small zero-initialised fp32 accumulators (SelfGating channel sums, gate-backward dots) carved
    from one buffer that a single fill re-zeroes per training step, instead of one
    ``torch.zeros`` launch each (~80 fills per flagship step). Only active between
    ``zero_arena_begin()`` and ``zero_arena_end()`` (the trainer brackets its step with them), so
    nothing handed out can outlive the step; elsewhere, on the first step (sizing) and on overflow
    it falls back to ``torch.zeros``. Slices are built with ``set_`` rather than as views, so each
    has its own autograd version counter."""

    ALIGN = 64  # fp32 elements: 256-B aligned slices

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None
        self.off = 0
        self.demand = 0
        self.active = False

    def begin(self, device: torch.device) -> None:
        if self.demand and (self.buf is None or self.buf.numel() < self.demand or self.buf.device != device):
            self.buf = torch.zeros(self.demand, dtype=F32, device=device)  # fresh zeros
        elif self.buf is not None and self.off:
            self.buf[:self.off].zero_()  # the slices handed out during the previous step
        self.off = 0
        self.demand = 0
        self.active = True

    def end(self) -> None:
        self.active = False

    def zeros(self, shape: Tuple[int, ...], device: torch.device) -> torch.Tensor:
        n = math.prod(shape)
        if not self.active:
            return torch.zeros(shape, dtype=F32, device=device)
        na = _ceil(n, self.ALIGN) * self.ALIGN
        self.demand += na
        buf = self.buf
        if buf is None or buf.device != device or self.off + na > buf.numel():
            return torch.zeros(shape, dtype=F32, device=device)
        stride = tuple(math.prod(shape[i + 1:]) for i in range(len(shape)))
        t = torch.empty(0, dtype=F32, device=device).set_(buf.untyped_storage(), self.off, tuple(shape), stride)
        self.off += na
        return t


_ARENA = _ZeroArena()


def zero_arena_begin(device: torch.device) -> None:
    """Training-step start: re-zero the accumulator arena and pre-pack the step's conv weights."""
    if device.type == "cuda":
        _ARENA.begin(device)
        _PACKER.begin(device)
        _refresh_headroom(device)


def zero_arena_end() -> None:
    _ARENA.end()
    _PACKER.end()


def _zeros_f32(shape: Tuple[int, ...], device: torch.device) -> torch.Tensor:
    return _ARENA.zeros(tuple(int(v) for v in shape), device)


def _ceil(a: int, b: int) -> int:
    return (a + b - 1) // b


# MILNCE_TUNE_LOG=path: append one line per wgrad tuning decision (layer shape -> kernel), for
# mapping a step trace's kernels to layers (tools/gpu scripts)
_TUNE_LOG = os.environ.get("MILNCE_TUNE_LOG", "")


def _tune_log(line: str) -> None:
    if _TUNE_LOG:
        with open(_TUNE_LOG, "a") as f:
            f.write(line + "\n")


def _plan_sig(plan) -> str:
    """Problem identity of a conv plan for rank-consistent tuning (tune_sync). Callers prefix the
    call context (direction, prologue, statistics / partial-row epilogue: ``_ctx_key``), so a
    variant is always timed for exactly the call that launches it."""
    return (f"|B{plan.B}T{plan.T}H{plan.H}W{plan.W}|{plan.Cin}>{plan.Cout}|k{plan.k}s{plan.s}p{plan.p}"
            f"|wo{plan.wo_override}")


# Plan hygiene counters (bench.py reports them under "plan"): ``fallbacks`` = launches whose tuned
# variant could not run in the call and ran as another, untimed variant. Every forward / dgrad
# call context is tuned on its own (ConvPlan.ctx), so this stays 0 unless a plan table entry
# disagrees with the running kernels.
_PLAN_EVENTS = {"fallbacks": 0, "contexts": 0}


def plan_events() -> dict:
    return dict(_PLAN_EVENTS)


def _decision(plan: "ConvPlan", ck: str, dgrad: bool, tune) -> Tuple[int, int]:
    """(variant, grid) of ``plan`` for call context ``ck``: the pinned variant, else the context's
    tuned decision (``tune()`` on its first call)."""
    pin = plan.pin_d if dgrad else plan.pin_f
    if pin:
        return pin, (plan.d_grid_m if dgrad else plan.grid_m)
    if ck not in plan.ctx:
        plan.ctx[ck] = tune()
        _PLAN_EVENTS["contexts"] += 1
    return plan.ctx[ck]


def _ctx_key(kind: str, *flags: str) -> str:
    """Call-context key of a tuned decision: kind (fwd / fwdpro / dgrad / dgradbn) plus flags
    (st: BN-statistics epilogue, p: producer-BN partial rows, fz / nf: the prologue input can /
    cannot be staged by the fused kernel)."""
    return kind + "".join("|" + f for f in flags if f)


# =========================================================================================
# Conv + BN + ReLU
# =========================================================================================
@dataclass
class ConvPlan:
    B: int
    T: int
    H: int
    W: int
    Cin: int       # channels as stored in x (4 for the stem)
    Cin_p: int     # channels of the weight parameter (3 for the stem)
    Cout: int
    k: Tuple[int, int, int]
    s: Tuple[int, int, int]
    p: Tuple[int, int, int]
    To: int
    Ho: int
    Wo: int
    M: int
    Ktot: int
    bn: int
    bk: int
    Npad: int
    Kpad: int
    grid_m: int
    # dgrad (stride 1 only)
    d_bn: int
    d_bk: int
    d_Npad: int
    d_Kpad: int
    d_grid_m: int
    # wgrad
    w_tn: int
    w_tk: int
    w_Npad: int
    w_Kpad: int
    w_splits: int
    wo_override: int = 0  # asymmetric w padding (paired-width stem): explicit output width
    impl: int = 0         # forward kernel variant (csrc/conv.hip launch_v3_impl); 0 = not tuned yet
    d_impl: int = 0       # dgrad kernel variant
    w_impl: int = 0       # wgrad kernel variant (2: register-staged, 3/4: LDS-DMA ring, 3/2 stages)
    w_occ: int = 4        # wgrad split-K target: workgroups per CU (fewer splits = smaller slab to reduce)
    # forward / dgrad decisions per call context (_ctx_key -> (variant, persistent grid)); impl /
    # grid_m and d_impl / d_grid_m hold the ones of the latest call
    ctx: Dict[str, Tuple[int, int]] = field(default_factory=dict)
    # tests / tools pin a variant for every context (the grid is then grid_m / d_grid_m as set)
    pin_f: int = 0
    pin_d: int = 0

    @property
    def taps(self) -> int:
        return self.k[0] * self.k[1] * self.k[2]


_PLANS: Dict[tuple, ConvPlan] = {}
_NUM_CU = 256
# CUs the wgrad split geometry fills (_wgrad_geom / halo / temporal-box plans); a side-stream wgrad
# may be launched on a fraction of them (MILNCE_SIDE_GRID_FRAC, A/B knob) to leave the rest of the
# chip to the main chain's kernels
_GRID_CU = [_NUM_CU]
_SIDE_GRID_FRAC = float(os.environ.get("MILNCE_SIDE_GRID_FRAC", "1.0"))
# LDS floor (KiB) per workgroup of the side-stream wgrads (csrc/common.h lds_floor): fewer wgrad
# workgroups per CU, LDS left for the main chain's kernels. 0 = off.
_SIDE_LDS_FLOOR = int(float(os.environ.get("MILNCE_SIDE_LDS_FLOOR", "0")) * 1024)


_WIDE_BN = (96, 160, 192)  # N tiles served by the LDS-DMA ring kernels only (csrc/conv.hip)
# persistent forward / dgrad workgroups per CU (each loops over M tiles). 2 = exactly the residency
# of the usual 2-stage ring variant (no second partial round of workgroups, half the BN partial
# rows): same-box bench 65.3 ms at 4, 64.4 at 2, 66.3 at 3, 69.6 at 1. MILNCE_FWD_WGS overrides.
_FWD_WGS_PER_CU = int(os.environ.get("MILNCE_FWD_WGS", "2"))
# their variants: 3 / 4 (128-row tiles, 3 / 2 stages); 192 also splits into the BK-32 4-stage
# ring (5) (csrc/conv.hip v3_fits). Its 256-row 8-wave tiles (7) win the isolated timing of the
# conv_2c dgrad but run 2.1 ms instead of 0.9 ms inside the step, so the tuner does not offer them.
_WIDE_IMPLS = {96: (3, 4), 160: (3, 4), 192: (3, 4, 5)}


# persistent grid sizes (workgroups per CU) the forward / dgrad tuner tries per shape next to the
# kernel variant: narrow tiles (BN 64: 48 KiB of LDS) fit three workgroups per CU, where the global
# default of two leaves a third of the LDS idle. MILNCE_FWD_WGS_TUNE="2" restores the fixed grid.
_FWD_WGS_TUNE = tuple(int(v) for v in os.environ.get("MILNCE_FWD_WGS_TUNE", "2,3").split(","))


# Persistent grids split their work statically over the workgroups, so a count just above the
# resident capacity (wgs per CU x CUs, rounded UP to a multiple of the N tiles) leaves a last round
# of a few workgroups that each run a full share while the chip idles. Round down instead
# (csrc/common.h fill_splits, the same rule for the halo / temporal wgrad split counts);
# MILNCE_SPLIT_CEIL=1 restores the rounded-up counts (A/B).
_SPLIT_CEIL = os.environ.get("MILNCE_SPLIT_CEIL", "0") == "1"


def _fill(target: int, ntiles: int) -> int:
    return max(1, _ceil(target, ntiles) if _SPLIT_CEIL else target // ntiles)


def _grid_for(M: int, npad: int, bn: int, wgs: int) -> int:
    return max(1, min(_ceil(M, 128), _fill(wgs * _NUM_CU, npad // bn)))


def _stats_rows(M: int, npad: int, bn: int) -> int:
    """Partial-statistics rows to allocate: the largest grid the tuner may pick."""
    return max(_grid_for(M, npad, bn, w) for w in (_FWD_WGS_PER_CU,) + _FWD_WGS_TUNE)


def _tune_fwd(launch, plan_impls: Tuple[int, ...], M: int, npad: int, bn: int,
              max_rows: Optional[int] = None, sig: str = "") -> Tuple[int, int]:
    """(impl, grid) of the fastest (kernel variant, persistent grid) pair; launch(impl, grid).
    Grids with more partial-statistics rows than ``max_rows`` (the caller's buffer) are skipped.
    ``sig`` names the problem for rank-consistent tuning (tune_sync)."""
    wgs = tuple(w for w in dict.fromkeys((_FWD_WGS_PER_CU,) + _FWD_WGS_TUNE)
                if w == _FWD_WGS_PER_CU or max_rows is None or _grid_for(M, npad, bn, w) <= max_rows)
    code = {(i, w): 10 * i + w for i in plan_impls if i not in _V4_WIDE_M + _BOX4_IMPLS for w in wgs}
    code.update({(i, w): 10 * i + w for i in plan_impls if i in _V4_WIDE_M for w in (1, 2)})
    # 4-wave box workgroups: two per CU is their residency (80 KiB of LDS each)
    code.update({(i, 2): 10 * i + 2 for i in plan_impls if i in _BOX4_IMPLS})
    inv = {v: k for k, v in code.items()}
    best = _tune(lambda c: launch(inv[c][0], _grid_for(M, npad, _box_eff_bn(inv[c][0], bn), inv[c][1])),
                 tuple(code.values()),
                 default=code.get((_DEFAULT_IMPL, _FWD_WGS_PER_CU)),
                 sig=f"{sig}|M{M}|N{npad}|bn{bn}|{sorted(code.values())}")
    if best not in inv:  # autotune off: the default variant on the default grid
        return best, _grid_for(M, npad, bn, _FWD_WGS_PER_CU)
    impl, w = inv[best]
    return impl, _grid_for(M, npad, _box_eff_bn(impl, bn), w)


_BOX4_FALLBACK = True  # (tests that pin a variant turn it off to see the refusal)


def _launch_tuned(launch, impl: int, grid: int, bn: int) -> None:
    """launch(impl, grid) with a plan's tuned variant. A plan is tuned on its first call, and a
    later call of the same shape can add LDS the timed launches did not have (producer-BN partial
    rows in a dgrad epilogue, BN statistics in a forward one): a 4-wave box variant that fit 80 KiB
    then no longer does. It runs as its 8-wave sibling instead (160 KiB; the same MFMA shape and
    summation order, so the same conv output bitwise; impl 15 for impl 16's 192-wide plans, which
    14 has no tile for) on the same grid, so the partial-row count matches (slots without a tile
    write zero rows). Every rank shares the plan (tune_sync) and so takes the same fallback."""
    try:
        launch(impl, grid)
        return
    except UnsupportedVariant:
        if impl not in _BOX4_IMPLS or not _BOX4_FALLBACK:
            raise
    _PLAN_EVENTS["fallbacks"] += 1
    launch(15 if impl == 17 or bn == 192 else 14, grid)


# v4 forward / dgrad (csrc/conv_v4.hip): LDS-DMA ring with scalar per-stage offsets, for convs
# whose input channel count is a multiple of 64 (every 64-wide K stage inside one tap). 8 / 10:
# 16x16x32 MFMA, 2 / 3 stages; 9 / 11: 32x32x16 MFMA (N tiles 64 / 128 / 192). MILNCE_V4=0
# leaves them out of the tuner (A/B runs); MILNCE_V4_IMPLS restricts the set.
_V4 = os.environ.get("MILNCE_V4", "1") != "0"
_V4_IMPLS = tuple(int(v) for v in os.environ.get("MILNCE_V4_IMPLS", "8,9,10,11,12,13").split(","))
# 12 / 13: 256-row tiles with 8 waves (one workgroup per CU at N 192 / 128): tuned on 1 or 2
# workgroups per CU of persistent grid instead of 2 or 3
_V4_WIDE_M = (12, 13, 14, 15)  # 8-wave workgroups, one per CU (12 / 13 v4, 14 / 15 box-tiled)

# Box-tiled forward / dgrad (csrc/conv_box.hip): stride-1 same-padded (1,3,3) / (3,1,1) convs over a
# multiple of 8 channels; the tile's input box is staged once per 64-channel block for every tap (a
# partial last block is zero-filled: the tuner weighs that MFMA waste against the other variants).
# 14: 16x16x32 MFMA (N tiles 64 / 96 / 128 / 160), 15: 32x32x16 (64 / 128 / 192). MILNCE_BOX=0 leaves
# them out.
_BOX = os.environ.get("MILNCE_BOX", "1") != "0"
_BOX_ROWS = 448
# 16 / 17: the box kernels on 4-wave workgroups, two per CU (128-row tiles, a 288-row (1,3,3) /
# 192-row (3,1,1) box, <= 80 KiB of LDS): one workgroup's barrier / stage waits / epilogue stores
# overlap the other's MFMAs. 16 runs a 192-wide N tile as two 96-wide ones. MILNCE_BOX4=0 leaves
# them out.
_BOX4 = os.environ.get("MILNCE_BOX4", "1") != "0"
_BOX4_IMPLS = (16, 17)


def _box_eff_bn(impl: int, bn: int) -> int:
    """N tile a (box) variant runs for the plan's N tile (csrc/conv_box.hip box_bn)."""
    return 96 if impl == 16 and bn == 192 else bn


def _box4_lds(bn: int, ks: tuple, pro: int = 0, epi: int = 0, cin: int = 0) -> int:
    """LDS bytes of a 4-wave box variant (csrc/conv_box.hip launch_box_t)."""
    k133 = tuple(ks) == (1, 3, 3)
    stages = (3 if bn <= 64 else 2) if k133 else (4 if bn <= 64 else 3 if bn <= 128 else 2)
    bnr = _ceil(bn, 32) * 32
    return ((288 if k133 else 192) * 160 + stages * bnr * 128 + (16 * bn + 256 if epi == 2 else 4 * bn if epi == 1 else 0)
            + (28 * cin if pro == 3 else 8 * cin if pro else 0))
# N tiles 96 / 160 and temporal tiles of T * P < 256 rows (T = 2); MILNCE_BOX_EXT=0 leaves them out
_BOX_EXT = os.environ.get("MILNCE_BOX_EXT", "1") != "0"


def _box_ok(bn: int, cin: int, kpad: int, impl: int, geo) -> bool:
    """Mirror of csrc/conv_box.hip fwd_box_supported; geo = (T, H, W, k, padding)."""
    if geo is None or impl not in _BOX_IMPLS:
        return False
    if not ((impl in (14, 16) and bn in (64, 96, 128, 160)) or (impl in (15, 17) and bn in (64, 128, 192))
            or (impl == 16 and bn == 192)):
        return False
    T, H, W, k, pad = geo
    if impl in _BOX4_IMPLS:
        if not _BOX4 or _box4_lds(_box_eff_bn(impl, bn), k) > 80 * 1024:
            return False
        if cin % 8 or kpad < (k[0] * k[1] * k[2] - 1) * cin + _ceil(cin, 64) * 64:
            return False
        if tuple(k) == (1, 3, 3) and tuple(pad) == (0, 1, 1):
            return 127 + (127 // W + 1) + (127 // (H * W) + 1) * (W + 2) + 2 * (W + 1) + 3 <= 288
        if tuple(k) == (3, 1, 1) and tuple(pad) == (1, 0, 0):
            return min(128 // T, 192 // (T + 2)) >= 1
        return False
    if not _BOX_EXT and (bn in (96, 160) or (tuple(k) == (3, 1, 1) and 256 % T)):
        return False
    # a partial last 64-channel block is zero-filled; its weight stage (past the tap's columns) must
    # stay inside the packed row
    if cin % 8 or kpad < (k[0] * k[1] * k[2] - 1) * cin + _ceil(cin, 64) * 64:
        return False
    if tuple(k) == (1, 3, 3) and tuple(pad) == (0, 1, 1):
        span = 255 + (255 // W + 1) + (255 // (H * W) + 1) * (W + 2) + 2 * (W + 1) + 3
        return span <= _BOX_ROWS
    if tuple(k) == (3, 1, 1) and tuple(pad) == (1, 0, 0):
        return min(256 // T, _BOX_ROWS // (T + 2)) >= 1  # P positions per frame and tile
    return False


def _v4_ok(bn: int, cin: int, taps: int, kpad: int, impl: int) -> bool:
    """Mirror of csrc/conv_v4.hip fwd_v4_supported."""
    if cin % 64 or kpad != taps * cin or taps > 32 or bn not in (64, 96, 128, 160, 192):
        return False
    if impl in (9, 11, 13) and (bn // 2) % 32:
        return False
    if impl in (10, 11) and 3 * (128 + bn) * 64 * 2 > 160 * 1024:  # three stages in LDS
        return False
    if impl in _V4_WIDE_M and bn % 64:
        return False
    return True


def _fwd_impls(bn: int, kpad: int, cin: int = 0, taps: int = 0, geo=None) -> Tuple[int, ...]:
    """Forward / dgrad variants the tuner tries for an N tile (csrc/conv.hip launch_v3_impl,
    csrc/conv_v4.hip, csrc/conv_box.hip); ``cin`` = channels of the gathered operand (0: v3
    variants only); ``geo`` = (T, H, W, k, padding) of a stride-1 conv (box-tiled candidates)."""
    base = _WIDE_IMPLS.get(bn, _IMPLS)
    if _V4 and cin:
        base = base + tuple(i for i in _V4_IMPLS if _v4_ok(bn, cin, taps, kpad, i))
    if _BOX and cin:
        base = base + tuple(i for i in _BOX_IMPLS if _box_ok(bn, cin, kpad, i, geo))
    return base


def _box_geo(plan: "ConvPlan"):
    """(T, H, W, k, padding) for the box-tiled kernel, or None (strided / resized output)."""
    if plan.s != (1, 1, 1) or plan.wo_override or (plan.To, plan.Ho, plan.Wo) != (plan.T, plan.H, plan.W):
        return None
    return (plan.T, plan.H, plan.W, plan.k, plan.p)


def _fwd_tiles(M: int, N: int, K: int) -> Tuple[int, int, int, int, int]:
    """N tile from {64, 96, 128, 160, 192}: least padded work, discounted for the lower operand
    reuse of narrow tiles (ties: the wider), e.g. 192 -> one 192 tile instead of two 128 tiles
    (25 % padding), 320 -> two 160s, 448 -> three 160s, 832 -> seven 128s."""
    eff = {192: 1.0, 160: 1.0, 128: 1.0, 96: 0.9, 64: 0.8}
    best = None
    for cand in (192, 160, 128, 96, 64):
        cost = _ceil(N, cand) * cand / eff[cand]
        if best is None or cost < best[1] - 1e-9:
            best = (cand, cost)
    bn = best[0]
    bk = 64 if (K >= 128 or bn in _WIDE_BN) else 32
    npad = _ceil(N, bn) * bn
    kpad = _ceil(K, bk) * bk
    m_tiles = _ceil(M, 128)
    n_tiles = npad // bn
    grid_m = max(1, min(m_tiles, _fill(_FWD_WGS_PER_CU * _NUM_CU, n_tiles)))
    return bn, bk, npad, kpad, grid_m


def conv_plan(x_shape, w_shape, stride, padding, wo_override: int = 0) -> ConvPlan:
    key = (tuple(x_shape), tuple(w_shape), tuple(stride), tuple(padding), wo_override)
    plan = _PLANS.get(key)
    if plan is not None:
        return plan
    B, T, H, W, Cin = x_shape
    Cout, Cin_p, kt, kh, kw = w_shape
    st, sh, sw = stride
    pt, ph, pw = padding
    To = (T + 2 * pt - kt) // st + 1
    Ho = (H + 2 * ph - kh) // sh + 1
    Wo = wo_override if wo_override else (W + 2 * pw - kw) // sw + 1
    M = B * To * Ho * Wo
    taps = kt * kh * kw
    Ktot = taps * Cin
    bn, bk, npad, kpad, grid_m = _fwd_tiles(M, Cout, Ktot)
    # dgrad: a stride-1 conv over dY (channels Cout) producing Cin_p channels
    d_bn, d_bk, d_npad, d_kpad, d_grid_m = _fwd_tiles(B * T * H * W, Cin_p, taps * Cout)
    # wgrad: output [Cout, Ktot], reduction over M
    w_tn = 128 if Cout > 64 else 64
    w_tk = 128 if Ktot > 64 else 64
    if Cin % 8 != 0:  # uint8 stem
        w_tn = 64
    w_npad = _ceil(Cout, w_tn) * w_tn
    w_kpad = _ceil(Ktot, w_tk) * w_tk
    tiles = (w_npad // w_tn) * (w_kpad // w_tk)
    splits = max(1, min(_ceil(4 * _NUM_CU, tiles), _ceil(M, 32 * 8)))
    plan = ConvPlan(B, T, H, W, Cin, Cin_p, Cout, (kt, kh, kw), (st, sh, sw), (pt, ph, pw), To, Ho, Wo, M, Ktot,
                    bn, bk, npad, kpad, grid_m, d_bn, d_bk, d_npad, d_kpad, d_grid_m, w_tn, w_tk, w_npad, w_kpad,
                    splits, wo_override)
    _PLANS[key] = plan
    return plan


class _PackDesc(ctypes.Structure):
    """Mirror of csrc/conv.hip ``PackDesc`` (64 bytes)."""
    _fields_ = [("w", ctypes.c_void_p), ("out", ctypes.c_void_p)] + \
        [(f, ctypes.c_int) for f in ("Cout", "Cin", "Cin_p", "KT", "KH", "KW", "Npad", "Kpad", "mode", "blk0",
                                     "ldo", "pad1")]


def _pack_pieces(ws, plan: ConvPlan, mode: int, out: torch.Tensor):
    """(weight, out address, Cout, Npad, Kpad, ldo) per descriptor packing ``ws`` into ``out``.
    One weight: the whole buffer. A concatenated group (``ws`` stacked along Cout): member i owns
    rows [off, off + c) of the mode-0 buffer, or columns [off, off + c) of the mode-1 buffer
    (row stride d_Kpad); the last member also zero-fills the padding rows / columns."""
    npad, kpad = (plan.Npad, plan.Kpad) if mode == 0 else (plan.d_Npad, plan.d_Kpad)
    if len(ws) == 1:
        return [(ws[0], out.data_ptr(), plan.Cout, npad, kpad, 0)]
    pieces, off = [], 0
    for i, w in enumerate(ws):
        c, last = int(w.shape[0]), i == len(ws) - 1
        if mode == 0:
            pieces.append((w, out.data_ptr() + off * kpad * 2, c, npad - off if last else c, kpad, 0))
        else:
            pieces.append((w, out.data_ptr() + off * 2, c, npad, kpad - off if last else c, kpad))
        off += c
    return pieces


class _WeightPacker:
    """Packs every conv weight of a training step in ONE kernel launch at step start (the weights
    are fixed between the previous optimizer step and this one), instead of one small pack launch
    per conv and direction. Entries register themselves the first time ``_pack`` / ``_pack_group``
    sees parameter weights inside a step (that step packs per call); from the next step on they
    return the pre-packed persistent buffer. The concatenated 1x1 group weights pack straight from
    their member parameters (no per-step torch.cat). Outside a step, or for weights that are not
    parameters, packing stays per call."""

    def __init__(self):
        self.entries: Dict[tuple, list] = {}  # (w ptrs, mode, plan) -> [weights, plan, mode, out]
        self.descs: Optional[torch.Tensor] = None
        self.ndescs = 0
        self.total_blocks = 0
        self.active = False
        self.packed = False

    def begin(self, device: torch.device) -> None:
        self.active = True
        self.packed = False
        if not self.entries:
            return
        if self.descs is None:
            pieces = [(pc, plan, mode) for ws, plan, mode, out in self.entries.values()
                      for pc in _pack_pieces(ws, plan, mode, out)]
            arr = (_PackDesc * len(pieces))()
            blk = 0
            for i, ((w, optr, cout, npad, kpad, ldo), plan, mode) in enumerate(pieces):
                kt, kh, kw = plan.k
                arr[i] = _PackDesc(w.data_ptr(), optr, cout, plan.Cin, plan.Cin_p, kt, kh, kw,
                                   npad, kpad, mode, blk, ldo, 0)
                blk += _ceil(npad * kpad, 256 * 8)
            host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            self.descs = host.to(device)
            self.ndescs = len(pieces)
            self.total_blocks = blk
        call("milnce_pack_weights_multi", ptr(self.descs), self.ndescs, self.total_blocks, stream())
        self.packed = True

    def end(self) -> None:
        self.active = False
        self.packed = False

    @staticmethod
    def _key(ws, plan: ConvPlan, mode: int) -> tuple:
        return (tuple(w.data_ptr() for w in ws), mode, id(plan))

    def lookup(self, ws, plan: ConvPlan, mode: int) -> Optional[torch.Tensor]:
        if not self.active:
            return None
        e = self.entries.get(self._key(ws, plan, mode))
        return e[3] if e is not None and self.packed else None

    def register(self, ws, plan: ConvPlan, mode: int, out: torch.Tensor) -> None:
        # parameters only (leaf, requires grad): their storage is fixed for the whole step; the
        # entry keeps a reference, so the address cannot be recycled for another tensor
        if self.active and all(w.is_leaf and w.requires_grad and w.is_contiguous() for w in ws):
            key = self._key(ws, plan, mode)
            if key not in self.entries:
                self.entries[key] = [tuple(ws), plan, mode, out]
                self.descs = None  # rebuilt at the next step start


_PACKER = _WeightPacker()


def _pack(weight: torch.Tensor, plan: ConvPlan, mode: int) -> torch.Tensor:
    pre = _PACKER.lookup((weight,), plan, mode)
    if pre is not None:
        return pre
    out = _pack_now(weight, plan, mode)
    _PACKER.register((weight,), plan, mode, out)
    return out


_GROUP_PREPACK = os.environ.get("MILNCE_GROUP_PREPACK", "1") != "0"
_GROUP_FIN = os.environ.get("MILNCE_GROUP_FIN", "1") != "0"  # one BN-finalize launch per fused 1x1 group


class _GroupApplyMember(ctypes.Structure):
    """Mirror of csrc/bn.hip ``GroupApplyMember`` (56 bytes)."""
    _fields_ = [("dz", ctypes.c_void_p), ("g", ctypes.c_void_p), ("dmean", ctypes.c_void_p), ("ss", ctypes.c_void_p),
                ("coef", ctypes.c_void_p), ("ldz", ctypes.c_int), ("ldg", ctypes.c_int), ("c0", ctypes.c_int),
                ("c", ctypes.c_int)]


# the group's BN-backward apply passes as one launch over whole rows (csrc/bn.hip
# bn_bwd_apply_group_kernel; MILNCE_GROUP_APPLY=0: one launch per member)
_GROUP_APPLY = os.environ.get("MILNCE_GROUP_APPLY", "1") != "0"


class _BwdFinMember(ctypes.Structure):
    """Mirror of csrc/bn.hip ``BwdFinMember`` (72 bytes)."""
    _fields_ = [(f, ctypes.c_void_p) for f in ("part", "gamma", "ss", "dgamma", "dbeta", "coef")] + \
        [(f, ctypes.c_int) for f in ("nparts", "ps", "C", "blk0", "accumulate", "pad")]


class _FinMember(ctypes.Structure):
    """Mirror of csrc/bn.hip ``FinMember`` (80 bytes)."""
    _fields_ = [(f, ctypes.c_void_p) for f in ("gamma", "beta", "rmean", "rvar", "nbt", "out", "yshift")] + \
        [(f, ctypes.c_int) for f in ("off", "C", "blk0")] + [("momentum", ctypes.c_float), ("eps", ctypes.c_float),
                                                              ("pad", ctypes.c_int)]
_GROUP_WGRAD_DIRECT = os.environ.get("MILNCE_GROUP_WGRAD_DIRECT", "1") != "0"


def _pack_group(ws, plan: ConvPlan, mode: int) -> torch.Tensor:
    """Packed buffer of the weights ``ws`` concatenated along Cout (the fused 1x1 group GEMM)."""
    if not _GROUP_PREPACK:
        return _pack_now(torch.cat([w.detach() for w in ws], 0), plan, mode)
    pre = _PACKER.lookup(ws, plan, mode)
    if pre is not None:
        return pre
    out = _pack_now(torch.cat([w.detach() for w in ws], 0), plan, mode)
    _PACKER.register(ws, plan, mode, out)
    return out


def _pack_now(weight: torch.Tensor, plan: ConvPlan, mode: int) -> torch.Tensor:
    kt, kh, kw = plan.k
    if mode == 0:
        out = torch.empty((plan.Npad, plan.Kpad), dtype=BF16, device=weight.device)
        call("milnce_pack_weight", ptr(weight), ptr(out), plan.Cout, plan.Cin, plan.Cin_p, kt, kh, kw,
             plan.Npad, plan.Kpad, 0, stream())
    else:
        out = torch.empty((plan.d_Npad, plan.d_Kpad), dtype=BF16, device=weight.device)
        call("milnce_pack_weight", ptr(weight), ptr(out), plan.Cout, plan.Cin, plan.Cin_p, kt, kh, kw,
             plan.d_Npad, plan.d_Kpad, 1, stream())
    return out


_IMPLS = (2, 3, 4, 5, 6, 7)
_W_IMPLS = (2, 3, 4, 5)  # wgrad: register-staged, LDS-DMA 3/2 stages, register-staged 2-deep
_AUTOTUNE = os.environ.get("MILNCE_CONV_AUTOTUNE", "1") != "0"
_DEFAULT_IMPL = int(os.environ.get("MILNCE_CONV_IMPL", "2"))
_TUNE_MARGIN = float(os.environ.get("MILNCE_TUNE_MARGIN", "0.97"))  # another variant must beat the default by 3 %


# Tune with cold caches (MILNCE_TUNE_FLUSH=0: back-to-back warm launches, the round-2 method): a
# variant timed on L2 / Infinity-Cache-resident repeats of its own inputs can lose inside the step
# (e.g. the 256-row dgrad with the producer-BN epilogue: 1.33 ms warm, 1.95 ms in the step).
_TUNE_FLUSH = os.environ.get("MILNCE_TUNE_FLUSH", "1") != "0"
_TUNE_ROUNDS = max(1, int(os.environ.get("MILNCE_TUNE_ROUNDS", "3")))
_FLUSH_BUF: Dict[int, torch.Tensor] = {}


def _tune_flush_buffer() -> torch.Tensor:
    dev = torch.cuda.current_device()
    buf = _FLUSH_BUF.get(dev)
    if buf is None:
        buf = _FLUSH_BUF[dev] = torch.empty((384 << 20) // 4, dtype=F32, device="cuda")  # > 256 MiB MALL + L2
    return buf


def release_tuning_buffers() -> None:
    """Free the cold-cache flush buffer (384 MiB per device) once the step's shapes are tuned."""
    _FLUSH_BUF.clear()


def _tune(launch, impls=_IMPLS, default: Optional[int] = None, sig: str = "") -> int:
    """Time each kernel variant on the real operands (outputs are simply overwritten) and keep
    the fastest; run once per conv shape and direction, then cached in the plan. Each variant
    is timed over >= ~0.5 ms of repetitions (at least one per round), and the default wins unless
    another is >= 3 % faster, so the choice is stable from run to run. Under data parallelism
    (tune_sync.region) only rank 0 times; every rank launches rank 0's choice."""
    if not _AUTOTUNE:
        return _DEFAULT_IMPL
    return tune_sync.decide(sig or f"impls{tuple(impls)}", lambda: _tune_local(launch, impls, default))


def _tune_local(launch, impls, default: Optional[int]) -> int:
    s = torch.cuda.current_stream()
    flush = _tune_flush_buffer() if _TUNE_FLUSH else None

    def timed(impl, reps):
        if flush is None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(reps):
                launch(impl)
            b.record(s)
            b.synchronize()
            return a.elapsed_time(b) / reps
        # cold caches, as inside the step (a layer's inputs were written a whole layer ago):
        # overwrite more than the Infinity Cache + L2 before each timed launch
        total = 0.0
        for _ in range(reps):
            flush.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            launch(impl)
            b.record(s)
            b.synchronize()
            total += a.elapsed_time(b)
        return total / reps

    # variants interleaved over _TUNE_ROUNDS rounds, median per variant: a clock or cache drift
    # during the tuning of one shape cannot favour whichever variant happened to run first
    reps = {}
    for impl in impls:
        try:
            launch(impl)  # warm (first launch sets kernel attributes)
        except UnsupportedVariant:  # a variant whose own checks (e.g. its LDS budget) decline the shape
            continue
        t0 = timed(impl, 1)
        reps[impl] = max(1, min(50 if flush is None else 18, int(0.5 / max(t0, 1e-3))) // _TUNE_ROUNDS)
    if not reps:
        raise UnsupportedVariant(f"no kernel variant of {tuple(impls)} supports this shape")
    impls = tuple(reps)
    samples = {impl: [] for impl in impls}
    for _ in range(_TUNE_ROUNDS):
        for impl in impls:
            samples[impl].append(timed(impl, reps[impl]))
    times = {impl: sorted(v)[len(v) // 2] for impl, v in samples.items()}
    best = min(times, key=times.get)
    default = _DEFAULT_IMPL if default is None else default
    if default in times and times[best] > _TUNE_MARGIN * times[default]:
        best = default
    return best


def conv_forward_raw(x: torch.Tensor, wp: torch.Tensor, plan: ConvPlan, stats: Optional[torch.Tensor],
                     pro=None, shift: Optional[torch.Tensor] = None):
    """Raw conv output y (bf16) with the BN-statistics epilogue when ``stats`` is given.

    ``shift`` (fp32 [Cout], with ``stats`` only): subtracted per channel before the bf16 rounding
    (``_bn_shift``); the statistics are those of the shifted values.

    ``pro = (z_out or None)``: x is a "pro" placeholder (``_pro_z``) standing for
    relu(y_prod * scale + shift) of its producer BN. A box-tiled variant applies that while
    staging its input and writes z to ``z_out`` (the wgrad operand); any other variant gets
    z materialised into ``z_out`` (or a scratch buffer) first."""
    y = torch.empty((plan.B, plan.To, plan.Ho, plan.Wo, plan.Cout), dtype=BF16, device=x.device)
    if stats is None:
        shift = None
    if pro is not None:
        z_out = pro[0]
        yp, ssp, ldp = x._milnce_bn
        fusable = x.shape[-1] == plan.Cin and ldp % 8 == 0  # y may be a channel slice (row stride ldp)
        zbuf = z_out if z_out is not None else torch.empty(x.shape, dtype=BF16, device=x.device)
        thw_in = plan.T * plan.H * plan.W

        def pro_ok(impl):
            # a 4-wave variant also needs its 80 KiB with the prologue's [Cin] constants: a plan first
            # tuned without the prologue (a plain-input call of the same shape) can hold one that
            # does not fit, which then runs on the materialised z instead
            if impl not in _BOX_IMPLS or not fusable:
                return False
            return impl not in _BOX4_IMPLS or _box4_lds(_box_eff_bn(impl, plan.bn), plan.k, pro=1,
                                                         epi=1 if stats is not None else 0,
                                                         cin=plan.Cin) <= 80 * 1024

        def launch_pro(impl, grid):
            if pro_ok(impl):
                call("milnce_conv_fwd_pro", ptr(yp), ldp, ptr(wp), ptr(y), ptr(stats), ptr(shift), ptr(ssp),
                     ptr(z_out),
                     plan.B, plan.T, plan.H, plan.W, plan.Cin, plan.Cout, *plan.k, *plan.p, plan.Kpad, plan.Npad,
                     plan.Cout, plan.bn, grid, impl, stream())
            else:  # the variant needs z in memory: its timing includes the BN-apply pass
                call("milnce_bn_relu_apply", ptr(yp), ldp, ptr(zbuf), plan.Cin, ptr(ssp), plan.Cin, plan.B, thw_in,
                     None, stream())
                call("milnce_conv_fwd", ptr(zbuf), 0, ptr(wp), ptr(y), ptr(stats), None, ptr(shift), 0,
                     plan.B, plan.T, plan.H, plan.W, plan.Cin, plan.Cout, *plan.k, *plan.s, *plan.p,
                     plan.Kpad, plan.Npad, plan.Cout, plan.bn, plan.bk, grid, plan.wo_override, impl, stream())

        ck = _ctx_key("fwdpro", "st" if stats is not None else "", "fz" if fusable else "nf")
        rows_p = stats.numel() // (2 * plan.Npad) if stats is not None else None
        # tuned on what each variant costs here (fused prologue vs apply pass + conv)
        plan.impl, plan.grid_m = _decision(plan, ck, False, lambda: _tune_fwd(
            launch_pro, _fwd_impls(plan.bn, plan.Kpad, plan.Cin, plan.taps, _box_geo(plan)), plan.M, plan.Npad,
            plan.bn, rows_p, sig=ck + _plan_sig(plan)))
        if pro_ok(plan.impl):
            launch_pro(plan.impl, plan.grid_m)
            return y
        # the tuned choice for this context is the apply pass + a plain variant (timed as such)
        x = _materialize(x, z_out)
        _materialized = True
    else:
        _materialized = False
    kt, kh, kw = plan.k
    st, sh, sw = plan.s
    pt, ph, pw = plan.p

    def launch(impl, grid):
        call("milnce_conv_fwd", ptr(x), int(x.dtype == torch.uint8), ptr(wp), ptr(y), ptr(stats), None,
             ptr(shift), 0, plan.B, plan.T, plan.H, plan.W, plan.Cin, plan.Cout, kt, kh, kw, st, sh, sw, pt, ph, pw,
             plan.Kpad, plan.Npad, plan.Cout, plan.bn, plan.bk, grid, plan.wo_override, impl, stream())

    rows = stats.numel() // (2 * plan.Npad) if stats is not None else None
    if not _materialized:
        ck = _ctx_key("fwd", "st" if stats is not None else "")
        if x.dtype == torch.uint8:
            plan.impl = plan.pin_f or 2
        else:
            plan.impl, plan.grid_m = _decision(plan, ck, False, lambda: _tune_fwd(
                launch, _fwd_impls(plan.bn, plan.Kpad, plan.Cin, plan.taps, _box_geo(plan)), plan.M, plan.Npad,
                plan.bn, rows, sig=ck + _plan_sig(plan)))
    if rows is not None and rows < plan.grid_m:
        raise ValueError(f"stats holds {rows} partial rows, the tuned grid writes {plan.grid_m} "
                         f"(allocate _stats_rows(M, Npad, bn) rows)")
    _launch_tuned(launch, plan.impl, plan.grid_m, plan.bn)
    return y


def conv_dgrad(dy: torch.Tensor, wd: torch.Tensor, plan: ConvPlan, producer_bn=None) -> torch.Tensor:
    """dX of a stride-1 conv. With ``producer_bn = (y, ss, ld)`` of the BN layer that produced X,
    the epilogue also emits that layer's BN-backward partial sums (attached to dX, consumed by
    its backward instead of a separate reduction pass over dX and y)."""
    kt, kh, kw = plan.k
    assert plan.s == (1, 1, 1), "dgrad is only needed for stride-1 convs"
    dx = torch.empty((plan.B, plan.T, plan.H, plan.W, plan.Cin_p), dtype=BF16, device=dy.device)
    pt, ph, pw = kt - 1 - plan.p[0], kh - 1 - plan.p[1], kw - 1 - plan.p[2]
    part = None
    md = plan.B * plan.T * plan.H * plan.W
    if producer_bn is not None:
        part = torch.empty((_stats_rows(md, plan.d_Npad, plan.d_bn) * 2 * plan.d_Npad,), dtype=F32, device=dy.device)

    def launch(impl, grid):
        call("milnce_conv_fwd", ptr(dy), 0, ptr(wd), ptr(dx), ptr(part),
             ptr(producer_bn[0]) if part is not None else None, ptr(producer_bn[1]) if part is not None else None,
             producer_bn[2] if part is not None else 0,
             plan.B, plan.To, plan.Ho, plan.Wo, plan.Cout, plan.Cin_p, kt, kh, kw, 1, 1, 1, pt, ph, pw,
             plan.d_Kpad, plan.d_Npad, plan.Cin_p, plan.d_bn, plan.d_bk, grid, 0, impl, stream())

    ck = _ctx_key("dgrad", "p" if part is not None else "")
    plan.d_impl, plan.d_grid_m = _decision(plan, ck, True, lambda: _tune_fwd(
        launch, _fwd_impls(plan.d_bn, plan.d_Kpad, plan.Cout, plan.taps, _box_geo(plan)), md, plan.d_Npad,
        plan.d_bn, sig=ck + _plan_sig(plan)))
    _launch_tuned(launch, plan.d_impl, plan.d_grid_m, plan.d_bn)
    if part is not None:
        attach_bn_partials(dx, part, plan.d_grid_m, plan.d_Npad)
    return dx


def conv_dgrad_bnbwd(dz: torch.Tensor, wd: torch.Tensor, plan: ConvPlan, producer_bn, y: torch.Tensor,
                     ss: torch.Tensor, coef: torch.Tensor, dy_out: torch.Tensor, impl: int = 0,
                     grid: int = 0, dx: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dX of a conv whose output went through BN -> ReLU, from dz (the gradient of the ReLU output):
    the box-tiled dgrad stages that BN's backward dy = k0 * (dz * mask - k1 - xhat * k2) itself
    (y / ss: the BN's raw conv output and constants, coef: milnce_bn_bwd_finalize output) and writes
    dy to ``dy_out`` for the wgrad, so the separate bn_bwd_apply pass (read dz and y, write dy) and
    the dgrad's read of dy become its reads of dz and y. Requires a box-tiled variant: ``impl`` /
    ``grid``, else the plan's tuned decision for this call context."""
    kt, kh, kw = plan.k
    if dx is None:
        dx = torch.empty((plan.B, plan.T, plan.H, plan.W, plan.Cin_p), dtype=BF16, device=dz.device)
    pt, ph, pw = kt - 1 - plan.p[0], kh - 1 - plan.p[1], kw - 1 - plan.p[2]
    if not impl:
        impl, grid = _decision(plan, _ctx_key("dgradbn", "p" if producer_bn is not None else ""), True, None)
    part = None
    if producer_bn is not None:
        md = plan.B * plan.T * plan.H * plan.W
        part = torch.empty((_stats_rows(md, plan.d_Npad, plan.d_bn) * 2 * plan.d_Npad,), dtype=F32, device=dz.device)
    call("milnce_conv_dgrad_bnbwd", ptr(dz), ptr(wd), ptr(dx), ptr(part),
         ptr(producer_bn[0]) if part is not None else None, ptr(producer_bn[1]) if part is not None else None,
         producer_bn[2] if part is not None else 0, ptr(y), ptr(ss), ptr(coef), ptr(dy_out),
         plan.B, plan.To, plan.Ho, plan.Wo, plan.Cout, plan.Cin_p, kt, kh, kw, pt, ph, pw, plan.d_Kpad, plan.d_Npad,
         plan.d_bn, grid, impl, stream())
    if part is not None:
        attach_bn_partials(dx, part, grid, plan.d_Npad)
    return dx


def _tune_dgrad_bnbwd(plan: ConvPlan, dz, weight, y, ss, gamma, part, nparts, ps, x_bn, training) -> None:
    """Tune a dgrad whose BN-backward apply the box kernel can take over on what each variant
    costs here: the fused dgrad (PRO 3) for box-tiled variants, bn_bwd apply pass + dgrad for the
    others. All runs write scratch buffers (the BN gradients are accumulated in place)."""
    C, dev = plan.Cout, dz.device
    wd = _pack(weight, plan, 1)
    coef = torch.empty((3 * C,), dtype=F32, device=dev)
    dg, db = torch.empty((C,), dtype=F32, device=dev), torch.empty((C,), dtype=F32, device=dev)
    call("milnce_bn_bwd_finalize", ptr(part), nparts, ps, C, float(plan.M), ptr(gamma), ptr(ss), ptr(dg), ptr(db),
         ptr(coef), 0, int(training), stream())
    dy_s = torch.empty_like(y)
    dx_s = torch.empty((plan.B, plan.T, plan.H, plan.W, plan.Cin_p), dtype=BF16, device=dev)
    md = plan.B * plan.T * plan.H * plan.W
    part_s = (torch.empty((_stats_rows(md, plan.d_Npad, plan.d_bn) * 2 * plan.d_Npad,), dtype=F32, device=dev)
              if x_bn is not None else None)
    kt, kh, kw = plan.k
    pt, ph, pw = kt - 1 - plan.p[0], kh - 1 - plan.p[1], kw - 1 - plan.p[2]

    def launch(impl, grid):
        if _box_pro3_ok(impl, plan):
            conv_dgrad_bnbwd(dz, wd, plan, x_bn, y, ss, coef, dy_s, impl, grid, dx_s)
            return
        call("milnce_bn_bwd", ptr(dz), C, ptr(y), C, ptr(ss), C, plan.M, ptr(gamma), ptr(part), nparts, ps, 1,
             ptr(dg), ptr(db), ptr(coef), ptr(dy_s), C, 0, int(training), stream())
        call("milnce_conv_fwd", ptr(dy_s), 0, ptr(wd), ptr(dx_s), ptr(part_s),
             ptr(x_bn[0]) if part_s is not None else None, ptr(x_bn[1]) if part_s is not None else None,
             x_bn[2] if part_s is not None else 0,
             plan.B, plan.To, plan.Ho, plan.Wo, plan.Cout, plan.Cin_p, kt, kh, kw, 1, 1, 1, pt, ph, pw,
             plan.d_Kpad, plan.d_Npad, plan.Cin_p, plan.d_bn, plan.d_bk, grid, 0, impl, stream())

    ck = _ctx_key("dgradbn", "p" if x_bn is not None else "")
    plan.ctx[ck] = _tune_fwd(launch, _fwd_impls(plan.d_bn, plan.d_Kpad, plan.Cout, plan.taps, _box_geo(plan)),
                             md, plan.d_Npad, plan.d_bn, sig=ck + _plan_sig(plan))
    _PLAN_EVENTS["contexts"] += 1
    if not _box_pro3_ok(plan.ctx[ck][0], plan):
        # the winner is the apply pass + a plain dgrad: that is what the plain dgrad call will run
        plan.ctx.setdefault(_ctx_key("dgrad", "p" if x_bn is not None else ""), plan.ctx[ck])


# MILNCE_BNBWD_FUSE=0 disables. First version measured slower in the step (conv_2c spatial dgrad
# 1.42 -> 2.74 ms against ~1.1 ms of bn_bwd_apply removed: seven per-channel constants re-read from
# LDS per staged element, applied serially after the block's MFMAs); with the constants in
# registers and the transform after tap 3's MFMAs: 2.35 ms, same-box bench 4285 -> 4303 pairs/s
# (profiles/r3_box_conv.md).
_BNBWD_FUSE = os.environ.get("MILNCE_BNBWD_FUSE", "1") != "0"


def _box_pro3_ok(impl: int, plan: ConvPlan) -> bool:
    """Box variant ``impl`` can run this plan's dgrad with the BN-backward prologue (PRO 3: N tiles
    <= 128; a 4-wave one also within 80 KiB with the prologue constants and producer partials)."""
    if impl not in _BOX_IMPLS or _box_eff_bn(impl, plan.d_bn) > 128:
        return False
    if impl in _BOX4_IMPLS:
        return _box4_lds(_box_eff_bn(impl, plan.d_bn), plan.k, pro=3, epi=2, cin=plan.Cout) <= 80 * 1024
    return True


def _bnbwd_fusable(plan: ConvPlan, dz: torch.Tensor, ck: str) -> bool:
    """The dgrad tuned for context ``ck`` takes over this layer's BN-backward apply
    (``conv_dgrad_bnbwd``)."""
    impl = plan.pin_d or plan.ctx.get(ck, (0, 0))[0]
    return (_BNBWD_FUSE and _PRO_FUSE and _box_pro3_ok(impl, plan) and _box_geo(plan) is not None
            and dz.dtype == BF16 and dz.shape[-1] == plan.Cout and plan.Cout % 8 == 0)


_FUSE_BN_BWD = True

# BN-ReLU outputs that only feed a SelfGating are not materialised: the producer computes just
# the gating sums, returns a stride-0 placeholder tagged with (y, ss, ld), and the gate applies
# relu(y * scale + shift) while scaling (csrc/gate.hip lazy segments).
_LAZY_GATE_Z = os.environ.get("MILNCE_LAZY_GATE_Z", "1") != "0"
# want_gsum == GSUM_DEFER (the Inception branches): a lazy branch's SelfGating sums are not computed
# by its own gsum-only pass but by ONE pass over all four branches of the block inside gate_concat
# (csrc/gate.hip gate_gsum_kernel). MILNCE_BATCH_GSUM=0 keeps the per-branch passes.
GSUM_DEFER = 2
_BATCH_GSUM = os.environ.get("MILNCE_BATCH_GSUM", "1") != "0"


def _defer_gsum(want) -> bool:
    return _BATCH_GSUM and int(want) == GSUM_DEFER
# Gradients that only feed their producer's BN backward are not stored either ("lazy dz"):
#  * SelfGating inputs: the gate backward computes only the BN partial sums and the BN backward
#    rebuilds dz = bf16(dout * g + dmean / thw) from dout (milnce_bn_bwd_gate);
#  * pool inputs (stem -> maxpool_2a, gate -> maxpool_3a): the pool backward computes only the BN
#    partial sums and a second gather pass applies the BN backward (milnce_maxpool_bwd_apply).
#    On by default since the stride-2 pool backward gathers per input quad (pool_bwd_quad): the
#    second gather is now cheaper than the dz round trip it saves (A/B on MI355X: 73.2 vs 73.9
#    ms/step; with the per-position gather it was 78.6 vs 78.3).
_LAZY_GATE_DZ = os.environ.get("MILNCE_LAZY_GATE_DZ", "1") != "0"
_LAZY_POOL_DZ = os.environ.get("MILNCE_LAZY_POOL_DZ", "1") != "0"
# The stem's BN-backward partial sums from the pooled side: maxpool_2a's forward also stores the raw
# stem output at each arg-max (yr, pooled shape) and tags its output with (yr, ss), so conv_2b's
# dgrad epilogue (producer-BN partials, EPI 2) reduces sum_o dout_o mask(yr_o) (1, xhat(yr_o)) --
# the same sums over the full-resolution dz -- and the partials-only gather pass over the stem
# output (dout, arg-max and the 2.6 GB stem output read) disappears. MILNCE_POOL_YR=0 disables.
_POOL_YR = os.environ.get("MILNCE_POOL_YR", "1") != "0"
# The same for the gated maxpool_3a (conv_2c -> SelfGating -> pool, _GatedPool): its input BN's
# dz = dx * g + dmean / thw is nonzero at every cell, so its partial sums are the pooled-side sums
# over (dout * g, yr) plus dmean / thw times the per-clip mask statistics (sum mask, sum mask *
# xhat), which the forward's gating-sum pass takes from the same read of y
# (milnce_bn_relu_gsum_mstat) -- one pass over the pooled tensors replaces the full-resolution
# partials gather (dout, codes, 2 GB of y). MILNCE_GATED_POOL_STATS=0 disables.
_GATED_POOL_STATS = os.environ.get("MILNCE_GATED_POOL_STATS", "1") != "0"


def _lazy_z(shape, device, bn_info) -> torch.Tensor:
    z = torch.empty((1,), dtype=BF16, device=device).expand(*shape)
    z._milnce_bn = bn_info
    z._milnce_lazy = True
    return z


def _is_lazy(t) -> bool:
    return bool(getattr(t, "_milnce_lazy", False))


# BN-ReLU outputs whose only consumer is another conv ("pro" placeholders, ``lazy_out``): the
# producer skips its bn_relu_apply pass and returns a stride-0 placeholder tagged with (y, ss, ld);
# the consumer's box-tiled kernel (csrc/conv_box.hip PRO) applies relu(y * scale + shift) while
# staging its input box and writes z once as a by-product (its wgrad operand): the separate pass
# (read y, write z) and the consumer's re-read of z become one read of y inside the conv. Other
# consumer kernels materialise z first (the old cost). MILNCE_PRO_FUSE=0 disables.
_PRO_FUSE = os.environ.get("MILNCE_PRO_FUSE", "1") != "0"
_BOX_IMPLS = (14, 15, 16, 17)


def _pro_z(shape, device, bn_info) -> torch.Tensor:
    z = torch.empty((1,), dtype=BF16, device=device).expand(*shape)
    z._milnce_bn = bn_info
    z._milnce_pro = True
    return z


def _is_pro(t) -> bool:
    return bool(getattr(t, "_milnce_pro", False))


def _materialize(z: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The bf16 relu(y * scale + shift) a lazy placeholder stands for (into ``out`` if given)."""
    y, ss, ld = z._milnce_bn
    if out is None:
        out = torch.empty(z.shape, dtype=BF16, device=z.device)
    B = z.shape[0]
    thw = out.numel() // (B * z.shape[-1])
    call("milnce_bn_relu_apply", ptr(y), ld, ptr(out), z.shape[-1], ptr(ss), z.shape[-1], B, thw, None, stream())
    return out


def _lazy_dz(shape, device, info) -> torch.Tensor:
    """Placeholder for a gradient that is not stored (see ``_LAZY_GATE_DZ``); info =
    ("gate", dout, channel offset, g, dmean, thw) or ("pool", dout, arg, geo, g, dmean, nparts)."""
    dz = torch.empty((1,), dtype=BF16, device=device).expand(*shape)
    dz._milnce_lazydz = info
    return dz


def _lazy_dz_info(dz):
    return getattr(dz, "_milnce_lazydz", None) if dz is not None else None


def _bn_bwd_lazy(info, B, M, y, ldy, ss, C, gamma, part, nparts, ps, dgamma, dbeta, coef, dy, lddy, accumulate,
                 training):
    """BN backward whose dz is a lazy gradient (see ``_lazy_dz``)."""
    if info[0] == "gate":
        _, dout, off, g, dmean, thw = info
        ld = dout.shape[-1]
        call("milnce_bn_bwd_gate", ptr(dout) + 2 * off, ld, ptr(g) + 4 * off, ptr(dmean) + 4 * off, ld, B, thw,
             ptr(y), ldy, ptr(ss), C, ptr(gamma), ptr(part), nparts, ps, ptr(dgamma), ptr(dbeta), ptr(coef),
             ptr(dy), lddy, int(accumulate), int(training), stream())
        return
    _, dout, arg, geo, g, dmean, pool_parts = info
    if lddy != C:
        raise RuntimeError("lazy pool gradient needs a dense output gradient")
    call("milnce_bn_bwd_finalize", ptr(part), nparts, ps, C, float(M), ptr(gamma), ptr(ss), ptr(dgamma), ptr(dbeta),
         ptr(coef), int(accumulate), int(training), stream())
    call("milnce_maxpool_bwd_apply", ptr(dout), ptr(arg), ptr(dy), *geo, ptr(y), ldy, ptr(ss), ptr(coef), ptr(g),
         ptr(dmean), pool_parts, stream())


def set_bn_bwd_fusion(enabled: bool) -> bool:
    """Toggle producer-side BN-backward partial sums (for A/B tests); returns the old value."""
    global _FUSE_BN_BWD
    old, _FUSE_BN_BWD = _FUSE_BN_BWD, bool(enabled)
    return old


def attach_bn_partials(dz: torch.Tensor, part: torch.Tensor, nparts: int, stride: int) -> None:
    """Mark dz with the BN-backward partial sums its producer computed. The version stamp makes
    the producer ignore them if autograd accumulated other gradients into dz in place."""
    dz._milnce_bnpart = (part, nparts, stride)
    dz._milnce_bnver = dz._version


def take_bn_partials(dz: torch.Tensor):
    if not _FUSE_BN_BWD:
        return None
    part = getattr(dz, "_milnce_bnpart", None)
    if part is None or getattr(dz, "_milnce_bnver", -1) != dz._version:
        return None
    return part


# -----------------------------------------------------------------------------------------
# Branch streams (MILNCE_BRANCH_STREAMS=1): an Inception block's branches 2 and 3 run on a second
# compute stream next to branch 1 (models/s3dg.py InceptionBlock), and autograd runs their backward
# on that stream too (PyTorch runs each backward op on its forward op's stream and syncs the
# gradients between streams). The small 13x13 / 7x7 layers' kernels do not fill the chip alone.
# Memory: a tensor allocated on one stream and used on another is recorded on the user stream
# (the caching allocator then defers its reuse): branch inputs / outputs at the fork and join,
# incoming gradients, lazy-gradient operands and BN partials at backward entry (``adopt``).
# grad_sink joins the branch stream wherever it joins the side stream (in-place gradient writes).
_BRANCH = os.environ.get("MILNCE_BRANCH_STREAMS", "0") == "1"
_BRANCH_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


def branch_streams_enabled(x: torch.Tensor) -> bool:
    return _BRANCH and x.is_cuda and not torch.cuda.is_current_stream_capturing()


def branch_stream(device: torch.device) -> "torch.cuda.Stream":
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _BRANCH_STREAMS.get(idx)
    if st is None:
        st = _BRANCH_STREAMS[idx] = torch.cuda.Stream(device=idx)
        grad_sink.add_stream(st)
    return st


def _backing(t):
    """The device tensors a (possibly placeholder) activation / gradient stands for."""
    out = []
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        return out
    out.append(t)
    for attr in ("_milnce_bn",):
        info = getattr(t, attr, None)
        if info is not None:
            out += [v for v in info if isinstance(v, torch.Tensor)]
    lz = getattr(t, "_milnce_lazydz", None)
    if lz is not None:
        out += [v for v in lz if isinstance(v, torch.Tensor)]
    part = getattr(t, "_milnce_bnpart", None)
    if part is not None:
        out.append(part[0])
    gs = getattr(t, "_milnce_gs", None)
    if isinstance(gs, torch.Tensor):
        out.append(gs)
    return out


def record_on(tensors, stream) -> None:
    """Record every backing tensor of ``tensors`` as used on ``stream``."""
    for t in tensors:
        for b in _backing(t):
            b.record_stream(stream)


def adopt(*tensors) -> None:
    """Backward entry under branch streams: the incoming tensors (possibly allocated on another
    stream) are used on the current one."""
    if _BRANCH_STREAMS:
        record_on(tensors, torch.cuda.current_stream())


# -----------------------------------------------------------------------------------------
# Direct gradient writes. Parameters whose .grad is a view into the data-parallel flat buffer
# (parallel/ddp.py marks them ``_milnce_flat_grad``) get their weight / BN gradients written
# (accumulated) in place by the producing kernel instead of being returned to autograd, which
# would launch one AccumulateGrad add per parameter; the bucketer is then told the gradient
# is ready through the sink it registered.
def _direct_grad(param: torch.Tensor) -> Optional[torch.Tensor]:
    if not param.is_leaf or not getattr(param, "_milnce_flat_grad", False):
        return None
    g = param.grad
    if g is not None and getattr(param, "_milnce_flat_grad", False) and g.dtype == F32 and g.is_contiguous():
        return g
    return None


def _grad_done(param: torch.Tensor) -> None:
    grad_sink.notify(param)


_STEM_WGRAD = os.environ.get("MILNCE_STEM_WGRAD", "1") != "0"
_STEM_UNSUPPORTED = -1  # csrc/conv.hip STEM_UNSUPPORTED: geometry not covered, use the generic conv
_STEM_FWD = os.environ.get("MILNCE_STEM_FWD", "1") != "0"


def _is_paired_stem(plan: ConvPlan) -> bool:
    """The paired-width stem conv (csrc/conv.hip stem_wgrad_kernel geometry)."""
    return (plan.Cin == 8 and plan.Cin_p == 8 and plan.Cout == 64 and plan.k == (3, 7, 4) and
            plan.s == (2, 2, 1) and plan.p == (1, 3, 2) and plan.Wo == plan.W)


def _wgrad_geom(Cout: int, Ktot: int, M: int, tn: int, tk: int, occ: int = 4) -> Tuple[int, int, int]:
    """(Npad, Kpad, splits) of a wgrad tiling: split-K over m until >= occ blocks per CU. More
    splits fill the chip better but every split writes (and the reduce reads) a full fp32 slab."""
    npad = _ceil(Cout, tn) * tn
    kpad = _ceil(Ktot, tk) * tk
    tiles = (npad // tn) * (kpad // tk)
    splits = max(1, min(_fill(occ * _GRID_CU[0], tiles), _ceil(M, 32 * 8)))
    return npad, kpad, splits


def _wgrad_tiles(Cout: int) -> List[int]:
    """N-tile candidates: 128 (64 for narrow layers) plus the wide register-staged tiles 96 / 192
    where they pad Cout less (192 -> one 192 or two 96 tiles instead of two 128s)."""
    if Cout <= 64:
        return [64]
    base = _ceil(Cout, 128) * 128
    return [128] + [t for t in (96, 192) if _ceil(Cout, t) * t < base]


_WIDE_W_IMPLS = {96: (2, 5), 192: (2,)}  # csrc/conv.hip launch_wgrad_impl: register-staged only


def _wide_w_impls(tn: int, tk: int) -> Tuple[int, ...]:
    if tk == 192:  # register-staged only; 2-deep fits at tn 64 (csrc/conv.hip launch_wgrad_impl)
        return (2, 5) if tn == 64 else (2,)
    if tn == 192 and tk == 64:  # the 2-deep register-staged 192 x 64 tile fits (192 x 128 would spill)
        return (2, 5)
    return _WIDE_W_IMPLS.get(tn, _W_IMPLS)


# K-tile candidates: 64 besides the default 128 where 128 pads the reduction width (e.g. a
# (3,1,1) conv over 192 channels: Ktot 576 -> 640 with 128-wide tiles; same-box bench 4010 ->
# 4050 pairs/s); MILNCE_W_TK64=0 disables, =2 offers 64 for every layer
_W_TK64 = int(os.environ.get("MILNCE_W_TK64", "1"))


def _wgrad_tks(plan: "ConvPlan") -> Tuple[int, ...]:
    tks = [plan.w_tk]
    if _W_TK64 and plan.w_tk == 128 and (plan.Ktot % 128 != 0 or _W_TK64 == 2):
        tks.append(64)
    if _W_TK192 and plan.Ktot % 192 == 0 and plan.Cin % 8 == 0:
        tks.append(192)
    return tuple(tks)


# 192-wide K tiles where they divide the reduction width (Ktot 576 = 3 x 192: a (3,1,1) or
# (1,3,3) conv over 192 / 64 channels): each dY tile is re-read Ktot / 192 times instead of
# Ktot / 64; N tiles 64 / 96 / 128 (csrc/conv.hip). MILNCE_W_TK192=0 disables
_W_TK192 = os.environ.get("MILNCE_W_TK192", "1") != "0"


def _wgrad_tiles_for(Cout: int, tk: int) -> List[int]:
    if tk == 192:
        return [t for t in (64, 96, 128) if t <= max(64, _ceil(Cout, 32) * 32)]
    return _wgrad_tiles(Cout)
# split-K occupancy candidates (workgroups per CU; more splits hide the wgrad kernels' latency at the
# price of bigger slabs: same-box bench 66.45 ms with (4, 2), 66.05 with (4, 2, 8), 65.72 with
# (4, 2, 8, 16)); MILNCE_W_OCCS overrides (A/B runs)
_W_OCCS = tuple(int(v) for v in os.environ.get("MILNCE_W_OCCS", "4,2,8,16").split(","))
_HALO_WGRAD = os.environ.get("MILNCE_HALO_WGRAD", "1") != "0"
_HALO_KERNELS = ((1, 3, 3), (3, 1, 1))
# The (3,1,1) kernel measured slower than the im2col kernel (3 taps amortise the per-box cost less:
# tools/halo_bench.py); offered to the tuner (channel chunks of 64 and 128) with MILNCE_HALO_T311=1,
# it was never picked in the step (same-box A/B round 3: 4271 / 4278 vs 4277 / 4277 pairs/s)
_HALO_TUNED = ((1, 3, 3), (3, 1, 1)) if os.environ.get("MILNCE_HALO_T311", "0") == "1" else ((1, 3, 3),)


def _halo_wgrad_supported(plan: ConvPlan, x: torch.Tensor) -> bool:
    """Box-tiled wgrad (csrc/conv_halo.hip) covers stride-1 same-padded (1,3,3) / (3,1,1) convs
    over bf16 activations."""
    return (x.dtype == BF16 and plan.k in _HALO_KERNELS and plan.s == (1, 1, 1)
            and plan.p == tuple(k // 2 for k in plan.k) and not plan.wo_override and plan.Cin % 8 == 0
            and plan.Cin == plan.Cin_p)


def _halo_wgrad_ok(plan: ConvPlan, x: torch.Tensor) -> bool:
    return _HALO_WGRAD and plan.k in _HALO_TUNED and _halo_wgrad_supported(plan, x)


_HALO_SPLITS: Dict[Tuple[int, int, int], Tuple[int, int]] = {}


# halo wgrad split targets to tune over, in workgroups per CU (same-box bench: 64.4 ms with 2 only,
# 63.7 with 1, 2, 4, 8); MILNCE_HALO_OCCS overrides
_HALO_OCCS = tuple(int(v) for v in os.environ.get("MILNCE_HALO_OCCS", "1,2,4,8").split(","))


def _halo_wgrad(dy, x, plan: ConvPlan, cc: int, target: Optional[torch.Tensor], accumulate: int,
                occ: int = 2):
    """Box-tiled wgrad; with ``target`` None the kernel only fills the split slab and the
    (slab, splits, Npad, Kpad) of the pending reduction is returned."""
    kt, kh, kw = plan.k
    key = (id(plan), cc, occ, _GRID_CU[0])
    geo = _HALO_SPLITS.get(key)
    if geo is None:
        floats, splits = ctypes.c_longlong(0), ctypes.c_int(0)
        rc = lib().milnce_halo_wgrad_plan(plan.B, plan.T, plan.H, plan.W, plan.Cin, plan.Cout, kt, kh, kw, 64, cc,
                                          occ * _GRID_CU[0], ctypes.byref(floats), ctypes.byref(splits))
        if rc != 0:
            raise RuntimeError(f"halo wgrad plan failed ({rc}) for {plan}")
        geo = _HALO_SPLITS[key] = (int(floats.value), int(splits.value))
    slab = torch.empty((geo[0],), dtype=F32, device=dy.device)
    call("milnce_halo_wgrad", ptr(dy), plan.Cout, ptr(x), ptr(slab), ptr(target) if target is not None else None,
         accumulate, plan.B, plan.T, plan.H, plan.W, plan.Cin, plan.Cin_p, plan.Cout, kt, kh, kw, 64, cc, geo[1],
         stream())
    return slab, geo[1], _ceil(plan.Cout, 64) * 64, kt * kh * kw * plan.Cin


# Temporal box wgrad (csrc/conv_twgrad.hip): (3,1,1) / stride 1 / padding (1,0,0) convs, output tiles
# of 64 / 128 / 192 channels x 64 input channels x 3 taps, boxes of 64 (frame, position) rows with
# their 3-frame halo staged once through a counted 3-deep LDS-DMA ring. In the wgrad tuner next to
# the im2col / halo kernels (impl codes 1000 + N tile); MILNCE_TWGRAD=0 leaves it out.
_TWGRAD = os.environ.get("MILNCE_TWGRAD", "1") != "0"
# A temporal conv whose input is a BN-ReLU placeholder ("pro") and whose tuned wgrad is the
# register-staged box wgrad: that wgrad applies the producer's BN-ReLU to its staged x rows itself,
# so the forward's box kernel runs PRO 1 (applies it, writes no z): the input-sized z write of the
# forward is gone (conv_2c's temporal conv: 2 GB per step). MILNCE_TW_PRO=0 keeps writing z.
_TW_PRO = os.environ.get("MILNCE_TW_PRO", "1") != "0"
_TW_OCCS = tuple(int(v) for v in os.environ.get("MILNCE_TW_OCCS", "1,2").split(","))
_TW_SPLITS: Dict[Tuple[int, int, int], Tuple[int, int]] = {}


def _twgrad_ok(plan: ConvPlan, x: torch.Tensor) -> bool:
    return (_TWGRAD and x.dtype == BF16 and plan.k == (3, 1, 1) and plan.s == (1, 1, 1) and plan.p == (1, 0, 0)
            and not plan.wo_override and plan.Cin % 8 == 0 and plan.Cin == plan.Cin_p and plan.Cout % 8 == 0)


def _tw_tiles(cout: int) -> Tuple[int, ...]:
    """Output tiles worth trying: no more than one 64-wide tile of padding."""
    return tuple(bn for bn in (192, 128, 64) if _ceil(cout, bn) * bn - cout < 64)


def _twgrad(dy, x, plan: ConvPlan, bn: int, target: Optional[torch.Tensor], accumulate: int, occ: int = 1,
            reg: int = 1, xss: Optional[torch.Tensor] = None):
    """Temporal box wgrad (reg: register-staged boxes, else the LDS-DMA ring); with ``target`` None
    only the split slab is filled and (slab, splits, Npad, Kpad) of the pending reduction is returned.
    ``xss`` (register-staged only): x is a BN layer's raw output and the operand relu(x * scale +
    shift) with that layer's constants (see _TW_PRO)."""
    key = (id(plan), bn, occ, _GRID_CU[0])
    geo = _TW_SPLITS.get(key)
    if geo is None:
        floats, splits = ctypes.c_longlong(0), ctypes.c_int(0)
        rc = lib().milnce_twgrad_plan(plan.B, plan.T, plan.H, plan.W, plan.Cin, plan.Cout, bn, occ * _GRID_CU[0],
                                      ctypes.byref(floats), ctypes.byref(splits))
        if rc != 0:
            raise RuntimeError(f"temporal wgrad plan failed ({rc}) for {plan}")
        geo = _TW_SPLITS[key] = (int(floats.value), int(splits.value))
    slab = torch.empty((geo[0],), dtype=F32, device=dy.device)
    call("milnce_twgrad", ptr(dy), plan.Cout, ptr(x), ptr(slab), ptr(target) if target is not None else None,
         accumulate, plan.B, plan.T, plan.H, plan.W, plan.Cin, plan.Cin_p, plan.Cout, bn, geo[1], int(reg), ptr(xss),
         stream())
    return slab, geo[1], _ceil(plan.Cout, bn) * bn, 3 * plan.Cin


# Deferred slab reductions (conv_wgrad(defer=True)): the split-K reduce of a parameter's wgrad is
# a small latency-bound kernel (~17 us, 58 per flagship step) that nothing in the backward pass
# waits for, so it can run on a side stream overlapping the next layer's kernels; grad_sink.drain()
# joins it before the gradients are read (all-reduce, optimizer). Opt-in (MILNCE_DEFER_WGRAD=1):
# same-box bench A/B 4012 pairs/s inline vs 4003 deferred -- the big kernels it would overlap
# already fill the chip, so there is no idle gap for the reduce to hide in.
_DEFER_WGRAD = os.environ.get("MILNCE_DEFER_WGRAD", "0") == "1"
# Side-stream weight gradients (default; MILNCE_WGRAD_SIDE=0 disables): the whole wgrad (kernel +
# slab reduction) of every conv+BN layer runs on the side stream, so the MFMA-heavy weight
# gradients overlap the rest of the backward chain (dgrads, BN / pool / gate backward passes) of the
# next layers; grad_sink joins them before the gradients are read. Same-box bench A/Bs
# (profiles/r5_wgrad_side.md): +2.8 / +3.2 % pairs/s; variants that kept the persistent dgrads off
# the side stream's work (dgrads waiting for it: +1 %) or enqueued each wgrad ahead of its layer's
# dgrad (+2.4 %), high-priority streams for either side (+1-2 %) and CU-masked side streams
# (-15 %) all measured lower.
_WGRAD_SIDE = os.environ.get("MILNCE_WGRAD_SIDE", "1") != "0"
# layers with more output rows than this keep their wgrad on the main stream (A/B knob; 0 = none)
_WGRAD_SIDE_MAX_M = int(os.environ.get("MILNCE_WGRAD_SIDE_MAX_M", "0"))
# Side-stream memory policy, decided per training step from the PREVIOUS step's peak allocated
# memory (each step start reads it and resets the counter; before any step was measured the wgrads
# run inline: step 0 of a near-capacity config must not take the side-stream regime). A side-stream
# wgrad's operands (dy, x: main-stream allocations) must stay alive until the side stream passed
# them, in one of two ways:
#   "record": Tensor.record_stream -- the caching allocator defers their reuse to an event; its
#             reserved pool then grows to ~6x the allocated peak (bs 256: 160 GiB reserved for
#             23 GiB allocated), and near capacity it thrashes (BASELINE config 5 at 2537-6960
#             ms/step instead of 488 inline);
#   "keep":   the references are held until the wgrad's event completed (or the backward pass's
#             drain made the current stream wait for it), _SideKeep: reserved ~= allocated (bs 256:
#             37.5 GiB reserved for 31.8 allocated; config 5: 2142 pairs/s vs 2098 inline at 248 GiB
#             peak), at ~0.5-1 % of the bs-256 step (same-box A/Bs, profiles/r6_side_memory.md).
# Below MILNCE_WGRAD_SIDE_MEM_FRAC (0.4) of the device the step uses "record" (fastest), below
# MILNCE_WGRAD_SIDE_KEEP_FRAC (0.93) "keep", above it inline; a "keep" step that went above the
# limit turns the side stream off for the rest of the run (no oscillation near capacity).
# MILNCE_SIDE_KEEP=1 forces "keep" wherever the side stream is used, =2 releases only at the drain.
# In "record" mode the reserved pool is bounded too: a step that left more than
# MILNCE_WGRAD_SIDE_RESERVED_FRAC (0.85) of the device reserved with a quarter of the device cached
# but unallocated releases the cache.
_WGRAD_SIDE_MEM_FRAC = float(os.environ.get("MILNCE_WGRAD_SIDE_MEM_FRAC", "0.4"))
_WGRAD_SIDE_KEEP_FRAC = float(os.environ.get("MILNCE_WGRAD_SIDE_KEEP_FRAC", "0.93"))
_WGRAD_SIDE_RESERVED_FRAC = float(os.environ.get("MILNCE_WGRAD_SIDE_RESERVED_FRAC", "0.85"))
_KEEP_ENV = int(os.environ.get("MILNCE_SIDE_KEEP", "0"))
_SIDE_MODE: Dict[int, str] = {}  # per device: "inline" | "record" | "keep" (training-step start)
_KEEP_TRIPPED: Dict[int, bool] = {}
_DEV_TOTAL: Dict[int, int] = {}
_HEADROOM_STATS = {"inline_steps": 0, "record_steps": 0, "keep_steps": 0, "cache_releases": 0}


def _refresh_headroom(device: torch.device) -> None:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    total = _DEV_TOTAL.get(idx)
    if total is None:
        total = _DEV_TOTAL[idx] = torch.cuda.get_device_properties(idx).total_memory
        # the counter covers whatever ran before the first step (model build, tuning): not a step
        mode = "inline"
    else:
        prev = _SIDE_MODE.get(idx, "inline")
        peak = torch.cuda.max_memory_allocated(idx)
        if prev == "keep" and peak >= _WGRAD_SIDE_KEEP_FRAC * total:
            _KEEP_TRIPPED[idx] = True
        if peak < _WGRAD_SIDE_MEM_FRAC * total:
            mode = "keep" if _KEEP_ENV else "record"
        elif peak < _WGRAD_SIDE_KEEP_FRAC * total and not _KEEP_TRIPPED.get(idx, False):
            mode = "keep"
        else:
            mode = "inline"
        reserved = torch.cuda.memory_reserved(idx)
        if prev == "record" and reserved > _WGRAD_SIDE_RESERVED_FRAC * total and reserved - peak > 0.25 * total:
            torch.cuda.empty_cache()  # cross-stream frees left the pool inflated
            _HEADROOM_STATS["cache_releases"] += 1
        if mode == "keep" and prev == "record":
            torch.cuda.empty_cache()  # record_stream's bloat from the earlier steps: keep tracks allocated
    _SIDE_MODE[idx] = mode
    torch.cuda.reset_peak_memory_stats(idx)
    _HEADROOM_STATS[mode + "_steps"] += 1


def _side_mode(device: torch.device) -> str:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return _SIDE_MODE.get(idx, "inline")


def _side_headroom(device: torch.device) -> bool:
    return _side_mode(device) != "inline"
_SIDE_STREAMS: Dict[int, torch.cuda.Stream] = {}



# wgrads round-robin over this many side streams (A/B knob; the batched reductions run on the
# first, after it waited for the others)
_N_SIDE = max(1, int(os.environ.get("MILNCE_SIDE_STREAMS", "1")))
_SIDE_RR: Dict[int, int] = {}


def _side_streams(device: torch.device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    ss = _SIDE_STREAMS.get(idx)
    if ss is None:
        ss = _SIDE_STREAMS[idx] = [torch.cuda.Stream(device=idx) for _ in range(_N_SIDE)]
    return ss


def _side_stream(device: torch.device) -> "torch.cuda.Stream":
    """The (first) side stream: reductions, joins."""
    return _side_streams(device)[0]


def _wgrad_stream(device: torch.device) -> "torch.cuda.Stream":
    """The side stream of the next weight gradient (round-robin when MILNCE_SIDE_STREAMS > 1)."""
    ss = _side_streams(device)
    if len(ss) == 1:
        return ss[0]
    idx = device.index if device.index is not None else torch.cuda.current_device()
    k = _SIDE_RR.get(idx, 0)
    _SIDE_RR[idx] = k + 1
    return ss[k % len(ss)]


class _ReduceDesc(ctypes.Structure):
    """Mirror of csrc/conv.hip ``ReduceDesc`` (56 bytes)."""
    _fields_ = [("slab", ctypes.c_void_p), ("dw", ctypes.c_void_p)] + \
        [(f, ctypes.c_int) for f in ("splits", "Npad", "Kpad", "Cout", "Cin", "Cin_param", "taps", "accumulate",
                                     "blk0", "nblk")]


# Batched side-stream slab reductions (MILNCE_REDUCE_BATCH, default on): a side-stream wgrad only
# fills its split-K slab; the reductions into the parameters' gradients queue here and run as ONE
# launch (csrc/conv.hip wgrad_reduce_batch_kernel, bitwise equal to one launch each) when 16 are
# pending or when anything reads the gradients (grad_sink.drain runs the flush first: the bucket
# all-reduces, the optimizer, the end of the backward pass). ~77 reduce launches per step -> ~6.
_REDUCE_BATCH = os.environ.get("MILNCE_REDUCE_BATCH", "1") != "0"
_REDUCE_BATCH_N = 16


class _ReduceBatcher:
    def __init__(self):
        self.items = []  # (slab address, grad address, splits, npad, kpad, rows, cin, cin_p, taps)
        self.slabs = []
        self.targets = set()  # grad addresses of the pending items
        self.device = None

    def add(self, slab: torch.Tensor, entries, device) -> None:
        if not self.items and not self.slabs:
            grad_sink.on_drain(self.flush)
            try:  # the end of the running backward pass drains (and so flushes)
                torch.autograd.Variable._execution_engine.queue_callback(grad_sink.drain)
            except RuntimeError:
                pass
        if any(e[1] in self.targets for e in entries):
            self.flush()  # one launch must not accumulate twice into a gradient (racing read-modify-writes)
        self.device = device
        self.slabs.append(slab)
        self.items.extend(entries)
        self.targets.update(e[1] for e in entries)
        if len(self.items) >= _REDUCE_BATCH_N:
            self.flush()

    def flush(self) -> None:
        if not self.items:
            return
        ss = _side_streams(self.device)
        side = ss[0]
        for other in ss[1:]:  # slabs written on any side stream
            side.wait_stream(other)
        arr = (_ReduceDesc * len(self.items))()
        for i, (sptr, gptr, splits, npad, kpad, rows, cin, cin_p, taps) in enumerate(self.items):
            arr[i] = _ReduceDesc(sptr, gptr, splits, npad, kpad, rows, cin, cin_p, taps, 1, 0, 0)
        call("milnce_wgrad_reduce_batch", ctypes.addressof(arr), len(self.items), side.cuda_stream)
        if len(ss) > 1:  # slabs of the other side streams were read here, on the first
            for slab in self.slabs:
                slab.record_stream(side)
        self.items, self.slabs = [], []  # slabs: side-stream allocations, reused in that stream's order
        self.targets = set()
        ev = torch.cuda.Event()
        ev.record(side)
        grad_sink.defer(ev)


_REDUCER = _ReduceBatcher()


class _SideKeep:
    """Operands (dy, x, ...) of the side-stream wgrads, kept referenced until the side stream is
    known to be past them -- their event completed, or a grad_sink.drain made the current stream
    wait for it -- instead of ``record_stream`` (MILNCE_SIDE_KEEP=1 / 2). With record_stream (the
    default) a tensor freed under a cross-stream record stays unusable for the caching allocator
    until its next event scan, so the reserved pool grows (bs 256: 93 GiB after 8 steps, 171 after
    43, for 27 GiB allocated); kept references bound it (41 GiB reserved, 31.8 GiB allocated) but
    measured ~0.8 % slower (same box, 40 steps: 4651 / 4630 and 4651 / 4659 vs 4694 / 4675)."""

    def __init__(self):
        self.q = collections.deque()
        self.hooked = False

    def add(self, event, tensors) -> None:
        if not self.hooked:
            grad_sink.after_drain(self.release)
            self.hooked = True
        self.q.append((event, tensors))
        while self.q and self.q[0][0] is not None and self.q[0][0].query():
            self.q.popleft()

    def release(self) -> None:
        self.q.clear()


_SIDE_KEEP = _SideKeep()
# (the operand lifetime of a side-stream wgrad: _side_mode "record" -> record_stream, "keep" ->
# released when its event completed or at the drain; MILNCE_SIDE_KEEP=2: only at the drain)


def _reduce_on_side(slab: torch.Tensor, dw: torch.Tensor, splits: int, npad: int, kpad: int, plan: ConvPlan,
                    accumulate: int) -> None:
    main = torch.cuda.current_stream(slab.device)
    side = _side_stream(slab.device)
    side.wait_stream(main)
    call("milnce_wgrad_reduce", ptr(slab), ptr(dw), splits, npad, kpad, plan.Cout, plan.Cin, plan.Cin_p,
         plan.k[0] * plan.k[1] * plan.k[2], accumulate, side.cuda_stream)
    slab.record_stream(side)  # the allocator must not hand the slab to the main stream before the reduce ran
    ev = torch.cuda.Event()
    ev.record(side)
    grad_sink.defer(ev)


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, plan: ConvPlan, out: Optional[torch.Tensor] = None,
               defer: bool = False, outs=None) -> Optional[torch.Tensor]:
    """dW of the conv; with ``out`` the result is accumulated into it (a parameter's grad).
    The first call of a plan tunes over (N tile, kernel variant) pairs on the real operands.
    ``defer`` (with ``out``): the whole wgrad runs on the side stream and is only complete after
    grad_sink.drain(). ``outs`` = [(row offset, rows, grad)]: the Cout rows are split over several
    parameters (a concatenated 1x1 group); each slice of the split-K reduction is accumulated
    into its own gradient and nothing is returned."""
    kt, kh, kw = plan.k
    st, sh, sw = plan.s
    pt, ph, pw = plan.p
    acc = int(out is not None or outs is not None)
    dw = out
    if dw is None and (outs is None or plan.w_impl == 0):  # (split outputs: only the tuner's scratch shape)
        dw = torch.empty((plan.Cout, plan.Cin_p, kt, kh, kw), dtype=F32, device=dy.device)
    ldd = plan.Cout
    xss = None
    if _is_pro(x):  # x stands for relu(y * scale + shift) of its producer BN (_TW_PRO)
        yp, ssp, ldp = x._milnce_bn
        if plan.w_impl >= 2000 and ldp == plan.Cin:  # the register-staged temporal wgrad applies it
            x, xss = yp, ssp
        else:
            x = _materialize(x)
    if _STEM_WGRAD and _is_paired_stem(plan) and x.dtype in (BF16, torch.uint8):
        slab = torch.empty((256 * 64 * 672,), dtype=F32, device=dy.device)
        rc = lib().milnce_stem_wgrad(ptr(dy), ptr(x), int(x.dtype == torch.uint8), ptr(slab), slab.numel(), ptr(dw),
                                     plan.B, plan.T, plan.H, plan.W, acc, stream())
        if rc == 0:
            return dw
        if rc != _STEM_UNSUPPORTED:  # a HIP error, not a geometry the stem kernel skips
            raise RuntimeError(f"milnce_stem_wgrad failed (hip error {rc}) for {plan}")

    def launch_with(tn, impl, occ, tk, target, accumulate):
        """Runs the wgrad into ``target``; with ``target`` None only the split slab is filled and
        (slab, splits, Npad, Kpad) returned for the caller's reduction."""
        if impl >= 1000:  # temporal box wgrad: N tile impl % 1000, register-staged from 2000,
            # software-pipelined across boxes from 3000
            return _twgrad(dy, x, plan, impl % 1000, target, accumulate, occ, impl // 1000 - 1,
                           xss if impl >= 2000 else None)
        if impl >= 100:  # box-tiled halo wgrad, channel chunk impl - 100
            return _halo_wgrad(dy, x, plan, impl - 100, target, accumulate, occ)
        npad, kpad, splits = _wgrad_geom(plan.Cout, plan.Ktot, plan.M, tn, tk, occ)
        slab = torch.empty((splits, npad, kpad), dtype=F32, device=dy.device)
        call("milnce_conv_wgrad", ptr(dy), ldd, ptr(x), int(x.dtype == torch.uint8), ptr(slab),
             ptr(target) if target is not None else None,
             plan.B, plan.T, plan.H, plan.W, plan.Cin, plan.Cin_p, plan.Cout, kt, kh, kw, st, sh, sw, pt, ph, pw,
             kpad, npad, tn, tk, splits, accumulate, plan.wo_override, impl, stream())
        return slab, splits, npad, kpad

    if plan.w_impl == 0:
        if x.dtype == torch.uint8 or not _AUTOTUNE:
            plan.w_impl = 2 if x.dtype == torch.uint8 else _DEFAULT_IMPL
        else:
            scratch = torch.empty_like(dw)  # tune on a scratch output: the real one may accumulate
            cands = []
            for tk in _wgrad_tks(plan):
                for tn in _wgrad_tiles_for(plan.Cout, tk):
                    for impl in _wide_w_impls(tn, tk):
                        for occ in _W_OCCS:
                            cands.append((tn, impl, occ, tk))
            if _halo_wgrad_ok(plan, x):
                cands += [(64, 164, occ, 0) for occ in _HALO_OCCS]
                if plan.k == (3, 1, 1) and plan.Cin % 128 == 0:  # temporal boxes also take 128-channel chunks
                    cands += [(64, 228, occ, 0) for occ in _HALO_OCCS]
            if _twgrad_ok(plan, x):
                cands += [(bn, base + bn, occ, 0) for base in (1000, 2000, 3000) for bn in _tw_tiles(plan.Cout)
                          for occ in _TW_OCCS]
            code = {c: i + 1 for i, c in enumerate(cands)}
            inv = {v: k for k, v in code.items()}
            default = (plan.w_tn, _DEFAULT_IMPL, 4, plan.w_tk)
            best = _tune(lambda c: launch_with(*inv[c], scratch, 0), tuple(code.values()),
                         default=code.get(default), sig=f"wgrad{_plan_sig(plan)}|{sorted(cands)}")
            tn, impl, occ, tk = inv[best]
            _tune_log(f"wgrad{_plan_sig(plan)} -> tn {tn} impl {impl} occ {occ} tk {tk}")
            plan.w_tn, plan.w_impl, plan.w_occ = tn, impl, occ
            if impl < 100:
                plan.w_tk = tk
            plan.w_Npad, plan.w_Kpad, plan.w_splits = _wgrad_geom(plan.Cout, plan.Ktot, plan.M, tn, plan.w_tk, occ)
    if outs is not None:
        if plan.w_impl >= 100:
            raise RuntimeError(f"split wgrad outputs need a split-K slab kernel, got impl {plan.w_impl}")

        def launch_split():
            slab, splits, npad, kpad = launch_with(plan.w_tn, plan.w_impl, plan.w_occ, plan.w_tk, None, 1)
            for off, rows, g in outs:
                call("milnce_wgrad_reduce", ptr(slab) + off * kpad * 4, ptr(g), splits, npad, kpad, rows,
                     plan.Cin, plan.Cin_p, kt * kh * kw, 1, stream())
    side_ok = (_WGRAD_SIDE and (_WGRAD_SIDE_MAX_M <= 0 or plan.M <= _WGRAD_SIDE_MAX_M)
               and _side_headroom(dy.device))
    if outs is not None and not (defer and side_ok):
        launch_split()
        return None
    if defer and (out is not None or outs is not None) and side_ok:
        # the whole weight gradient on the side stream, overlapping the rest of the backward
        # pass (its operands are kept alive for that stream; grad_sink joins it)
        main = torch.cuda.current_stream(dy.device)
        side = _wgrad_stream(dy.device)
        side.wait_stream(main)
        batched = _REDUCE_BATCH and plan.w_impl is not None
        with torch.cuda.stream(side):
            if _SIDE_GRID_FRAC < 1.0:
                _GRID_CU[0] = max(1, int(_NUM_CU * _SIDE_GRID_FRAC))
            if _SIDE_LDS_FLOOR:
                lib().milnce_set_lds_floor(_SIDE_LDS_FLOOR)
            try:
                if batched:  # the slab now, its reduction(s) with the next batch (_ReduceBatcher)
                    slab, splits, npad, kpad = launch_with(plan.w_tn, plan.w_impl, plan.w_occ, plan.w_tk, None, 1)
                    taps = kt * kh * kw
                    dsts = outs if outs is not None else [(0, plan.Cout, dw)]
                    entries = [(ptr(slab) + off * kpad * 4, ptr(g), splits, npad, kpad, rows, plan.Cin, plan.Cin_p,
                                taps) for off, rows, g in dsts]
                elif outs is not None:
                    launch_split()
                else:
                    launch_with(plan.w_tn, plan.w_impl, plan.w_occ, plan.w_tk, dw, acc)
            finally:  # later plans key their split geometry on _GRID_CU: never leave it reduced
                _GRID_CU[0] = _NUM_CU
                if _SIDE_LDS_FLOOR:
                    lib().milnce_set_lds_floor(0)
        if _side_mode(dy.device) == "keep":
            kev = None
            if _KEEP_ENV != 2:
                kev = torch.cuda.Event()
                kev.record(side)
            _SIDE_KEEP.add(kev, (dy, x, xss))
        else:
            for t in (dy, x, xss):
                if t is not None:
                    t.record_stream(side)
        if batched:
            _REDUCER.add(slab, entries, dy.device)
        else:
            ev = torch.cuda.Event()
            ev.record(side)
            grad_sink.defer(ev)
        if outs is not None:
            return None
    elif defer and out is not None and _DEFER_WGRAD:
        slab, splits, npad, kpad = launch_with(plan.w_tn, plan.w_impl, plan.w_occ, plan.w_tk, None, acc)
        _reduce_on_side(slab, dw, splits, npad, kpad, plan, acc)
    else:
        launch_with(plan.w_tn, plan.w_impl, plan.w_occ, plan.w_tk, dw, acc)
    return dw


def _bn_nparts(M: int) -> int:
    # >= ~4 blocks per CU for parallelism, >= 64 rows per block, <= 2048 partial rows
    return int(max(1, min(2048, max(min(1024, _ceil(M, 64)), _ceil(M, 2048)))))


# Pre-BN storage shift (MILNCE_BN_SHIFT, reference s3dg.py:107-111 trains BN on fp32 conv outputs):
# in training, the conv epilogue stores y - running_mean (per channel) in bf16 instead of y, so a
# channel whose mean is large against its spread keeps its precision in the rounding (trained
# S3D-G layers have |mean| >> std). The statistics, the finalize's mean and everything reading y
# (BN apply, lazy z, BN backward, the fused partial epilogues) live in the shifted frame, which is
# exact: BN is invariant to a per-channel constant. bn_finalize adds the shift back for the running
# mean. Eval stores y unshifted (its BN folds the running statistics).
_BN_SHIFT = os.environ.get("MILNCE_BN_SHIFT", "1") == "1"


def _bn_shift(rmeans, training: bool) -> Optional[torch.Tensor]:
    """The epilogue shift for conv outputs feeding the BNs with running means ``rmeans`` (in
    output channel order): the running mean itself for one BN, else a persistent concatenated
    buffer kept on the first running mean, which bn_finalize advances to the new running means
    (so no concatenation launch per step; a stale value is only a different, equally exact shift)."""
    if not (training and _BN_SHIFT) or any(r is None or r.dtype != F32 or not r.is_contiguous() for r in rmeans):
        return None
    if len(rmeans) == 1:
        return rmeans[0]
    ctot = sum(int(r.numel()) for r in rmeans)
    cached = getattr(rmeans[0], "_milnce_group_shift", None)
    # rebuilt when a running mean was modified from Python (load_state_dict, copy_: the version
    # counters move; the finalize kernel's own updates do not, and it advances the buffer itself)
    vers = tuple(r._version for r in rmeans)
    if cached is None or cached[1] != vers or cached[0].numel() != ctot or cached[0].device != rmeans[0].device:
        cached = (torch.cat([r.detach() for r in rmeans]), vers)
        rmeans[0]._milnce_group_shift = cached
    return cached[0]


def _conv_bn_stats(x, weight, gamma, beta, rmean, rvar, nbt, stride, padding, momentum, eps, training,
                   wo_override=0, pro=None):
    """conv (statistics epilogue) + BN finalize: returns (plan, raw conv output y, ss)."""
    plan = conv_plan(x.shape, weight.shape, stride, padding, wo_override)
    dev = x.device
    wp = _pack(weight, plan, 0)
    nparts = plan.grid_m
    shift = _bn_shift([rmean], training)
    y = None
    if _STEM_FWD and _is_paired_stem(plan) and x.dtype in (BF16, torch.uint8):
        # halo-tiled stem kernel (csrc/conv.hip stem_fwd_kernel); its statistics rows are per workgroup
        y = torch.empty((plan.B, plan.To, plan.Ho, plan.Wo, plan.Cout), dtype=BF16, device=dev)
        stats = torch.empty((256 * 128,), dtype=F32, device=dev)
        rc = lib().milnce_stem_fwd(ptr(x), int(x.dtype == torch.uint8), ptr(wp), plan.Kpad, ptr(y), ptr(stats),
                                   stats.numel(), ptr(shift), plan.B, plan.T, plan.H, plan.W, stream())
        if rc > 0:
            nparts = rc
        elif rc == _STEM_UNSUPPORTED:
            y = None
        else:
            raise RuntimeError(f"milnce_stem_fwd failed (hip error {-rc - 1000}) for {plan}")
    if y is None:
        stats = (torch.empty((_stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), dtype=F32, device=dev)
                 if training else None)
        y = conv_forward_raw(x, wp, plan, stats, pro, shift=shift)
        nparts = plan.grid_m  # as tuned
    C = plan.Cout
    ss = torch.empty((4 * C,), dtype=F32, device=dev)
    call("milnce_bn_finalize", ptr(stats), nparts, plan.Npad, C, float(plan.M), ptr(gamma), ptr(beta),
         ptr(rmean), ptr(rvar), ptr(nbt) if training else None, float(momentum), float(eps), int(training),
         ptr(ss), ptr(shift), stream())
    return plan, y, ss


# Stem wgrad straight from the maxpool_2a backward (csrc/conv.hip stem_wgrad_kernel POOL): the BN
# backward's dy of the stem is rebuilt per item from the pooled gradient, arg-max and raw stem
# output instead of being written by milnce_maxpool_bwd_apply and read back. Opt-in
# (MILNCE_STEM_POOL_WGRAD=1): same-box bench 4140 pairs/s without, 4121 with (the fused kernel's
# register pressure costs more than the dy round trip it saves; csrc/conv.hip stem_wgrad_kernel).
_STEM_POOL_WGRAD = os.environ.get("MILNCE_STEM_POOL_WGRAD", "0") == "1"


def _stem_pool_wgrad_ok(plan: ConvPlan, lazy, x: torch.Tensor, C: int) -> bool:
    if not (_STEM_POOL_WGRAD and _STEM_WGRAD and lazy[0] == "pool" and lazy[4] is None and C == 64
            and _is_paired_stem(plan) and x.dtype in (BF16, torch.uint8)):
        return False
    geo = lazy[3]
    B, T, H, W, _, To, Ho, Wo = geo[:8]
    # (1,3,3) window, (1,2,2) stride, TF-SAME pads (0,0 / 0,1 / 0,1) over an even plane: 2x2 quads
    return (tuple(geo[8:14]) == (1, 3, 3, 1, 2, 2) and tuple(geo[14:20]) == (0, 0, 0, 1, 0, 1)
            and H == 2 * Ho and W == 2 * Wo and To == T)


def _stem_pool_wgrad(lazy, x, y, ss, coef, weight, plan: ConvPlan) -> Optional[torch.Tensor]:
    _, dout, arg, geo, _, _, _ = lazy
    w_direct = _direct_grad(weight)
    dw = w_direct if w_direct is not None else torch.empty(
        (plan.Cout, plan.Cin_p) + tuple(plan.k), dtype=F32, device=dout.device)
    slab = torch.empty((256 * 64 * 672,), dtype=F32, device=dout.device)
    rc = lib().milnce_stem_wgrad_pool(ptr(dout), ptr(arg), ptr(y), ptr(ss), ptr(coef), ptr(x),
                                      int(x.dtype == torch.uint8), ptr(slab), slab.numel(), ptr(dw), plan.B, plan.T,
                                      plan.H, plan.W, int(w_direct is not None), stream())
    if rc != 0:
        raise RuntimeError(f"milnce_stem_wgrad_pool failed ({rc}) for {plan}")
    if w_direct is not None:
        _grad_done(weight)
        return None
    return dw


def _conv_bn_backward(ctx, dz, x, weight, y, ss, gamma):
    """Backward of conv -> BN -> ReLU from dz (grad of the ReLU output): BN backward (fused
    partials when the producer of dz attached them), dgrad, wgrad; BN and weight gradients are
    accumulated in place into flat-buffer grads when possible."""
    adopt(dz)
    plan: ConvPlan = ctx.plan
    lazy = _lazy_dz_info(dz)
    if lazy is None:
        dz = dz.contiguous()
    C = plan.Cout
    dev = dz.device
    fused = take_bn_partials(dz)
    if lazy is not None and fused is None:
        raise RuntimeError("lazy gradient without its BN partial sums")
    if fused is not None:
        part, nparts, ps = fused
    else:
        nparts = _bn_nparts(plan.M)
        part = torch.empty((nparts * 2 * C,), dtype=F32, device=dev)
        ps = C
    coef = torch.empty((3 * C,), dtype=F32, device=dev)
    beta = ctx.beta
    g_direct, b_direct = _direct_grad(gamma), _direct_grad(beta)
    direct_bn = g_direct is not None and b_direct is not None
    dgamma = g_direct if direct_bn else torch.empty((C,), dtype=F32, device=dev)
    dbeta = b_direct if direct_bn else torch.empty((C,), dtype=F32, device=dev)
    if (lazy is not None and not ctx.needs_input_grad[0] and ctx.needs_input_grad[1]
            and _stem_pool_wgrad_ok(plan, lazy, x, C)):
        # stem -> maxpool_2a: the stem wgrad rebuilds dy from the pooled gradient (no dy tensor)
        call("milnce_bn_bwd_finalize", ptr(part), nparts, ps, C, float(plan.M), ptr(gamma), ptr(ss), ptr(dgamma),
             ptr(dbeta), ptr(coef), int(direct_bn), int(ctx.training), stream())
        if direct_bn:
            _grad_done(gamma)
            _grad_done(beta)
            dgamma = dbeta = None
        dw = _stem_pool_wgrad(lazy, x, y, ss, coef, weight, plan)
        return None, dw, dgamma, dbeta
    dy = torch.empty_like(y)
    dx = None
    ck = _ctx_key("dgradbn", "p" if ctx.x_bn is not None else "")
    if (lazy is None and fused is not None and ctx.needs_input_grad[0] and not plan.pin_d and ck not in plan.ctx
            and _BNBWD_FUSE and _PRO_FUSE and _box_geo(plan) is not None and dz.dtype == BF16
            and plan.Cout % 8 == 0):
        _tune_dgrad_bnbwd(plan, dz, weight, y, ss, gamma, part, nparts, ps, ctx.x_bn, ctx.training)
    if lazy is None and fused is not None and ctx.needs_input_grad[0] and _bnbwd_fusable(plan, dz, ck):
        # BN-backward apply inside the dgrad's staging (dy written there for the wgrad)
        call("milnce_bn_bwd_finalize", ptr(part), nparts, ps, C, float(plan.M), ptr(gamma), ptr(ss), ptr(dgamma),
             ptr(dbeta), ptr(coef), int(direct_bn), int(ctx.training), stream())
        dx = conv_dgrad_bnbwd(dz, _pack(weight, plan, 1), plan, ctx.x_bn, y, ss, coef, dy)
    elif lazy is not None:
        _bn_bwd_lazy(lazy, plan.B, plan.M, y, C, ss, C, gamma, part, nparts, ps, dgamma, dbeta, coef, dy, C,
                     direct_bn, ctx.training)
    else:
        call("milnce_bn_bwd", ptr(dz), C, ptr(y), C, ptr(ss), C, plan.M, ptr(gamma), ptr(part), nparts, ps,
             int(fused is not None), ptr(dgamma), ptr(dbeta), ptr(coef), ptr(dy), C, int(direct_bn),
             int(ctx.training), stream())
    if direct_bn:
        _grad_done(gamma)
        _grad_done(beta)
        dgamma = dbeta = None
    if ctx.needs_input_grad[0] and dx is None:
        wd = _pack(weight, plan, 1)
        dx = conv_dgrad(dy, wd, plan, ctx.x_bn)
    dw = None
    if ctx.needs_input_grad[1]:
        w_direct = _direct_grad(weight)
        dw = conv_wgrad(dy, x, plan, out=w_direct, defer=True)
        if w_direct is not None:
            _grad_done(weight)
            dw = None
    return dx, dw, dgamma, dbeta


class _ConvBNReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, rmean, rvar, nbt, stride, padding, momentum, eps, training,
                want_gsum, wo_override=0, lazy_out=False, need_z=True):
        pro, x_saved = None, x
        if _is_pro(x):
            # x stands for its producer's relu(y * scale + shift): this conv's kernel applies it
            # and writes z (the wgrad operand) when one is needed -- not when the tuned wgrad
            # applies it itself (_TW_PRO: x stays the placeholder)
            plan0 = conv_plan(x.shape, weight.shape, stride, padding, wo_override)
            if need_z and _TW_PRO and plan0.w_impl >= 2000 and x._milnce_bn[2] == plan0.Cin:
                pro = (None,)
                ctx.x_pro = x._milnce_bn
            else:
                x_saved = torch.empty(x.shape, dtype=BF16, device=x.device) if need_z else None
                pro = (x_saved,)
        plan, y, ss = _conv_bn_stats(x, weight, gamma, beta, rmean, rvar, nbt, stride, padding, momentum, eps,
                                     training, wo_override, pro)
        C = plan.Cout
        gsum = _zeros_f32((plan.B, C), x.device) if want_gsum else None
        if lazy_out and not want_gsum and _PRO_FUSE:
            z = _pro_z(y.shape, y.device, (y, ss, C))  # applied by the consuming conv
        else:
            lazy = bool(want_gsum) and _LAZY_GATE_Z
            z = _lazy_z(y.shape, y.device, (y, ss, C)) if lazy else torch.empty_like(y)
            if lazy and _defer_gsum(want_gsum):
                gsum._milnce_gsum_deferred = True  # summed with the block's other branches (gate_concat)
            elif (lazy and _GATED_POOL_STATS and training and C <= 2048
                  and not torch.cuda.is_current_stream_capturing()):
                # a single-branch SelfGating (conv_2c -> gated maxpool_3a): also the mask statistics
                mstat = torch.empty((plan.B, 2, C), dtype=F32, device=x.device)
                call("milnce_bn_relu_gsum_mstat", ptr(y), C, ptr(ss), C, plan.B, plan.To * plan.Ho * plan.Wo,
                     ptr(gsum), ptr(mstat), stream())
                gsum._milnce_mstat = mstat
            else:
                call("milnce_bn_relu_apply", ptr(y), C, None if lazy else ptr(z), C, ptr(ss), C, plan.B,
                     plan.To * plan.Ho * plan.Wo, ptr(gsum), stream())
        ctx.save_for_backward(x_saved, weight, y, ss, gamma)
        ctx.beta = beta  # parameter handle only (its gradient buffer may be written in place)
        ctx.training = bool(training)
        ctx.plan = plan
        ctx.x_bn = getattr(x, "_milnce_bn", None)  # (y, ss, ld) of the BN layer that produced x
        z._milnce_bn = (y, ss, C)
        if gsum is None:
            return z
        ctx.mark_non_differentiable(gsum)
        ctx.set_materialize_grads(False)  # no zero-filled (B, C) gradient launch for gsum
        return z, gsum

    @staticmethod
    def backward(ctx, dz, *unused):
        x, weight, y, ss, gamma = ctx.saved_tensors
        x_pro = getattr(ctx, "x_pro", None)
        if x_pro is not None and not _is_pro(x):  # (the saved placeholder without its tags)
            x = _pro_z(x.shape, x.device, x_pro)
        dx, dw, dgamma, dbeta = _conv_bn_backward(ctx, dz, x, weight, y, ss, gamma)
        return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None, None


class _ConvBNReLUPool(torch.autograd.Function):
    """conv -> BN -> ReLU -> TF-SAME max pool (the stem and maxpool_2a, ``s3dg.py:226-228``)
    with the BN+ReLU applied inside the pool's loads: the full-resolution ReLU output is never
    written. Backward: pool backward (dz at full resolution, with the BN-backward partial
    sums), then the conv-BN backward."""

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, rmean, rvar, nbt, stride, padding, momentum, eps, training,
                wo_override, pool_k, pool_s):
        plan, y, ss = _conv_bn_stats(x, weight, gamma, beta, rmean, rvar, nbt, stride, padding, momentum, eps,
                                     training, wo_override)
        B, T, H, W, C = plan.B, plan.To, plan.Ho, plan.Wo, plan.Cout
        pads = aten.tf_same_pad(pool_k, pool_s)
        To = _pool_out(T, pool_k[0], pool_s[0], *pads[0])
        Ho = _pool_out(H, pool_k[1], pool_s[1], *pads[1])
        Wo = _pool_out(W, pool_k[2], pool_s[2], *pads[2])
        out = torch.empty((B, To, Ho, Wo, C), dtype=BF16, device=x.device)
        arg = torch.empty((B, To, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        geo = [B, T, H, W, C, To, Ho, Wo, *pool_k, *pool_s, pads[0][0], pads[0][1], pads[1][0], pads[1][1],
               pads[2][0], pads[2][1], 1]
        # the raw conv output at each arg-max: the consumer's dgrad epilogue then emits this BN's
        # backward partial sums over the pooled gradient (see _POOL_YR)
        yr = torch.empty_like(out) if (_POOL_YR and training and _FUSE_BN_BWD) else None
        call("milnce_bn_relu_maxpool_fwd", ptr(y), ptr(ss), ptr(out), ptr(arg), *geo, ptr(yr), stream())
        if yr is not None:
            out._milnce_bn = (yr, ss, C)
        ctx.save_for_backward(x, weight, y, ss, gamma, arg)
        ctx.beta = beta
        ctx.training = bool(training)
        ctx.plan, ctx.geo = plan, geo
        ctx.x_bn = getattr(x, "_milnce_bn", None)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, weight, y, ss, gamma, arg = ctx.saved_tensors
        geo = ctx.geo
        B, T, H, W, C = geo[:5]
        pre = take_bn_partials(dout)  # from the consumer's dgrad epilogue over (dout, yr)
        dout = dout.contiguous()
        nparts = _pool_nparts(B * T * H * W * (C // 8))
        if pre is not None and _LAZY_POOL_DZ:
            # sum_i dz_i mask_i (1, xhat_i) = sum_o dout_o mask(yr_o) (1, xhat(yr_o)): no partials pass
            dz = _lazy_dz((B, T, H, W, C), dout.device, ("pool", dout, arg, geo, None, None, nparts))
            attach_bn_partials(dz, *pre)
            dx, dw, dgamma, dbeta = _conv_bn_backward(ctx, dz, x, weight, y, ss, gamma)
            return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None
        part = torch.empty((nparts * 2 * C,), dtype=F32, device=dout.device)
        if _LAZY_POOL_DZ and _FUSE_BN_BWD:
            # BN partial sums only; the BN backward re-gathers dz and applies itself in one pass
            call("milnce_maxpool_bwd", ptr(dout), ptr(arg), None, *geo, ptr(y), C, ptr(ss), ptr(part), nparts,
                 stream())
            dz = _lazy_dz((B, T, H, W, C), dout.device, ("pool", dout, arg, geo, None, None, nparts))
        else:
            dz = torch.empty((B, T, H, W, C), dtype=BF16, device=dout.device)
            call("milnce_maxpool_bwd", ptr(dout), ptr(arg), ptr(dz), *geo, ptr(y), C, ptr(ss), ptr(part), nparts,
                 stream())
        attach_bn_partials(dz, part, nparts, C)
        dx, dw, dgamma, dbeta = _conv_bn_backward(ctx, dz, x, weight, y, ss, gamma)
        return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None


def conv_bn_relu(x, weight, bn, stride, padding, training: bool, want_gsum: bool = False, lazy_out: bool = False):
    """conv -> BN -> ReLU. ``lazy_out``: the output feeds only another conv_bn_relu, which may
    apply this BN itself (a "pro" placeholder is returned, see ``_pro_z``)."""
    if not _is_pro(x):
        if x.dtype not in (torch.uint8, BF16):
            x = x.to(BF16)
        x = x.contiguous()
    momentum = bn.momentum if bn.momentum is not None else 0.1
    need_z = torch.is_grad_enabled() and weight.requires_grad  # the wgrad reads the (fused) input
    out = _ConvBNReLU.apply(x, weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                            tuple(stride), tuple(padding), momentum, bn.eps, bool(training), int(want_gsum), 0,
                            bool(lazy_out), bool(need_z))
    return out


# -----------------------------------------------------------------------------------------
# Paired-width stem. The 3x7x7 stride-(2,2,2) stem conv over RGB(+0) pixels has 4-byte operand
# chunks. Reading the bf16 clip [B,T,H,W,4] as width PAIRS [B,T,H,W/2,8] turns it into an
# ordinary conv with 8 input channels, kernel (3,7,4), stride (2,2,1), padding (1,3,2|1):
#     x2[w2][p*4 + c] = x[2*w2 + p][c],  w2[co][p*4 + c][kt][kh][kw4] = w[co][c][kt][kh][2*kw4 + p - 1]
# (zero where c == 3 or the tap index falls outside 0..6), so every operand load is 16 B. The
# weight remap is a differentiable gather, so autograd folds dW2 back into dW.
_STEM_MAP: Dict[torch.device, Tuple[torch.Tensor, torch.Tensor]] = {}


def _stem_pair_map(device) -> Tuple[torch.Tensor, torch.Tensor]:
    hit = _STEM_MAP.get(device)
    if hit is not None:
        return hit
    idx = torch.zeros((8, 3, 7, 4), dtype=torch.long)
    mask = torch.zeros((8, 3, 7, 4), dtype=F32)
    for p_ in range(2):
        for c in range(4):
            for kt in range(3):
                for kh in range(7):
                    for kw4 in range(4):
                        dw = 2 * kw4 + p_ - 1
                        if c < 3 and 0 <= dw < 7:
                            idx[p_ * 4 + c, kt, kh, kw4] = ((c * 3 + kt) * 7 + kh) * 7 + dw
                            mask[p_ * 4 + c, kt, kh, kw4] = 1.0
    hit = (idx.reshape(-1).to(device), mask.reshape(-1).to(device))
    _STEM_MAP[device] = hit
    return hit


def stem_conv_bn_relu_pool(x, weight, bn, training: bool, pool_k, pool_s):
    """The stem unit followed by its TF-SAME max pool (maxpool_2a), fused: see
    ``_ConvBNReLUPool`` and ``stem_conv_bn_relu``."""
    B, T, H, W, C = x.shape
    if C != 4 or W % 2 or tuple(weight.shape) != (64, 3, 3, 7, 7) or x.dtype not in (BF16, torch.uint8):
        raise ValueError(f"stem expects bf16/uint8 [B,T,H,W even,4] and a (64,3,3,7,7) weight, got "
                         f"{tuple(x.shape)} {x.dtype}")
    idx, mask = _stem_pair_map(x.device)
    cout = weight.shape[0]
    w2 = (weight.reshape(cout, -1).index_select(1, idx) * mask).view(cout, 8, 3, 7, 4)
    x2 = x.contiguous().view(B, T, H, W // 2, 8)
    wo = (W + 2 * 3 - 7) // 2 + 1
    momentum = bn.momentum if bn.momentum is not None else 0.1
    return _ConvBNReLUPool.apply(x2, w2, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                 bn.num_batches_tracked, (2, 2, 1), (1, 3, 2), momentum, bn.eps, bool(training), wo,
                                 tuple(pool_k), tuple(pool_s))


def stem_conv_bn_relu(x, weight, bn, training: bool):
    """S3D-G conv1 (``s3dg.py:226``: 3->64, k (3,7,7), s 2, p (1,3,3)) + BN + ReLU on the clip
    ``[B,T,H,W,4]`` (channel 3 zero) via the paired-width formulation above. The clip is bf16, or
    the native uint8 clip, which the stem kernels scale by 1/255 while staging it (no separate
    conversion pass)."""
    B, T, H, W, C = x.shape
    if C != 4 or W % 2 or tuple(weight.shape) != (64, 3, 3, 7, 7):
        raise ValueError(f"stem expects [B,T,H,W even,4] bf16 and a (64,3,3,7,7) weight, got {tuple(x.shape)}")
    if x.dtype not in (BF16, torch.uint8):
        raise TypeError("stem input must be bf16 or uint8 (see prepare_stem_input)")
    idx, mask = _stem_pair_map(x.device)
    cout = weight.shape[0]
    w2 = (weight.reshape(cout, -1).index_select(1, idx) * mask).view(cout, 8, 3, 7, 4)
    x2 = x.contiguous().view(B, T, H, W // 2, 8)
    wo = (W + 2 * 3 - 7) // 2 + 1
    momentum = bn.momentum if bn.momentum is not None else 0.1
    return _ConvBNReLU.apply(x2, w2, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                             (2, 2, 1), (1, 3, 2), momentum, bn.eps, bool(training), False, wo)


class _Conv1x1GroupBNReLU(torch.autograd.Function):
    """Several 1x1x1 conv -> BN -> ReLU units that read the same input (Inception branches
    0, 1a and 2a, ``s3dg.py:13-18``) as ONE implicit GEMM with the output channels
    concatenated: the input is read once, the small branch widths (16/24/32/48) stop wasting
    most of an N tile, and the backward is one dgrad GEMM (no per-branch dX sums) and one wgrad.
    Each branch keeps its own BatchNorm (statistics are per channel, so slicing the fused
    output is exact). Returns the branch outputs, plus the gating sum of the first one."""

    @staticmethod
    def forward(ctx, x, n, training, want_gsum0, hyper, *args):
        return _group_forward(ctx, x, n, training, want_gsum0, hyper, args, ())

    @staticmethod
    def backward(ctx, *grads):
        dx, rest = _group_backward(ctx, grads)
        return (dx, *rest)


def _group_forward(ctx, x, n, training, want_gsum0, hyper, args, extra_saved, lazy_out=()):
    """Forward of the fused 1x1 group (see ``_Conv1x1GroupBNReLU``); ``extra_saved`` tensors are
    appended to the saved tensors (read back by ``_group_backward`` callers)."""
    ws = args[:n]
    bns = [args[n + 5 * i: n + 5 * i + 5] for i in range(n)]  # gamma, beta, rmean, rvar, nbt
    widths = [int(w.shape[0]) for w in ws]
    ctot = sum(widths)
    plan = conv_plan(x.shape, (ctot,) + tuple(ws[0].shape[1:]), (1, 1, 1), (0, 0, 0))
    dev = x.device
    wp = _pack_group(ws, plan, 0)
    stats = (torch.empty((_stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), dtype=F32, device=dev)
             if training else None)
    shift = _bn_shift([b[2] for b in bns], training)
    y = conv_forward_raw(x, wp, plan, stats, shift=shift)
    thw = plan.To * plan.Ho * plan.Wo
    zs, sss, gsum = [], [], None
    off = 0
    y2 = y.view(-1, ctot)
    ss_all = torch.empty((4 * ctot,), dtype=F32, device=dev)  # member i: [4][c] at 4 * off
    if _GROUP_FIN and n <= 4:
        members = (_FinMember * n)()
        o = 0
        for i, (c, (gamma, beta, rmean, rvar, nbt)) in enumerate(zip(widths, bns)):
            members[i] = _FinMember(ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), ptr(nbt) if training else None,
                                    ptr(ss_all) + 16 * o, ptr(shift) + 4 * o if shift is not None else None,
                                    o, c, 0, float(hyper[i][0]), float(hyper[i][1]), 0)
            o += c
        call("milnce_bn_finalize_group", ctypes.addressof(members), n, ptr(stats), plan.grid_m, plan.Npad,
             float(plan.M), int(training), stream())
    for i, (c, (gamma, beta, rmean, rvar, nbt)) in enumerate(zip(widths, bns)):
        ss = ss_all[4 * off:4 * (off + c)]
        if not (_GROUP_FIN and n <= 4):
            st = stats[off:] if training else None
            call("milnce_bn_finalize", ptr(st), plan.grid_m, plan.Npad, c, float(plan.M), ptr(gamma), ptr(beta),
                 ptr(rmean), ptr(rvar), ptr(nbt) if training else None, float(hyper[i][0]),
                 float(hyper[i][1]), int(training), ptr(ss), ptr(shift[off:off + c] if shift is not None else None),
                 stream())
        g = _zeros_f32((plan.B, c), dev) if (i == 0 and want_gsum0) else None
        ysl = y2[:, off:off + c]
        zshape = (plan.B, plan.To, plan.Ho, plan.Wo, c)
        if g is None and i < len(lazy_out) and lazy_out[i] and _PRO_FUSE:
            z = _pro_z(zshape, dev, (ysl, ss, ctot))  # applied by the consuming conv (a channel slice)
        else:
            lazy = g is not None and _LAZY_GATE_Z
            z = _lazy_z(zshape, dev, (ysl, ss, ctot)) if lazy else torch.empty(zshape, dtype=BF16, device=dev)
            if lazy and _defer_gsum(want_gsum0):
                g._milnce_gsum_deferred = True  # summed with the block's other branches (gate_concat)
            else:
                call("milnce_bn_relu_apply", ptr(ysl), ctot, None if lazy else ptr(z), c, ptr(ss), c, plan.B, thw,
                     ptr(g), stream())
        z._milnce_bn = (ysl, ss, ctot)
        zs.append(z)
        sss.append(ss)
        if g is not None:
            gsum = g
        off += c
    ctx.save_for_backward(x, y, *sss, *[b[0] for b in bns], *extra_saved)
    ctx.ws = ws  # the member parameters (packed for the dgrad, direct wgrad targets)
    ctx.betas = [b[1] for b in bns]
    ctx.training = bool(training)
    ctx.plan, ctx.widths, ctx.n = plan, widths, n
    ctx.x_bn = getattr(x, "_milnce_bn", None)
    if gsum is not None:
        ctx.mark_non_differentiable(gsum)
        ctx.set_materialize_grads(False)  # no zero-filled (B, C) gradient launch for gsum
        return (*zs, gsum)
    return tuple(zs)

def _group_backward(ctx, grads, saved=None):
    """Backward of the fused 1x1 group: returns (dX of the GEMM, the remaining grads tuple)."""
    n, widths, plan = ctx.n, ctx.widths, ctx.plan
    adopt(*[g for g in grads if g is not None])
    saved = ctx.saved_tensors if saved is None else saved
    x, y = saved[:2]
    sss = saved[2:2 + n]
    gammas = saved[2 + n:2 + 2 * n]
    ctot = sum(widths)
    dev = y.device
    dY = torch.empty((plan.M, ctot), dtype=BF16, device=dev)
    y2 = y.view(-1, ctot)
    mem = []  # per member: dz, lazy info, partials (part, nparts, ps, fused), coef, dgamma, dbeta, direct
    for i, c in enumerate(widths):
        dz = grads[i]
        if dz is None:
            dz = torch.zeros((plan.M, c), dtype=BF16, device=dev)
        lazy = _lazy_dz_info(dz)
        if lazy is None:
            dz = dz.contiguous()
        fused = take_bn_partials(dz)
        if lazy is not None and fused is None:
            raise RuntimeError("lazy gradient without its BN partial sums")
        if fused is not None:
            part, nparts, ps = fused
        else:
            nparts = _bn_nparts(plan.M)
            part = torch.empty((nparts * 2 * c,), dtype=F32, device=dev)
            ps = c
        coef = torch.empty((3 * c,), dtype=F32, device=dev)
        g_direct, b_direct = _direct_grad(gammas[i]), _direct_grad(ctx.betas[i])
        direct_bn = g_direct is not None and b_direct is not None
        dgamma = g_direct if direct_bn else torch.empty((c,), dtype=F32, device=dev)
        dbeta = b_direct if direct_bn else torch.empty((c,), dtype=F32, device=dev)
        mem.append((dz, lazy, (part, nparts, ps, fused is not None), coef, dgamma, dbeta, direct_bn))
    # one finalize launch for the whole group when every member's partial sums are ready and its
    # apply pass has an apply-only entry (plain or SelfGating-lazy dz)
    grouped = _GROUP_FIN and n <= 4 and all(m[2][3] and (m[1] is None or m[1][0] == "gate") for m in mem)
    if grouped:
        members = (_BwdFinMember * n)()
        for i, (c, (dz, lazy, (part, nparts, ps, _), coef, dgamma, dbeta, direct_bn)) in enumerate(zip(widths, mem)):
            members[i] = _BwdFinMember(ptr(part), ptr(gammas[i]), ptr(sss[i]), ptr(dgamma), ptr(dbeta), ptr(coef),
                                       nparts, ps, c, 0, int(direct_bn), 0)
        call("milnce_bn_bwd_finalize_group", ctypes.addressof(members), n, float(plan.M), int(ctx.training),
             stream())
    dgs, dbs = [], []
    off = 0
    one_pass = grouped and _GROUP_APPLY and ctot % 8 == 0 and ctot <= 2048
    if one_pass:
        arr = (_GroupApplyMember * n)()
        o = 0
        thw = plan.To * plan.Ho * plan.Wo
        for i, (c, (dz, lazy, _, coef, _, _, _)) in enumerate(zip(widths, mem)):
            if lazy is not None:
                _, dout, goff, g, dmean, _ = lazy
                ld = dout.shape[-1]
                arr[i] = _GroupApplyMember(ptr(dout) + 2 * goff, ptr(g) + 4 * goff, ptr(dmean) + 4 * goff, ptr(sss[i]),
                                           ptr(coef), ld, ld, o, c)
            else:
                arr[i] = _GroupApplyMember(ptr(dz), None, None, ptr(sss[i]), ptr(coef), c, 0, o, c)
            o += c
        call("milnce_bn_bwd_apply_group", ctypes.addressof(arr), n, ptr(y2), ctot, plan.B, thw, ptr(dY), stream())
    for i, (c, (dz, lazy, (part, nparts, ps, have_part), coef, dgamma, dbeta, direct_bn)) in enumerate(zip(widths,
                                                                                                       mem)):
        if one_pass:
            pass  # applied above
        elif grouped and lazy is not None:
            _, dout, goff, g, dmean, thw = lazy
            ld = dout.shape[-1]
            call("milnce_bn_bwd_gate_apply", ptr(dout) + 2 * goff, ld, ptr(g) + 4 * goff, ptr(dmean) + 4 * goff, ld,
                 plan.B, thw, ptr(y2[:, off:]), ctot, ptr(sss[i]), ptr(coef), c, ptr(dY[:, off:]), ctot, stream())
        elif grouped:
            call("milnce_bn_bwd_apply", ptr(dz), c, ptr(y2[:, off:]), ctot, ptr(sss[i]), ptr(coef), c, plan.M,
                 ptr(dY[:, off:]), ctot, stream())
        elif lazy is not None:
            _bn_bwd_lazy(lazy, plan.B, plan.M, y2[:, off:], ctot, sss[i], c, gammas[i], part, nparts, ps, dgamma,
                         dbeta, coef, dY[:, off:], ctot, direct_bn, ctx.training)
        else:
            call("milnce_bn_bwd", ptr(dz), c, ptr(y2[:, off:]), ctot, ptr(sss[i]), c, plan.M, ptr(gammas[i]),
                 ptr(part), nparts, ps, int(have_part), ptr(dgamma), ptr(dbeta), ptr(coef),
                 ptr(dY[:, off:]), ctot, int(direct_bn), int(ctx.training), stream())
        if direct_bn:
            _grad_done(gammas[i])
            _grad_done(ctx.betas[i])
            dgamma = dbeta = None
        dgs.append(dgamma)
        dbs.append(dbeta)
        off += c
    dYv = dY.view(plan.B, plan.To, plan.Ho, plan.Wo, ctot)
    dx = None
    if ctx.needs_input_grad[0]:
        dx = conv_dgrad(dYv, _pack_group(ctx.ws, plan, 1), plan, ctx.x_bn)
    directs = [_direct_grad(w) for w in ctx.ws]
    if _GROUP_WGRAD_DIRECT and all(d is not None for d in directs):
        # each member's slice of the split-K reduction lands in its flat-buffer gradient (on the
        # side stream, with the wgrad): no dW concat tensor, no AccumulateGrad adds
        offs = [sum(widths[:i]) for i in range(n)]
        conv_wgrad(dYv, x, plan, defer=True, outs=list(zip(offs, widths, directs)))
        for w in ctx.ws:
            _grad_done(w)
        dws = [None] * n
    else:
        dwcat = conv_wgrad(dYv, x, plan)
        dws, off = [], 0
        for c in widths:
            dws.append(dwcat[off:off + c])
            off += c
    bn_grads = []
    for dg, db in zip(dgs, dbs):
        bn_grads += [dg, db, None, None, None]
    return dx, (None, None, None, None, *dws, *bn_grads)


def conv1x1_group_bn_relu(x, weights, bns, training: bool, want_gsum0: bool = False):
    """Fused 1x1x1 conv-BN-ReLU units sharing input x; see ``_Conv1x1GroupBNReLU``."""
    if x.dtype != BF16:
        x = x.to(BF16)
    x = x.contiguous()
    args = list(weights)
    for bn in bns:
        args += [bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked]
    hyper = tuple((bn.momentum if bn.momentum is not None else 0.1, bn.eps) for bn in bns)
    return _Conv1x1GroupBNReLU.apply(x, len(weights), bool(training), int(want_gsum0), hyper, *args)


class _InceptionHead(torch.autograd.Function):
    """Everything an Inception block reads its input x with (``s3dg.py:13-21``): the fused 1x1
    group GEMM of branches 0/1a/2a and the branch-3 max pool (3x3x3, stride 1, -inf padding).
    Owning both consumers of x lets the backward produce dX in ONE pass: the pool backward
    kernel gathers the pooled gradient, adds the GEMM's dX (no separate autograd add) and,
    when x is a SelfGating output, also emits the previous gate's reduction
    sum_thw dX * x (attached to dX; ``_GateConcat.backward`` then skips its reduce pass).
    Returns (*branch outputs, [gating sum of branch 0], pooled x)."""

    @staticmethod
    def forward(ctx, x, n, training, want_gsum0, hyper, lazy_out, *args):
        B, T, H, W, C = x.shape
        pooled = torch.empty_like(x)
        arg = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
        geo = [B, T, H, W, C, T, H, W, 3, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0]
        side = None
        if _HEAD_POOL_SIDE and x.is_cuda:
            # the branch-3 pool on the (forward-idle) side stream, overlapping the group GEMM and
            # its BN passes; pooled / arg belong to this stream, which joins before returning them
            main = torch.cuda.current_stream(x.device)
            side = _side_stream(x.device)
            side.wait_stream(main)
            call("milnce_maxpool_fwd", ptr(x), ptr(pooled), ptr(arg), *geo, side.cuda_stream)
        else:
            call("milnce_maxpool_fwd", ptr(x), ptr(pooled), ptr(arg), *geo, stream())
        outs = _group_forward(ctx, x, n, training, want_gsum0, hyper, args, (arg,), lazy_out)
        if side is not None:
            main.wait_stream(side)
        ctx.x_gate = bool(getattr(x, "_milnce_gate", False))
        return (*outs, pooled)

    @staticmethod
    def backward(ctx, *grads):
        saved = ctx.saved_tensors
        arg = saved[-1]
        x = saved[0]
        dpooled = grads[-1]
        if dpooled is not None:
            adopt(dpooled)
        dx1, rest = _group_backward(ctx, grads[:-1], saved[:-1])
        rest = (None,) + tuple(rest)  # lazy_out
        B, T, H, W, C = x.shape
        if dpooled is None or not ctx.needs_input_grad[0]:
            return (dx1, *rest)
        dx = torch.empty_like(x)
        gs = torch.empty((B, C), dtype=F32, device=x.device) if ctx.x_gate else None
        call("milnce_maxpool_s1_bwd_fused", ptr(dpooled.contiguous()), ptr(arg), ptr(dx1), ptr(x), ptr(gs),
             ptr(dx), B, T, H, W, C, stream())
        if gs is not None:
            dx._milnce_gs = gs
            dx._milnce_gsver = dx._version
        return (dx, *rest)


_FUSE_HEAD = os.environ.get("MILNCE_FUSE_INCEPTION_HEAD", "1") != "0"
_HEAD_POOL_SIDE = os.environ.get("MILNCE_HEAD_POOL_SIDE", "0") == "1"


def inception_head(x, weights, bns, training: bool, want_gsum0: bool = False, lazy_out=()):
    """Fused 1x1 group + branch-3 pool on the Inception input; see ``_InceptionHead``.
    ``lazy_out[i]``: branch i's output feeds only a conv that may apply its BN + ReLU itself."""
    if x.dtype != BF16:
        x = x.to(BF16)
    x = x.contiguous()
    B, T, H, W, C = x.shape
    if not _FUSE_HEAD or T * H > 512 or C % 8:  # csrc/pool.hip milnce_maxpool_s1_bwd_fused limits
        outs = conv1x1_group_bn_relu(x, weights, bns, training, want_gsum0)
        return (*outs, maxpool3d(x, (3, 3, 3), (1, 1, 1), False))
    args = list(weights)
    for bn in bns:
        args += [bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked]
    hyper = tuple((bn.momentum if bn.momentum is not None else 0.1, bn.eps) for bn in bns)
    return _InceptionHead.apply(x, len(weights), bool(training), int(want_gsum0), hyper,
                                tuple(bool(v) for v in lazy_out), *args)


def take_gate_sums(dout: torch.Tensor):
    """sum_thw dout * out per (clip, channel) if the producer of dout attached it."""
    gs = getattr(dout, "_milnce_gs", None)
    if gs is None or getattr(dout, "_milnce_gsver", -1) != dout._version:
        return None
    return gs


# =========================================================================================
# SelfGating + concat
# =========================================================================================
def _arr(ctype, vals):
    return (ctype * len(vals))(*vals)


def gate_fc_backward(src, g, mean, ws, bs, widths):
    """SelfGating fc backward of every branch in one kernel (csrc/gate.hip gate_fc_bwd_kernel):
    dpre = src * (1 - g) (src itself when g is None), dmean = dpre W, dW = dpre^T mean, db = sum_b
    dpre per branch. Weight / bias gradients that live in the data-parallel flat buffer are
    accumulated there in place (returned as None), the others are returned as fresh tensors."""
    B, ctot = mean.shape
    if ctot != sum(widths):
        raise ValueError("gate_fc_backward: mean / src rows must be the concat of the branches")
    dev = mean.device
    dmean = torch.empty((B, ctot), dtype=F32, device=dev)
    dws, dbs, acc_mask, done = [], [], 0, []
    for i, (w, b, c) in enumerate(zip(ws, bs, widths)):
        wd, bd = _direct_grad(w), _direct_grad(b)
        if wd is not None and bd is not None:
            dws.append(wd)
            dbs.append(bd)
            acc_mask |= 1 << i
            done.append(i)
        else:
            dws.append(torch.empty((c, c), dtype=F32, device=dev))
            dbs.append(torch.empty((c,), dtype=F32, device=dev))
    call("milnce_gate_fc_bwd", len(widths), _arr(ctypes.c_int, widths), ptr(src.contiguous()),
         ptr(None if g is None else g.contiguous()), ptr(mean.contiguous()),
         _arr(ctypes.c_void_p, [ptr(w) for w in ws]), _arr(ctypes.c_void_p, [ptr(d) for d in dws]),
         _arr(ctypes.c_void_p, [ptr(d) for d in dbs]), acc_mask, B, ptr(dmean), stream())
    for i in done:
        _grad_done(ws[i])
        _grad_done(bs[i])
        dws[i] = dbs[i] = None
    return dmean, dws, dbs


class _GateConcat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, nseg, gsum, *args):
        zs = args[:nseg]
        ws = args[nseg:2 * nseg]
        bs = args[2 * nseg:3 * nseg]
        B, T, H, W = zs[0].shape[:4]
        thw = T * H * W
        widths = [int(z.shape[-1]) for z in zs]
        ctot = sum(widths)
        dev = zs[0].device
        mean = torch.empty((B, ctot), dtype=F32, device=dev)
        g = torch.empty((B, ctot), dtype=F32, device=dev)
        out = torch.empty((B, T, H, W, ctot), dtype=BF16, device=dev)
        lazy = [int(_is_lazy(z)) for z in zs]
        bn_info = [z._milnce_bn if _is_lazy(z) else (None, None, 0) for z in zs]
        gsum_pass = int(bool(getattr(gsum, "_milnce_gsum_deferred", False)))  # all branches summed here
        call("milnce_gate_fwd", nseg, _arr(ctypes.c_int, widths), _arr(ctypes.c_void_p, [ptr(z) for z in zs]),
             _arr(ctypes.c_void_p, [ptr(w) for w in ws]), _arr(ctypes.c_void_p, [ptr(b) for b in bs]),
             ptr(gsum), B, thw, ptr(mean), ptr(g), ptr(out), _arr(ctypes.c_int, lazy),
             _arr(ctypes.c_void_p, [ptr(i[0]) for i in bn_info]), _arr(ctypes.c_void_p, [ptr(i[1]) for i in bn_info]),
             _arr(ctypes.c_int, [int(i[2]) for i in bn_info]), gsum_pass, stream())
        ctx.save_for_backward(*zs, *ws, g, mean)
        ctx.nseg, ctx.widths, ctx.thw = nseg, widths, thw
        ctx.bs = bs  # parameter handles only (their gradient buffers may be written in place)
        ctx.z_bn = [getattr(z, "_milnce_bn", None) for z in zs]
        ctx.lazy = lazy
        out._milnce_gate = True  # consumers may return sum_thw dout * out with the gradient
        return out

    @staticmethod
    def backward(ctx, dout):
        nseg = ctx.nseg
        saved = ctx.saved_tensors
        zs = saved[:nseg]
        ws = saved[nseg:2 * nseg]
        g, mean = saved[2 * nseg], saved[2 * nseg + 1]
        dout = dout.contiguous()
        B = g.shape[0]
        ctot = g.shape[1]
        dev = dout.device
        widths = _arr(ctypes.c_int, ctx.widths)
        gs = take_gate_sums(dout)
        # gs = sum dout * bf16(z * g) = g * sum dout * z, so dpre = gs * (1 - g) (in gate_fc_backward)
        if gs is None:
            dpre = _zeros_f32((B, ctot), dev)
            zr = [_materialize(z) if _is_lazy(z) else z for z in zs]
            call("milnce_gate_bwd_reduce", nseg, widths, _arr(ctypes.c_void_p, [ptr(z) for z in zr]), ptr(dout),
                 ptr(g), B, ctx.thw, ptr(dpre), stream())
        if gs is not None:
            dmean, dws, dbs = gate_fc_backward(gs, g, mean, ws, ctx.bs, ctx.widths)
        else:
            dmean, dws, dbs = gate_fc_backward(dpre, None, mean, ws, ctx.bs, ctx.widths)
        have_bn = all(zb is not None for zb in ctx.z_bn)
        nparts = B * int(max(1, min(_ceil(2048, B), _ceil(ctx.thw, 128))))
        part = torch.empty((nparts * 2 * ctot,), dtype=F32, device=dev) if have_bn else None
        # a lazy input's gradient is not stored either: its BN backward rebuilds it from dout
        lazy_dz = [bool(have_bn and _FUSE_BN_BWD and _LAZY_GATE_DZ and lz) for lz in ctx.lazy]
        offs = [sum(ctx.widths[:i]) for i in range(nseg)]
        dzs = [_lazy_dz(z.shape, dev, ("gate", dout, offs[i], g, dmean, ctx.thw)) if lazy_dz[i]
               else torch.empty(z.shape, dtype=BF16, device=dev) for i, z in enumerate(zs)]
        call("milnce_gate_bwd_apply", nseg, widths,
             _arr(ctypes.c_void_p, [0 if lz else ptr(d) for lz, d in zip(lazy_dz, dzs)]), ptr(dout),
             ptr(g), ptr(dmean), B, ctx.thw,
             _arr(ctypes.c_void_p, [ptr(zb[0]) for zb in ctx.z_bn]) if have_bn else None,
             _arr(ctypes.c_void_p, [ptr(zb[1]) for zb in ctx.z_bn]) if have_bn else None,
             _arr(ctypes.c_int, [int(zb[2]) for zb in ctx.z_bn]) if have_bn else None,
             ptr(part), nparts, stream())
        if have_bn:
            off = 0
            for d, c in zip(dzs, ctx.widths):
                attach_bn_partials(d, part[off:], nparts, ctot)
                off += c
        return (None, None, *dzs, *dws, *dbs)


def gate_concat(branches, fc_weights, fc_biases, gsums=None):
    branches = [b if _is_lazy(b) else (b.contiguous() if b.dtype == BF16 else b.to(BF16).contiguous())
                for b in branches]
    if gsums is None or any(s is None for s in gsums):
        gsums = [b.float().sum(dim=(1, 2, 3)) for b in branches]
    deferred = [bool(getattr(s, "_milnce_gsum_deferred", False)) for s in gsums]
    if all(deferred) and all(_is_lazy(b) for b in branches):
        # every branch's sums in one pass inside the gate forward (gsum_pass)
        gsum = _zeros_f32((branches[0].shape[0], sum(int(b.shape[-1]) for b in branches)), branches[0].device)
        gsum._milnce_gsum_deferred = True
    else:
        for s, b, d in zip(gsums, branches, deferred):
            if d:  # a deferred branch next to non-deferred ones: its own gsum-only pass now
                y, ss, ld = b._milnce_bn
                C = int(b.shape[-1])
                call("milnce_bn_relu_apply", ptr(y), ld, None, C, ptr(ss), C, b.shape[0],
                     b.numel() // (b.shape[0] * C), ptr(s), stream())
        gsum = gsums[0] if len(gsums) == 1 else torch.cat(gsums, dim=1)
    return _GateConcat.apply(len(branches), gsum.contiguous(), *branches, *fc_weights, *fc_biases)


# =========================================================================================
# Pools
# =========================================================================================
def _pool_out(n: int, k: int, s: int, p0: int, p1: int) -> int:
    np_ = n + p0 + p1
    o = -(-(np_ - k) // s) + 1
    if (o - 1) * s >= np_:
        o -= 1
    return o


_POOL_SPECIAL = {((1, 3, 3), (1, 2, 2)), ((3, 3, 3), (2, 2, 2)), ((2, 2, 2), (2, 2, 2))}
# Workgroups (= BN partial rows) of the gather pool backwards (MILNCE_POOL_PARTS; 2560, a multiple
# of the 5-blocks-per-CU residency, measured 0.5 % slower than 2048 in a same-box A/B)
_POOL_PARTS = int(os.environ.get("MILNCE_POOL_PARTS", "2048"))


def _pool_nparts(chunks: int) -> int:
    """Blocks of a pool backward over `chunks` 8-channel cells (256 threads, one cell each per pass)."""
    return int(max(1, min(_POOL_PARTS, _ceil(chunks, 256))))



class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, stride, tf_same):
        B, T, H, W, C = x.shape
        if tf_same:
            pads = aten.tf_same_pad(kernel, stride)
            zero_pad = 1
        else:
            pads = [(1, 1)] * 3
            zero_pad = 0
        To = _pool_out(T, kernel[0], stride[0], *pads[0])
        Ho = _pool_out(H, kernel[1], stride[1], *pads[1])
        Wo = _pool_out(W, kernel[2], stride[2], *pads[2])
        y = torch.empty((B, To, Ho, Wo, C), dtype=BF16, device=x.device)
        arg = torch.empty((B, To, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        geo = [B, T, H, W, C, To, Ho, Wo, *kernel, *stride, pads[0][0], pads[0][1], pads[1][0], pads[1][1],
               pads[2][0], pads[2][1], zero_pad]
        call("milnce_maxpool_fwd", ptr(x), ptr(y), ptr(arg), *geo, stream())
        ctx.geo = geo
        xb = getattr(x, "_milnce_bn", None)
        special = (tuple(kernel), tuple(stride)) in _POOL_SPECIAL  # csrc/pool.hip MILNCE_POOL_SHAPES
        # (the stride-1 plane sweep's codes are read by its own backward only, which takes no BN
        # partials: csrc/pool.hip S1Geo)
        s1 = tuple(kernel) == (3, 3, 3) and tuple(stride) == (1, 1, 1) and not tf_same
        ctx.x_bn = xb if (xb is not None and not s1 and (special or (256 % (C // 8) == 0 and xb[2] == C))) else None
        # a SelfGating output: the backward also returns the gate's reduction sum dx * x
        ctx.x_gate = bool(getattr(x, "_milnce_gate", False)) and special and tf_same and ctx.x_bn is None
        if ctx.x_gate:
            ctx.save_for_backward(arg, x)
        else:
            ctx.save_for_backward(arg)
        return y

    @staticmethod
    def backward(ctx, dy):
        arg = ctx.saved_tensors[0]
        geo = ctx.geo
        B, T, H, W, C = geo[:5]
        dx = torch.empty((B, T, H, W, C), dtype=BF16, device=dy.device)
        nparts = _pool_nparts(B * T * H * W * (C // 8))
        if ctx.x_gate:
            x = ctx.saved_tensors[1]
            gs = _zeros_f32((B, C), dy.device)
            call("milnce_maxpool_bwd_gate", ptr(dy.contiguous()), ptr(arg), ptr(dx), *geo, ptr(x), ptr(gs), nparts,
                 stream())
            dx._milnce_gs = gs
            dx._milnce_gsver = dx._version
            return dx, None, None, None
        xb = ctx.x_bn
        part = torch.empty((nparts * 2 * C,), dtype=F32, device=dy.device) if xb is not None else None
        call("milnce_maxpool_bwd", ptr(dy.contiguous()), ptr(arg), ptr(dx), *geo,
             ptr(xb[0]) if xb is not None else None, int(xb[2]) if xb is not None else 0,
             ptr(xb[1]) if xb is not None else None, ptr(part), nparts, stream())
        if part is not None:
            attach_bn_partials(dx, part, nparts, C)
        return dx, None, None, None


_FUSE_GATE_POOL = os.environ.get("MILNCE_FUSE_GATE_POOL", "1") != "0"


class _GatedPool(torch.autograd.Function):
    """SelfGating of a lazy BN-ReLU output followed by its TF-SAME max pool (conv_2c -> gating ->
    maxpool_3a, ``s3dg.py:290-296``) without the full-resolution gate output: the pool applies
    BN + ReLU + gate inside its loads. Backward: the gate reduction is taken on the pooled tensor
    (sum_thw dx * x = sum dy * pooled, every routed gradient lands on its arg-max cell), so the fc
    backward runs first and the pool backward then yields the BN layer's dz = bf16(dx * g + dmean /
    thw) directly (with its BN partial sums; lazily, see ``_LAZY_POOL_DZ``)."""

    @staticmethod
    def forward(ctx, z, gsum, w, bias, kernel, stride):
        y, ss, ld = z._milnce_bn
        B, T, H, W, C = z.shape
        dev = y.device
        mean = torch.empty((B, C), dtype=F32, device=dev)
        g = torch.empty((B, C), dtype=F32, device=dev)
        call("milnce_gate_fwd", 1, _arr(ctypes.c_int, [C]), _arr(ctypes.c_void_p, [0]), _arr(ctypes.c_void_p, [ptr(w)]),
             _arr(ctypes.c_void_p, [ptr(bias)]), ptr(gsum), B, T * H * W, ptr(mean), ptr(g), None, None, None, None,
             None, 0, stream())
        pads = aten.tf_same_pad(kernel, stride)
        To = _pool_out(T, kernel[0], stride[0], *pads[0])
        Ho = _pool_out(H, kernel[1], stride[1], *pads[1])
        Wo = _pool_out(W, kernel[2], stride[2], *pads[2])
        out = torch.empty((B, To, Ho, Wo, C), dtype=BF16, device=dev)
        arg = torch.empty((B, To, Ho, Wo, C), dtype=torch.uint8, device=dev)
        geo = [B, T, H, W, C, To, Ho, Wo, *kernel, *stride, pads[0][0], pads[0][1], pads[1][0], pads[1][1],
               pads[2][0], pads[2][1], 1]
        # pooled-side BN-backward partials (_GATED_POOL_STATS): the raw y at each arg-max, and the
        # mask statistics the gating-sum pass left on gsum
        mstat = getattr(gsum, "_milnce_mstat", None)
        yr = (torch.empty((B, To, Ho, Wo, C), dtype=BF16, device=dev)
              if mstat is not None and ld == C and _LAZY_POOL_DZ and _FUSE_BN_BWD else None)
        call("milnce_bn_relu_gate_maxpool_fwd", ptr(y), ptr(ss), ptr(g), ptr(out), ptr(arg), *geo, ptr(yr), stream())
        ctx.save_for_backward(y, ss, g, mean, w, out, arg, yr, mstat if yr is not None else None)
        ctx.geo, ctx.ld = geo, ld
        ctx.bias = bias
        return out

    @staticmethod
    def backward(ctx, dout):
        y, ss, g, mean, w, out, arg, yr, mstat = ctx.saved_tensors
        geo = ctx.geo
        B, T, H, W, C, To, Ho, Wo = geo[:8]
        dout = dout.contiguous()
        gs = _zeros_f32((B, C), dout.device)
        call("milnce_gate_dot", ptr(dout), ptr(out), B, To * Ho * Wo, C, ptr(gs), stream())
        dmean, (dw,), (db,) = gate_fc_backward(gs, g, mean, [w], [ctx.bias], [C])
        nparts = _pool_nparts(B * T * H * W * (C // 8))
        lazy = _LAZY_POOL_DZ and _FUSE_BN_BWD
        if yr is not None and lazy:
            # partials from the pooled side (see _GATED_POOL_STATS); the apply pass still gathers
            rows = To * Ho * Wo
            splits = max(1, _ceil(rows, 64 * (256 // (C // 8))))
            part = torch.empty((splits * B * 2 * C,), dtype=F32, device=dout.device)
            call("milnce_gated_pool_bn_partials", ptr(dout), ptr(yr), ptr(g), ptr(dmean), ptr(ss), ptr(mstat), C, B,
                 rows, T * H * W, splits, ptr(part), stream())
            dz = _lazy_dz((B, T, H, W, C), dout.device, ("pool", dout, arg, geo, g, dmean, nparts))
            attach_bn_partials(dz, part, splits * B, C)
            return dz, None, dw, db, None, None
        part = torch.empty((nparts * 2 * C,), dtype=F32, device=dout.device)
        dz = None if lazy else torch.empty((B, T, H, W, C), dtype=BF16, device=dout.device)
        call("milnce_maxpool_bwd_gated", ptr(dout), ptr(arg), ptr(dz), *geo, ptr(y), ctx.ld, ptr(ss), ptr(part),
             nparts, ptr(g), ptr(dmean), stream())
        if lazy:
            dz = _lazy_dz((B, T, H, W, C), dout.device, ("pool", dout, arg, geo, g, dmean, nparts))
        attach_bn_partials(dz, part, nparts, C)
        return dz, None, dw, db, None, None


def gated_maxpool(z, gsum, fc_weight, fc_bias, kernel, stride):
    """SelfGating(z) followed by a TF-SAME max pool; fused (``_GatedPool``) when z is a lazy
    BN-ReLU output with its gating sum."""
    C = z.shape[-1]
    if (_FUSE_GATE_POOL and _is_lazy(z) and gsum is not None and (tuple(kernel), tuple(stride)) in _POOL_SPECIAL
            and C % 8 == 0 and C // 8 <= 256 and z._milnce_bn[2] == C):
        return _GatedPool.apply(z, gsum.contiguous(), fc_weight, fc_bias, tuple(kernel), tuple(stride))
    x = gate_concat([z], [fc_weight], [fc_bias], None if gsum is None else [gsum])
    return maxpool3d(x, kernel, stride, True)


def maxpool3d(x, kernel, stride, tf_same: bool):
    return _MaxPool.apply(x.contiguous(), tuple(kernel), tuple(stride), bool(tf_same))


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        B, T, H, W, C = x.shape
        out = torch.zeros((B, C), dtype=F32, device=x.device)
        call("milnce_avgpool", ptr(x), B, T * H * W, C, ptr(out), stream())
        ctx.shape = (B, T, H, W, C)
        ctx.x_gate = bool(getattr(x, "_milnce_gate", False))
        if ctx.x_gate:
            ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dout):
        B, T, H, W, C = ctx.shape
        thw = T * H * W
        dout = dout.contiguous().float()
        dx = torch.empty((B, T, H, W, C), dtype=BF16, device=dout.device)
        call("milnce_avgpool_bwd", ptr(dout), B, thw, C, ptr(dx), stream())
        if ctx.x_gate:
            # the SelfGating reduction of x's producer comes for free: dx is the broadcast
            # bf16(dout / thw), so sum_thw dx * x = bf16(dout / thw) * thw * mean(x)
            (mean,) = ctx.saved_tensors
            dx._milnce_gs = (dout / thw).to(BF16).float() * (mean * thw)
            dx._milnce_gsver = dx._version
        return dx


def global_avgpool(x):
    return _AvgPool.apply(x.contiguous())


# =========================================================================================
# Text tower
# =========================================================================================
class _TextTower(torch.autograd.Function):
    """fc2(max_w relu(fc1(table[tokens]))) (``s3dg.py:196-204``). Forward: the gather, fc1, bias,
    ReLU and the max over words run in ONE MFMA kernel (csrc/misc.hip text_fc1_max_kernel), so
    neither the gathered embeddings [N*Wd, 300] nor the fc1 output [N*Wd, 2048] is stored.
    ``table`` is the bf16 embedding table zero-padded to ``kp`` (multiple of 32) columns."""

    @staticmethod
    def forward(ctx, tokens, table, w1, b1, w2, b2):
        N, Wd = tokens.shape
        F_, D = w1.shape
        kp = table.shape[1]
        w1p = torch.zeros((F_, kp), dtype=BF16, device=w1.device)
        w1p[:, :D] = w1
        hm = torch.empty((N, F_), dtype=F32, device=w1.device)
        arg = torch.empty((N, F_), dtype=torch.uint8, device=w1.device)
        tok = tokens.to(torch.int64).contiguous()
        if _text_fused_ok(Wd, kp, F_):
            call("milnce_text_fc1_max", ptr(tok), N, Wd, ptr(table), ptr(w1p), ptr(b1.float().contiguous()), F_, kp,
                 ptr(hm), ptr(arg), stream())
        else:
            # any other sentence length / embedding width: gathered rows, one bf16 GEMM, then the
            # ReLU + max-over-words kernel (same hm / arg contract as the fused kernel)
            e = table.index_select(0, tok.reshape(-1))
            # fp32 accumulate + fp32 bias, rounded to bf16 once (as the fused kernel does: the
            # arg-max word that routes the gradient is decided on the same values)
            h = torch.addmm(b1.float(), e.float(), w1p.float().t()).to(BF16).view(N, Wd, F_)
            call("milnce_text_relu_max", ptr(h), N, Wd, F_, ptr(hm), ptr(arg), stream())
        out = torch.addmm(b2, hm, w2.t())
        ctx.save_for_backward(tok, table, hm, arg, w2)
        ctx.dims = (N, Wd, F_, D)
        return out

    @staticmethod
    def backward(ctx, dout):
        tok, table, hm, arg, w2 = ctx.saved_tensors
        N, Wd, F_, D = ctx.dims
        dout = dout.contiguous().float()
        dw2 = dout.t().mm(hm)
        db2 = dout.sum(0)
        dhm = dout.mm(w2).contiguous()
        dh = torch.empty((N * Wd, F_), dtype=BF16, device=dout.device)
        call("milnce_text_relu_max_bwd", ptr(dhm), ptr(hm), ptr(arg), N, Wd, F_, ptr(dh), stream())
        # dW1 = dh^T e over the N*Wd word rows: the bf16 wgrad GEMM of a 1x1 conv with M = N*Wd
        # rows (fp32 result; an fp32 vendor GEMM here took ~0.28 ms/step at bs 256)
        kp = table.shape[1]
        rows = N * Wd
        e = table.index_select(0, tok.reshape(-1))  # [rows, kp] bf16, re-gathered (not kept from the forward)
        plan = conv_plan((1, 1, 1, rows, kp), (F_, kp, 1, 1, 1), (1, 1, 1), (0, 0, 0))
        dw1 = conv_wgrad(dh, e, plan).view(F_, kp)[:, :D]
        db1 = dh.sum(0, dtype=F32)
        return None, None, dw1, db1, dw2, db2


def text_table_padded(weight: torch.Tensor) -> torch.Tensor:
    """bf16 copy of the embedding table with its rows zero-padded to a multiple of 32 columns
    (the K step of the fused text kernel; 300 -> 320)."""
    V, D = weight.shape
    kp = _ceil(D, 32) * 32
    t = torch.zeros((V, kp), dtype=BF16, device=weight.device)
    t[:, :D] = weight.detach()
    return t


_TXT_FT = 64  # csrc/misc.hip TXT_FT: fc1 output-feature tile of the fused kernel


def _text_fused_ok(Wd: int, kp: int, F_: int) -> bool:
    """Geometry of the fused gather + fc1 + max kernel (csrc/misc.hip milnce_text_fc1_max):
    <= 32 words, the 300-d word2vec table (320 padded columns), fc1 width a multiple of TXT_FT."""
    return 1 <= Wd <= 32 and kp == 320 and F_ % _TXT_FT == 0


def text_tower(tokens, table_padded, w1, b1, w2, b2):
    if tokens.shape[1] > 255:  # the arg-max is a uint8 word index
        raise ValueError(f"text tower supports up to 255 words per sentence, got {tokens.shape[1]}")
    return _TextTower.apply(tokens.contiguous(), table_padded, w1, b1, w2, b2)


def text_relu_max(h):
    N, Wd, F_ = h.shape
    hb = h.to(BF16).contiguous()
    hm = torch.empty((N, F_), dtype=F32, device=h.device)
    arg = torch.empty((N, F_), dtype=torch.uint8, device=h.device)
    call("milnce_text_relu_max", ptr(hb), N, Wd, F_, ptr(hm), ptr(arg), stream())
    return hm


# =========================================================================================
# MIL-NCE
# =========================================================================================
class _MILNCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, v, t):
        B = v.shape[0]
        K = t.shape[0] // B
        x = v.mm(t.t()).contiguous()
        den = torch.empty((B,), dtype=F32, device=v.device)
        nom = torch.empty((B,), dtype=F32, device=v.device)
        loss = torch.empty((1,), dtype=F32, device=v.device)
        call("milnce_loss_fwd", ptr(x), B, K, ptr(den), ptr(nom), ptr(loss), stream())
        ctx.save_for_backward(v, t, x, den, nom)
        ctx.K = K
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        v, t, x, den, nom = ctx.saved_tensors
        B, K = v.shape[0], ctx.K
        dx = torch.empty_like(x)
        gg = g.reshape(1).float().contiguous()
        call("milnce_loss_bwd", ptr(x), ptr(den), ptr(nom), ptr(gg), B, K, ptr(dx), stream())
        return dx.mm(t), dx.t().mm(v)


class _MILNCEFused(torch.autograd.Function):
    """MIL-NCE without the [Bg, Bg*K] logits (csrc/milnce_fused.hip): split-bf16 MFMA logit tiles
    with row / block-column log-sum-exp partials forward, tile-wise recompute backward. The
    workspace (partials + the split operand copies) is kept for the backward."""

    @staticmethod
    def forward(ctx, v, t):
        B, D = v.shape
        K = t.shape[0] // B
        ws = torch.empty((int(lib().milnce_fused_ws_floats(B, K, D)),), dtype=F32, device=v.device)
        den = torch.empty((B,), dtype=F32, device=v.device)
        nom = torch.empty((B,), dtype=F32, device=v.device)
        loss = torch.empty((1,), dtype=F32, device=v.device)
        call("milnce_fused_fwd", ptr(v), ptr(t), B, K, D, ptr(ws), ptr(den), ptr(nom), ptr(loss), stream())
        ctx.save_for_backward(ws, den, nom)
        ctx.dims = (B, K, D)
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        ws, den, nom = ctx.saved_tensors
        B, K, D = ctx.dims
        dv = torch.empty((B, D), dtype=F32, device=ws.device)
        dt = torch.empty((B * K, D), dtype=F32, device=ws.device)
        gg = g.reshape(1).float().contiguous()
        sv, st = ctypes.c_int(1), ctypes.c_int(1)
        lib().milnce_fused_bwd_splits(B, K, ctypes.byref(sv), ctypes.byref(st))
        sv, st = int(sv.value), int(st.value)
        part = torch.empty((max(sv * B, st * B * K if st > 1 else 0) * D if max(sv, st) > 1 else 1,), dtype=F32,
                           device=ws.device)
        call("milnce_fused_bwd", ptr(ws), B, K, D, ptr(den), ptr(nom), ptr(gg), ptr(dv), ptr(dt), sv, st,
             ptr(part), stream())
        return dv, dt


# Fused from Bg * Bg*K >= 2048 * 8192 logits (BASELINE configs 3 and 5: Bg 2048 on 8 GPUs, Bg 8192):
# the split-bf16 fused loss (csrc/milnce_fused.hip) runs at the speed of the hipBLASLt-materialised
# one there -- steady state on one MI355X, forward + backward: Bg 2048 0.64 vs 0.61 ms, Bg 8192
# 7.75 vs 7.61 ms (tools/milnce_bench.py) -- and never allocates the [Bg, Bg*K] logits (peak +344
# MiB vs +2128 MiB at Bg 8192, tests/test_gpu_halo.py). Smaller batches keep the materialised path
# (Bg 1024: 0.32 vs 0.25 ms). MILNCE_FUSED_LOSS=0/1 forces either path.
_FUSED_LOSS = os.environ.get("MILNCE_FUSED_LOSS", "auto")
_FUSED_MIN_LOGITS = 2048 * 8192


def milnce_fused_ok(v: torch.Tensor, t: torch.Tensor) -> bool:
    B, D = v.shape
    K = t.shape[0] // max(1, B)
    return K >= 1 and 64 % K == 0 and t.shape[0] == B * K and D % 128 == 0 and D <= 512


def milnce_loss(video_embd, text_embd, fused: Optional[bool] = None):
    v, t = video_embd.float().contiguous(), text_embd.float().contiguous()
    if fused is None:
        fused = _FUSED_LOSS == "1" or (_FUSED_LOSS == "auto" and v.shape[0] * t.shape[0] >= _FUSED_MIN_LOGITS)
    if fused and milnce_fused_ok(v, t):
        return _MILNCEFused.apply(v, t)
    return _MILNCE.apply(v, t)


# =========================================================================================
# Optimizer, data, stem input
# =========================================================================================
def adam_step(p, g, m, v, lr, b1, b2, eps, wd, bc1, bc2, grad_scale):
    call("milnce_adam", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), float(lr), float(b1), float(b2), float(eps),
         float(wd), float(bc1), float(bc2), float(grad_scale), stream())


def synth_meta(base: int, B: int, K: int, W: int, vocab: int, ncls: int, seed: int, class_words: int,
               device: torch.device):
    """(tokens int64 [B, K, W], labels int64 [B], labels int32 [B], ids int32 [B]) of the synthetic
    samples base .. base + B - 1 in one launch (data/synthetic.py holds the torch formula)."""
    tok = torch.empty((B, K, W), dtype=torch.int64, device=device)
    lab = torch.empty((B,), dtype=torch.int64, device=device)
    small = torch.empty((2, B), dtype=torch.int32, device=device)
    call("milnce_synth_meta", base, B, K, W, vocab, ncls, seed, class_words, ptr(tok), ptr(lab), ptr(small[0]),
         ptr(small[1]), stream())
    return tok, lab, small[0], small[1]


def synth_video(labels_i32, ids_i32, T, S, seed):
    B = labels_i32.shape[0]
    out = torch.empty((B, T, S, S, 4), dtype=torch.uint8, device=labels_i32.device)
    call("milnce_synth_video", ptr(labels_i32.contiguous()), ptr(ids_i32.contiguous()), B, T, S, ptr(out), stream())
    return out


_STEM_U8 = os.environ.get("MILNCE_STEM_U8", "1") != "0"


def prepare_stem_input(video, native: bool, keep_u8: Optional[bool] = None):
    """Any accepted clip format -> the stem's ``[B,T,H,W,4]`` operand (channel 3 zero).
    uint8 clips stay uint8 (``keep_u8``, default on): the stem kernels convert them (x/255 in
    bf16) while staging their halo, so the clip is never materialised in bf16. Otherwise the
    result is bf16 (values /255 for uint8). Native clips are uint8 ``[B,T,H,W,4]`` already."""
    keep_u8 = _STEM_U8 if keep_u8 is None else keep_u8
    if native:
        v = video.contiguous()
        if v.dtype == BF16:
            return v
        if v.dtype != torch.uint8:
            return v.to(BF16)
        if keep_u8:
            return v
    else:
        B, C, T, H, W = video.shape
        assert C == 3
        video = video.contiguous()
        if video.dtype == torch.uint8:
            v = torch.empty((B, T, H, W, 4), dtype=torch.uint8, device=video.device)
            call("milnce_stem_prep", ptr(video), 0, B, T, H, W, ptr(v), stream())
            if keep_u8:
                return v
        else:
            if video.dtype not in (F32, BF16):
                video = video.float()
            out = torch.empty((B, T, H, W, 4), dtype=BF16, device=video.device)
            call("milnce_stem_prep", ptr(video), 1 if video.dtype == F32 else 2, B, T, H, W, ptr(out), stream())
            return out
    out = torch.empty(v.shape, dtype=BF16, device=v.device)
    call("milnce_u8_to_bf16", ptr(v), ptr(out), v.numel(), stream())
    return out