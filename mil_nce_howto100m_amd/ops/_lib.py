"""ctypes binding of ``libmilnce_hip.so`` (built from ``csrc/*.hip`` by ``csrc/build.py``).

The library exposes a plain C ABI (raw device pointers + ``hipStream_t``), so it needs no torch
headers and builds in seconds. ``torch`` must be imported first so the already-loaded HIP
runtime (soname ``libamdhip64.so.7``) is shared with PyTorch's allocator and streams.
Every call checks the returned ``hipError_t`` and raises on failure — there is no fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_float, c_int, c_longlong, c_void_p
from typing import Dict

import torch  # noqa: F401  (must precede the library load)

_HERE = os.path.dirname(os.path.abspath(__file__))
# MILNCE_LIB_PATH: an alternative build of the same sources (A/B of compile-time kernel options)
LIB_PATH = os.environ.get("MILNCE_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "_native", "libmilnce_hip.so")

P, I, F, D, L = c_void_p, c_int, c_float, c_double, c_longlong

SIGNATURES: Dict[str, list] = {
    "milnce_conv_fwd": [P, I, P, P, P, P, P, I] + [I] * 6 + [I] * 9 + [I] * 8 + [P],
    "milnce_conv_fwd_pro": [P, I, P, P, P, P, P, P] + [I] * 6 + [I] * 3 + [I] * 3 + [I] * 6 + [P],
    "milnce_conv_dgrad_bnbwd": [P, P, P, P, P, P, I, P, P, P, P] + [I] * 6 + [I] * 3 + [I] * 3 + [I] * 5 + [P],
    "milnce_conv_wgrad": [P, I, P, I, P, P] + [I] * 7 + [I] * 9 + [I] * 8 + [P],
    "milnce_pack_weight": [P, P] + [I] * 9 + [P],
    "milnce_halo_wgrad_plan": [I] * 12 + [P, P],
    "milnce_halo_wgrad": [P, I, P, P, P, I] + [I] * 13 + [P],
    "milnce_wgrad_reduce": [P, P] + [I] * 8 + [P],
    "milnce_wgrad_reduce_batch": [P, I, P],
    "milnce_pack_weights_multi": [P, I, I, P],
    "milnce_bn_finalize": [P, I, I, I, D, P, P, P, P, P, F, F, I, P, P, P],
    "milnce_bn_finalize_group": [P, I, P, I, I, D, I, P],
    "milnce_bn_bwd_finalize_group": [P, I, D, I, P],
    "milnce_bn_bwd_apply": [P, I, P, I, P, P, I, L, P, I, P],
    "milnce_bn_bwd_gate_apply": [P, I, P, P, I, I, I, P, I, P, P, I, P, I, P],
    "milnce_bn_relu_apply": [P, I, P, I, P, I, I, I, P, P],
    "milnce_bn_bwd": [P, I, P, I, P, I, L, P, P, I, I, I, P, P, P, P, I, I, I, P],
    "milnce_gate_fwd": [I, P, P, P, P, P, I, I, P, P, P, P, P, P, P, I, P],
    "milnce_gate_bwd_reduce": [I, P, P, P, P, I, I, P, P],
    "milnce_gate_fc_bwd": [I, P, P, P, P, P, P, P, I, I, P, P],
    "milnce_pool_set_quad": [I],
    "milnce_gate_bwd_apply": [I, P, P, P, P, P, I, I, P, P, P, P, I, P],
    "milnce_avgpool": [P, I, I, I, P, P],
    "milnce_avgpool_bwd": [P, I, I, I, P, P],
    "milnce_maxpool_fwd": [P, P, P] + [I] * 21 + [P],
    "milnce_maxpool_bwd": [P, P, P] + [I] * 21 + [P, I, P, P, I, P],
    "milnce_bn_relu_maxpool_fwd": [P, P, P, P] + [I] * 21 + [P, P],
    "milnce_maxpool_s1_bwd_fused": [P, P, P, P, P, P] + [I] * 5 + [P],
    "milnce_set_pool_s1_impl": [I],
    "milnce_set_lds_floor": [I],
    "milnce_bn_bwd_apply_group": [P, I, P, I, I, I, P, P],
    "milnce_set_pool_s1_maxthr": [I],
    "milnce_set_pool_s1_codes": [I],
    "milnce_stem_wgrad": [P, P, I, P, L, P, I, I, I, I, I, P],
    "milnce_stem_wgrad_pool": [P, P, P, P, P, P, I, P, L, P, I, I, I, I, I, P],
    "milnce_stem_fwd": [P, I, P, I, P, P, L, P, I, I, I, I, P],
    "milnce_maxpool_bwd_gate": [P, P, P] + [I] * 21 + [P, P, I, P],
    "milnce_bn_relu_gate_maxpool_fwd": [P, P, P, P, P] + [I] * 21 + [P, P],
    "milnce_bn_relu_gsum_mstat": [P, I, P, I, I, I, P, P, P],
    "milnce_gated_pool_bn_partials": [P, P, P, P, P, P, I, I, I, I, I, P, P],
    "milnce_maxpool_bwd_gated": [P, P, P] + [I] * 21 + [P, I, P, P, I, P, P, P],
    "milnce_maxpool_bwd_apply": [P, P, P] + [I] * 21 + [P, I, P, P, P, P, I, P],
    "milnce_gate_dot": [P, P, I, I, I, P, P],
    "milnce_bn_bwd_gate": [P, I, P, P, I, I, I, P, I, P, I, P, P, I, I, P, P, P, P, I, I, I, P],
    "milnce_bn_bwd_finalize": [P, I, I, I, D, P, P, P, P, P, I, I, P],
    "milnce_adam": [P, P, P, P, L, F, F, F, F, F, F, F, F, P],
    "milnce_synth_video": [P, P, I, I, I, P, P],
    "milnce_synth_meta": [L, I, I, I, I, I, I, I, P, P, P, P, P],
    "milnce_peer_scatter": [P, P, I, L, P],
    "milnce_stem_prep": [P, I, I, I, I, I, P, P],
    "milnce_u8_to_bf16": [P, P, L, P],
    "milnce_text_relu_max": [P, I, I, I, P, P, P],
    "milnce_text_relu_max_bwd": [P, P, P, I, I, I, P, P],
    "milnce_text_fc1_max": [P, I, I, P, P, P, I, I, P, P, P],
    "milnce_loss_fwd": [P, I, I, P, P, P, P],
    "milnce_fused_fwd": [P, P, I, I, I, P, P, P, P, P],
    "milnce_fused_bwd": [P, I, I, I, P, P, P, P, P, I, I, P, P],
    "milnce_fused_ws_floats": [I, I, I],
    "milnce_fused_bwd_splits": [I, I, P, P],
    "milnce_loss_bwd": [P, P, P, P, I, I, P, P],
    "milnce_softdtw_fwd": [P, I, I, I, I, I, L, L, F, F, I, P, P, L, L, L, L, P, P, P],
    "milnce_softdtw_bwd": [P, P, I, I, I, I, I, L, L, F, F, I, P, P, L, L, L, L, P, P, P, P, P],
    "milnce_rowstat": [P, L, I, I, P, P],
    "milnce_rowscale_add": [P, P, P, L, I, P],
    "milnce_dtw_path": [P, I, I, I, P, P, P],
    "milnce_box_set_trace": [P],
    "milnce_twgrad_plan": [I] * 8 + [P, P],
    "milnce_twgrad": [P, I, P, P, P, I] + [I] * 10 + [P, P],
}

# entry points that return something other than an int status
RESTYPES = {"milnce_fused_ws_floats": ctypes.c_longlong}

_lib = None


class NativeLibraryError(RuntimeError):
    pass


class UnsupportedVariant(NativeLibraryError):
    """A kernel variant declined the shape (status -1, csrc/conv_common.h V4_UNSUPPORTED)."""


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python csrc/build.py` (or __graft_entry__.build()). "
            "GPU tensors require the HIP kernels; there is no ATen fallback.")
    l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(l, name, None)
        if fn is None:
            continue
        fn.argtypes = argtypes
        fn.restype = RESTYPES.get(name, c_int)
    _lib = l
    return l


# MILNCE_DEBUG_SYNC=1: synchronise after every native call so an asynchronous kernel fault is
# reported at the op that caused it (the analogue of HIP_LAUNCH_BLOCKING for this library), and
# native calls are counted so the failure names the call index.
_DEBUG_SYNC = os.environ.get("MILNCE_DEBUG_SYNC", "0") == "1"
_calls = 0


def call(name: str, *args) -> None:
    global _calls
    fn = getattr(lib(), name)
    rc = fn(*args)
    if rc == -1:
        raise UnsupportedVariant(f"{name}: the requested kernel variant does not support this shape")
    if rc != 0:
        raise NativeLibraryError(f"{name} failed with hipError {rc}")
    if _DEBUG_SYNC:
        _calls += 1
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:  # the fault surfaced at this op
            raise NativeLibraryError(f"{name} (native call #{_calls}) faulted asynchronously: {e}") from e


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream
