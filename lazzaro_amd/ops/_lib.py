"""Loader for the in-tree HIP kernel library (``lazzaro_amd/_lib/liblzk.so``).

The library is plain C ABI and is loaded with :mod:`ctypes` *after* torch, so
its HIP calls bind to the ``libamdhip64.so.7`` torch already mapped (one HIP
runtime per process; device pointers and streams are shared with torch).

Policy: device tensors ALWAYS go through these kernels. If the library is
missing on a machine with a GPU, :func:`lib` raises -- there is no silent
eager fallback. CPU tensors use the torch reference implementations in
:mod:`lazzaro_amd.ops.reference` (that is the CPU test tier, not a fallback).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# LZK_DEBUG=1 selects the build with device-side bounds asserts
# (``python -m lazzaro_amd._build --debug``)
LIB_PATH = os.path.join(_HERE, "_lib", "liblzk_debug.so" if os.environ.get("LZK_DEBUG") == "1" else "liblzk.so")

_lock = threading.Lock()
_lib = None

P = C.c_void_p
I = C.c_int
L = C.c_long
F = C.c_float
D = C.c_double

# name -> (restype, argtypes)
_SIGS = {
    "lzk_flat_topk_chunks": (I, [I, I, I]),
    "lzk_flat_topk_kslot": (I, [I]),
    "lzk_flat_topk_partial": (I, [P, L, I, P, L, I, P, P, P, F, I, I, I, P, P, P]),
    "lzk_topk_merge": (I, [P, P, I, I, I, I, L, P, P, P]),
    "lzk_flat_topk_partial_masked": (I, [P, L, I, P, L, I, P, P, P, F, I, I, I, P, P, P, P]),
    "lzk_topk_merge_masked": (I, [P, P, I, I, I, I, L, P, P, P, P]),
    "lzk_topk_merge64": (I, [P, P, I, I, I, P, P, P]),
    "lzk_segment_topk": (I, [P, P, L, P, P, P, L, I, I, I, F, P, I, I, P, P, P]),
    "lzk_flat_cand_dual": (I, [P, L, I, P, L, I, I, P, P, P, F, P, P, I, P, P, P, P, P, P, P, I, P, P]),
    "lzk_flat_cand": (I, [P, L, I, P, L, I, I, P, P, P, F, P, I, P, P, P, P, I, P, P]),
    "lzk_flat_top1": (I, [P, L, I, P, L, I, I, P, P, P, P]),
    "lzk_flat_top1_grouped": (I, [P, L, P, L, P, I, P, I, I, P, P, P, P]),
    "lzk_cand_gather": (I, [P, I, P, I, I, I, P, P, P, P, P, P, P]),
    "lzk_cand_grid": (I, [I, I, I]),
    "lzk_cand_select": (I, [P, P, P, I, I, I, I, L, P, P, P, P, P]),
}


class KernelLibraryMissing(RuntimeError):
    pass


def _bind(lib):
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def register(name: str, restype, argtypes) -> None:
    """Let op modules declare additional kernel signatures."""
    _SIGS[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name, None)
        if fn is not None:
            fn.restype = restype
            fn.argtypes = argtypes


def lib():
    """Return the loaded kernel library or raise loudly."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            if os.environ.get("LZK_AUTOBUILD", "1") == "1":
                from .. import _build
                _build.build_kernels(verbose=True, debug=os.environ.get("LZK_DEBUG") == "1")
            if not os.path.exists(LIB_PATH):
                raise KernelLibraryMissing(
                    f"HIP kernel library not found at {LIB_PATH}; run `python -m lazzaro_amd._build`")
        l = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        _bind(l)
        _lib = l
        return _lib


def available() -> bool:
    return os.path.exists(LIB_PATH)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    """The current HIP stream of ``device`` as a raw pointer (called for every
    kernel launch: the raw accessor skips building a Stream object)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        else:
            idx = device.index if isinstance(device, torch.device) else torch.device(device).index
            if idx is None:
                idx = torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, what: str) -> None:
    """Every kernel launch reports through here: typed error + fault point."""
    from ..utils.faults import KernelError, fault_point
    fault_point("kernel." + what)
    if rc != 0:
        raise KernelError(f"{what} failed with hipError {rc}")


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
