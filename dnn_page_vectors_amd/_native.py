"""ctypes loaders for the two in-tree native libraries.

* ``libpagevec_rt.so``  — C++ host runtime (featurizer, JSONL reader). CPU only.
* ``libpagevec_hip.so`` — hand-written HIP/CDNA4 kernels (gfx950).

Policy: on a machine with a GPU the HIP library is *required* — ops raise
``NativeUnavailable`` instead of silently falling back to PyTorch.  The pure
PyTorch reference ops are used only when no GPU is present (CPU tests) or when
explicitly requested (``backend="torch"``, used as the eager baseline in
``bench.py``).

HIP symbols follow one convention: every launcher is
``int pv_<op>(..., void* stream)`` returning a ``hipError_t`` code (0 = ok).
Torch must be imported before the HIP library is loaded so the process has a
single HIP runtime (the library's ``libamdhip64.so.7`` NEEDED entry resolves
to the one torch already loaded).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

from . import _build

_lock = threading.Lock()
_rt: Optional[ctypes.CDLL] = None
_hip: Optional[ctypes.CDLL] = None
_hip_err: Optional[str] = None
_hip_debug: Optional[ctypes.CDLL] = None
_use_debug = os.environ.get("PAGEVEC_DEBUG_KERNELS", "0") == "1"
DEBUG_UNITS = ("convfwd", "convbwd", "convf32", "embed", "loss")
DEBUG_BITS = {0: "id out of range", 1: "LDS index out of range", 2: "shape precondition", 3: "sort key out of range",
              4: "argmax out of range", 5: "sorted slot out of range", 6: "positive index out of range"}


class NativeUnavailable(RuntimeError):
    pass


def _autobuild() -> bool:
    return os.environ.get("PAGEVEC_NO_AUTOBUILD", "0") != "1"


def runtime() -> ctypes.CDLL:
    """The host runtime library (built on demand with g++)."""
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            if _autobuild():
                _build.build_runtime()
            if not os.path.exists(_build.RT_LIB):
                raise NativeUnavailable(f"{_build.RT_LIB} missing; run python -m dnn_page_vectors_amd._build")
            lib = ctypes.CDLL(_build.RT_LIB)
            _declare_rt(lib)
            _rt = lib
    return _rt


def _declare_rt(lib: ctypes.CDLL) -> None:
    c = ctypes
    lib.pv_vocab_new.restype = c.c_void_p
    lib.pv_vocab_free.argtypes = [c.c_void_p]
    lib.pv_vocab_add.argtypes = [c.c_void_p, c.c_char_p, c.c_int32]
    lib.pv_vocab_size.argtypes = [c.c_void_p]
    lib.pv_vocab_size.restype = c.c_int64
    lib.pv_featurize.argtypes = [c.POINTER(c.c_char_p), c.c_int, c.c_int, c.c_int, c.c_void_p, c.c_int,
                                 c.c_int, c.c_int, c.c_void_p, c.c_int]
    lib.pv_featurize.restype = c.c_int
    lib.pv_clean_str.argtypes = [c.c_char_p, c.c_char_p, c.c_int64]
    lib.pv_clean_str.restype = c.c_int64
    lib.pv_normalize_html.argtypes = [c.c_char_p, c.c_char_p, c.c_int64]
    lib.pv_normalize_html.restype = c.c_int64
    lib.pv_dataset_open.argtypes = [c.c_char_p, c.c_int, c.c_int]
    lib.pv_dataset_open.restype = c.c_void_p
    lib.pv_dataset_size.argtypes = [c.c_void_p]
    lib.pv_dataset_size.restype = c.c_int64
    lib.pv_dataset_skipped.argtypes = [c.c_void_p]
    lib.pv_dataset_skipped.restype = c.c_int64
    lib.pv_dataset_close.argtypes = [c.c_void_p]
    lib.pv_dataset_batch.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int, c.c_void_p,
                                     c.c_int, c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_int]
    lib.pv_dataset_batch.restype = c.c_int
    lib.pv_dataset_row_text.argtypes = [c.c_void_p, c.c_int64, c.c_int, c.c_char_p, c.c_int64]
    lib.pv_dataset_row_text.restype = c.c_int64


def gpu_present() -> bool:
    """True when a GPU is visible. Uses device_count (does not initialise HIP)."""
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


def use_debug_kernels(on: bool = True) -> None:
    """Route all ops to libpagevec_hip_debug.so (PV_CHECK preconditions compiled in)."""
    global _use_debug
    _use_debug = bool(on)


def hip_debug() -> ctypes.CDLL:
    global _hip_debug
    with _lock:
        if _hip_debug is None:
            import torch  # noqa: F401

            if _build.hip_stale(debug=True):
                if not _autobuild():
                    raise NativeUnavailable(f"{_build.HIP_DEBUG_LIB} is missing or stale; run python -m "
                                            "dnn_page_vectors_amd._build --debug")
                _build.build_hip(debug=True)
            if not os.path.exists(_build.HIP_DEBUG_LIB):
                raise NativeUnavailable(f"{_build.HIP_DEBUG_LIB} missing; run python -m dnn_page_vectors_amd._build "
                                        "--debug")
            lib = ctypes.CDLL(_build.HIP_DEBUG_LIB)
            from .ops import _sigs

            _sigs.declare(lib)
            for u in DEBUG_UNITS:
                fn = getattr(lib, f"pv_debug_{u}")
                fn.argtypes = [ctypes.c_int]
                fn.restype = ctypes.c_uint
            _hip_debug = lib
    return _hip_debug


def debug_status(reset: bool = True) -> dict:
    """{unit: [violated preconditions]} recorded by the debug kernels since the last reset
    (call after a device synchronize)."""
    lib = hip_debug()
    out = {}
    for u in DEBUG_UNITS:
        v = int(getattr(lib, f"pv_debug_{u}")(int(reset)))
        bits = [DEBUG_BITS.get(b, f"bit{b}") for b in range(32) if v >> b & 1]
        if bits:
            out[u] = bits
    return out


def hip(required: bool = True) -> Optional[ctypes.CDLL]:
    """The HIP kernel library. Raises when ``required`` and it cannot be loaded."""
    global _hip, _hip_err
    if _use_debug:
        return hip_debug()
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None and _hip_err is None:
            try:
                import torch  # noqa: F401  (single HIP runtime, see module docstring)

                path = os.environ.get("PAGEVEC_HIP_LIB") or _build.HIP_LIB  # variant A/B builds (tools/)
                if path == _build.HIP_LIB and _build.hip_stale():
                    # missing, or linked from other sources than the tree's (the .so is git-ignored
                    # but travels with the snapshot): rebuild, or refuse to run a stale binary
                    if not _autobuild():
                        raise NativeUnavailable(f"{path} is missing or stale (its link stamp does not match the "
                                                "kernel sources); run python -m dnn_page_vectors_amd._build --hip")
                    _build.build_hip()
                if not os.path.exists(path):
                    raise NativeUnavailable(f"{path} missing")
                lib = ctypes.CDLL(path)
                from .ops import _sigs

                _sigs.declare(lib)
                _hip = lib
            except Exception as e:  # pragma: no cover - exercised on broken installs
                _hip_err = f"{type(e).__name__}: {e}"
    if _hip is None and required:
        raise NativeUnavailable(f"HIP kernel library unavailable: {_hip_err}")
    return _hip


def loaded_libraries() -> list:
    """Paths of in-tree native libraries mapped into this process (for smoke checks)."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libpagevec_" in line:
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out
