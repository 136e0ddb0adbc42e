"""Loader for the in-tree native build (dpvo_amd/_native/).

The three extension modules keep the reference's module names -- cuda_corr,
cuda_ba, lietorch_backends (setup.py:12-37 of cuteboyqq/DPVO) -- so that code
written against the reference (`import cuda_corr`) finds them once
dpvo_amd is imported.  There is no fallback: if the build is missing the
import fails loudly with the command that produces it.
"""
from __future__ import annotations

import ctypes
import importlib
import os
import sys

NATIVE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_native")
LIB_PATH = os.path.join(NATIVE_DIR, "libdpvo_hot.so")
EXT_NAMES = ("cuda_corr", "cuda_ba", "lietorch_backends")

_BUILD_HINT = "build it with `python -m dpvo_amd.build` (hipcc --offload-arch=gfx950)"


class NativeBuildMissing(ImportError):
    pass


def _ensure_path():
    if NATIVE_DIR not in sys.path:
        sys.path.insert(0, NATIVE_DIR)


def load_extension(name: str):
    """Import one of the extension modules from the in-tree build."""
    import torch  # noqa: F401  (loads libtorch / the HIP runtime first)

    _ensure_path()
    try:
        mod = importlib.import_module(name)
    except ImportError as e:  # pragma: no cover - exercised when unbuilt
        raise NativeBuildMissing(f"dpvo_amd native extension '{name}' not found in "
                                 f"{NATIVE_DIR}: {_BUILD_HINT}") from e
    path = os.path.realpath(getattr(mod, "__file__", ""))
    if not path.startswith(os.path.realpath(NATIVE_DIR)):
        raise NativeBuildMissing(f"'{name}' resolved to {path}, not the in-tree MI355X build; "
                                 f"{_BUILD_HINT}")
    return mod


_lib = None


def c_abi():
    """ctypes handle to libdpvo_hot.so (the C ABI of include/dpvo_hot.h)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeBuildMissing(f"{LIB_PATH} missing: {_BUILD_HINT}")
        import torch  # noqa: F401  (share torch's HIP runtime: same SONAME)

        _lib = ctypes.CDLL(LIB_PATH)
        _lib.dpvo_version.restype = ctypes.c_char_p
        _lib.dpvo_status_string.restype = ctypes.c_char_p
        _lib.dpvo_ba_workspace_bytes.restype = ctypes.c_size_t
    return _lib


def require_gpu(t):
    """Fail loudly instead of silently running anything on the CPU."""
    import torch

    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError("dpvo_amd runs on the GPU only (HIP tensors); got a CPU tensor")
