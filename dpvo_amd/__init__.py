"""dpvo_amd -- MI355X-native (gfx950) DPVO per-frame update hot path.

Drop-in replacements for cuteboyqq/DPVO's native surface:

  cuda_corr          A-CORR / A-PATCH (+ backward)   -> dpvo_amd.altcorr
  cuda_ba            F-BA / F-REPROJ / F-NBR          -> dpvo_amd.fastba
  lietorch_backends  L-SE3 (SO3 / SE3)                -> dpvo_amd.lietorch

Importing the package puts the in-tree native build on sys.path, so code
written against the reference (`import cuda_corr`) runs the HIP kernels.
"""
from ._native import EXT_NAMES, NATIVE_DIR, c_abi, load_extension  # noqa: F401

__version__ = "0.1.0"

__all__ = ["altcorr", "fastba", "lietorch", "projective_ops", "load_extension", "c_abi"]
