"""cda — MI355X-native data-availability engine for celestia-app's DA hot path.

Python surface mirroring the reference's packages (pkg/da, pkg/wrapper,
rsmt2d, pkg/inclusion, pkg/proof); the compute lives in libcda.so (HIP, gfx950) behind include/cda.h.
"""
from . import appconsts, da, inclusion, proof, rsmt2d, square, wrapper
from ._native import CdaError, Context, MultiContext, build_info, default_context, lib

__all__ = ["appconsts", "da", "inclusion", "proof", "rsmt2d", "square", "wrapper", "CdaError", "Context", "MultiContext", "default_context",
           "lib"]
