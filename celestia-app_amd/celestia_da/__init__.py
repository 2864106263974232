"""celestia_da -- MI355X-native celestia-app data-availability hot path.

Host-side mirror of the reference's Go API (pkg/da, pkg/wrapper, rsmt2d,
go-square square) over the C ABI of libcda.so (include/cda.h).  See DESIGN.md.
"""
from . import _lib, app, blobfactory, da, inclusion, malicious, proof, replay, rsmt2d, square, wrapper  # noqa: F401
from ._lib import (ByzantineDataError, CdaError, Context, PushOrderError, SquareError, UnrepairableError,  # noqa: F401
                   default_context, load)

__all__ = ["app", "da", "rsmt2d", "wrapper", "square", "inclusion", "proof", "replay", "malicious", "blobfactory", "Context", "CdaError", "PushOrderError", "SquareError",
           "ByzantineDataError", "UnrepairableError",
           "default_context", "load"]
