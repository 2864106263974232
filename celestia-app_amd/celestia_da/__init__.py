"""celestia_da -- MI355X-native celestia-app data-availability hot path.

Host-side mirror of the reference's Go API (pkg/da, pkg/wrapper, rsmt2d) over
the C ABI of libcda.so (include/cda.h).  See DESIGN.md.
"""
from . import _lib, da, rsmt2d, wrapper  # noqa: F401
from ._lib import CdaError, Context, PushOrderError, default_context, load  # noqa: F401

__all__ = ["da", "rsmt2d", "wrapper", "Context", "CdaError", "PushOrderError", "default_context", "load"]
