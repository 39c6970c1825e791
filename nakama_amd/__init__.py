"""nakama_amd — MI355X-native matchmaker interval pass (drop-in behind
Nakama's server.Matchmaker interface, server/matchmaker.go:169-183).

`LocalMatchmaker` is the product: it binds nakama_amd/libnakama_mm.so (HIP,
gfx950) through the C ABI of include/nakama_mm.h.  There is no CPU fallback:
if the library is missing or no gfx950 device is usable, construction raises.
"""
import os

from . import capi
from .capi import (ErrMatchmakerDelete, ErrMatchmakerDuplicateSession, ErrMatchmakerIndex,  # noqa: F401
                   ErrMatchmakerNotAvailable, ErrMatchmakerQueryInvalid, ErrMatchmakerTicketNotFound,
                   ErrMatchmakerTooManyTickets, ErrMatchmakerUnsupportedQuery, MatchmakerError, Presence, Ticket)

# NKM_LIBRARY: another build of the same library (A/B runs of tools/ scripts)
LIB_PATH = os.environ.get("NKM_LIBRARY") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnakama_mm.so")
_lib = None


def load_library():
    """Loads the HIP library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        _lib = capi.load_library(LIB_PATH)
        if _lib.mm_backend_name() != b"hip-gfx950":
            raise ImportError("libnakama_mm.so is not the HIP backend")
    return _lib


class LocalMatchmaker(capi.Matchmaker):
    """LocalMatchmaker (server/matchmaker.go:185) on a gfx950 device."""

    def __init__(self, **kw):
        lib = load_library()
        super().__init__(lib, **kw)
