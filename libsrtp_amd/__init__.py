"""libsrtp_amd -- Python view of libsrtp_mi355x.so (the MI355X SRTP engine).

The product is the C ABI in include/srtp_mi355x.h (a drop-in for libsrtp's
srtp_create / srtp_protect / srtp_unprotect plus a batch extension); this
module only binds it with ctypes so tests and bench.py can drive it.  There is
no Python or CPU crypto path: if the shared library (HIP kernels inside) is
missing, importing this package raises.
"""
import ctypes as C
import os

from . import srtp as _srtp_mod  # noqa: F401  (re-exported names below)
from .srtp import (  # noqa: F401
    LIB_PATH, lib, build, Status, Policy, CryptoPolicy, MasterKey,
    SSRC_SPECIFIC, SSRC_ANY_INBOUND, SSRC_ANY_OUTBOUND, Session,
    policy_setter, DeviceBatch, EventData, install_event_handler,
    session_broadcast,
)

# fail loudly at import when the HIP library is absent: there is no fallback
lib()

__all__ = [
    "LIB_PATH", "lib", "build", "Status", "Policy", "CryptoPolicy",
    "MasterKey", "Session", "policy_setter", "DeviceBatch",
    "SSRC_SPECIFIC", "SSRC_ANY_INBOUND", "SSRC_ANY_OUTBOUND",
    "session_broadcast",
]
