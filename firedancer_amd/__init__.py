"""firedancer_amd -- MI355X-native ed25519 batch verification behind the
reference's fd_ed25519_verify API (lijunwangs/firedancer src/ballet/ed25519).

The product is firedancer_amd/libfd_ed25519_amd.so (HIP kernels for gfx950 +
a C-ABI, include/fd_ed25519_amd.h).  This package is its Python mirror:

    from firedancer_amd import ed25519
    ed25519.verify(msg, sig, pub)            # drop-in, one signature
    eng = ed25519.Engine(device=0)           # batch engine
    err = eng.verify_soa(pub, sig, off, sz, blob)
"""
from . import ed25519  # noqa: F401
from .ed25519 import (  # noqa: F401
    FD_ED25519_SUCCESS, FD_ED25519_ERR_SIG, FD_ED25519_ERR_PUBKEY, FD_ED25519_ERR_MSG,
    Engine, verify, sign, public_from_private, strerror,
)

__all__ = ["ed25519", "Engine", "verify", "sign", "public_from_private", "strerror",
           "FD_ED25519_SUCCESS", "FD_ED25519_ERR_SIG", "FD_ED25519_ERR_PUBKEY", "FD_ED25519_ERR_MSG"]
