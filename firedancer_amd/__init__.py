"""firedancer_amd -- MI355X-native batched Ed25519 signature verification for
the Firedancer verify stage.

The product is the C-ABI shared library libfd_ed25519_gpu.so
(include/fd_ed25519_gpu.h: HIP kernels for gfx950 + host engine); this
package is the Python mirror of the reference's interface over it.
"""
from .ed25519 import (ERR_MSG, ERR_PUBKEY, ERR_SIG, SUCCESS, TXN_DTYPE, VerifyEngine,  # noqa: F401
                      strerror, verify, verify_batch_single_msg)

__all__ = ["SUCCESS", "ERR_SIG", "ERR_PUBKEY", "ERR_MSG", "TXN_DTYPE", "VerifyEngine", "verify",
           "verify_batch_single_msg", "strerror"]
