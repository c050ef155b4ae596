"""Seeded synthetic verify workloads: wraps tools/libfdgen.so
(OpenSSL-signed legacy Solana transactions) and assembles adversarial sets.

cfg1: single-signature txns, msg ~ U[180,220] B, 10% with one bit flipped in
      the signature, message or public key (seed 0x5EED0001).
cfg3: 1-12 signatures sharing one message, payload <= 1232 B (seed 0x5EED0003).
"""
import ctypes
import os

import numpy as np

from .ed25519 import TXN_DTYPE

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN_PATH = os.path.join(_REPO, "tools", "libfdgen.so")
_GEN = None

CFG1_SEED = 0x5EED0001
CFG3_SEED = 0x5EED0003


def gen():
    global _GEN
    if _GEN is None:
        if not os.path.exists(GEN_PATH):
            raise RuntimeError(f"workload generator not built: {GEN_PATH}")
        g = ctypes.CDLL(GEN_PATH)
        c = ctypes
        g.fdgen_txns.argtypes = [c.c_uint64, c.c_uint64, c.c_int, c.c_uint32, c.c_uint32, c.c_uint32, c.c_double,
                                 c.c_uint32, c.c_void_p, c.c_void_p, c.c_void_p, c.c_int]
        g.fdgen_txns.restype = c.c_int
        g.fdgen_sign.argtypes = [c.c_char_p, c.c_char_p, c.c_uint64, c.c_char_p, c.c_char_p]
        g.fdgen_sign.restype = c.c_int
        _GEN = g
    return _GEN


def default_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def make_txns(n, seed, multi=False, msg_lo=180, msg_hi=220, max_sigs=12, corrupt=0.10, nthreads=None):
    """Returns (arena uint8[n*stride + slack], txns TXN_DTYPE[n], modes uint8[n])."""
    stride = 1232 + 16 if multi else ((1 + 64 + max(msg_hi, 256) + 15) // 16) * 16
    arena = np.zeros(n * stride + 256, dtype=np.uint8)
    txns = np.zeros(n, dtype=TXN_DTYPE)
    modes = np.zeros(n, dtype=np.uint8)
    rc = gen().fdgen_txns(n, seed, 1 if multi else 0, msg_lo, msg_hi, max_sigs, corrupt, stride,
                          arena.ctypes.data, txns.ctypes.data, modes.ctypes.data, nthreads or default_threads())
    if rc != 0:
        raise RuntimeError(f"fdgen_txns failed: {rc}")
    return arena[: n * stride], txns, modes


def cfg1(n, seed=CFG1_SEED, nthreads=None):
    return make_txns(n, seed, multi=False, nthreads=nthreads)


def cfg3(n, seed=CFG3_SEED, nthreads=None):
    return make_txns(n, seed, multi=True, nthreads=nthreads)


def sign(prv, msg):
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    if gen().fdgen_sign(bytes(prv), bytes(msg), len(msg), pub, sig) != 0:
        raise RuntimeError("fdgen_sign failed")
    return pub.raw, sig.raw


def pack_single(records):
    """records: iterable of (msg, sig, pub) bytes -> (arena, txns) with one
    signature per transaction (sig/pub placed before the message)."""
    chunks, txns, off = [], [], 0
    for msg, sig, pub in records:
        msg, sig, pub = bytes(msg), bytes(sig), bytes(pub)
        chunks += [sig, pub, msg]
        txns.append((off + 96, len(msg), off, off + 64, 1))
        off += 96 + len(msg)
    arena = np.frombuffer(b"".join(chunks) or b"\0", dtype=np.uint8).copy()
    return arena, np.array(txns, dtype=TXN_DTYPE)
