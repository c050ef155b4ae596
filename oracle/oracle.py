"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by firedancer_amd/.
"""
import ctypes
import os

import numpy as np

SUCCESS, ERR_SIG, ERR_PUBKEY, ERR_MSG = 0, -1, -2, -3
MAP_AVX512, MAP_REF = 0, 1

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OracleTxn(ctypes.Structure):
    _fields_ = [("msg_off", ctypes.c_uint32), ("msg_sz", ctypes.c_uint32),
                ("sig_off", ctypes.c_uint32), ("pub_off", ctypes.c_uint32),
                ("sig_cnt", ctypes.c_uint32)]


TXN_DTYPE = np.dtype([("msg_off", "<u4"), ("msg_sz", "<u4"), ("sig_off", "<u4"),
                      ("pub_off", "<u4"), ("sig_cnt", "<u4")])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        u8p, c = ctypes.c_char_p, ctypes
        L.oracle_verify.argtypes = [u8p, c.c_uint64, u8p, u8p, c.c_int]
        L.oracle_verify_batch_single_msg.argtypes = [u8p, c.c_uint64, u8p, u8p, c.c_uint32, c.c_int]
        L.oracle_verify_detail.argtypes = [u8p, c.c_uint64, u8p, u8p, c.c_int,
                                           c.POINTER(c.c_int), c.POINTER(c.c_int), c.c_char_p]
        L.oracle_verify_txns.argtypes = [c.c_void_p, c.c_void_p, c.c_uint64, c.c_void_p, c.c_int, c.c_int]
        L.oracle_verify_txns_pinned.argtypes = [c.c_void_p, c.c_void_p, c.c_uint64, c.c_void_p, c.c_int, c.c_int,
                                                c.c_void_p]
        L.oracle_point_decode.argtypes = [u8p, c.c_int, c.POINTER(c.c_int), c.c_char_p]
        L.oracle_sha512.argtypes = [u8p, c.c_uint64, c.c_char_p]
        L.oracle_scalar_reduce.argtypes = [c.c_char_p, u8p]
        L.oracle_scalar_validate.argtypes = [u8p]
        L.oracle_public_from_private.argtypes = [c.c_char_p, u8p]
        L.oracle_sign.argtypes = [c.c_char_p, u8p, c.c_uint64, u8p, u8p]
        L.oracle_init()
        _LIB = L
    return _LIB


def verify(msg, sig, pub, mapping=MAP_AVX512):
    return lib().oracle_verify(bytes(msg), len(msg), bytes(sig), bytes(pub), mapping)


def verify_batch_single_msg(msg, sigs, pubs, n, mapping=MAP_AVX512):
    return lib().oracle_verify_batch_single_msg(bytes(msg), len(msg), bytes(sigs), bytes(pubs), n, mapping)


def verify_detail(msg, sig, pub, mapping=MAP_AVX512):
    p1, eq = ctypes.c_int(), ctypes.c_int()
    k = ctypes.create_string_buffer(32)
    lib().oracle_verify_detail(bytes(msg), len(msg), bytes(sig), bytes(pub), mapping,
                               ctypes.byref(p1), ctypes.byref(eq), k)
    return p1.value, eq.value, k.raw


def point_decode(enc, mapping=MAP_AVX512):
    so = ctypes.c_int()
    xy = ctypes.create_string_buffer(64)
    rc = lib().oracle_point_decode(bytes(enc), mapping, ctypes.byref(so), xy)
    return rc, so.value, (xy.raw if rc == 0 else None)


def sha512(data):
    out = ctypes.create_string_buffer(64)
    lib().oracle_sha512(bytes(data), len(data), out)
    return out.raw


def scalar_reduce(x64):
    out = ctypes.create_string_buffer(32)
    lib().oracle_scalar_reduce(out, bytes(x64))
    return out.raw


def scalar_validate(s):
    return bool(lib().oracle_scalar_validate(bytes(s)))


def public_from_private(prv):
    out = ctypes.create_string_buffer(32)
    lib().oracle_public_from_private(out, bytes(prv))
    return out.raw


def sign(msg, pub, prv):
    out = ctypes.create_string_buffer(64)
    lib().oracle_sign(out, bytes(msg), len(msg), bytes(pub), bytes(prv))
    return out.raw


def verify_txns(arena, txns, mapping=MAP_AVX512, nthreads=1, cpus=None):
    """arena: uint8 ndarray; txns: ndarray of TXN_DTYPE. Returns int8 codes.
    cpus: list of CPU ids, one pinned worker thread each (overrides nthreads)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    txns = np.ascontiguousarray(txns, dtype=TXN_DTYPE)
    codes = np.zeros(len(txns), dtype=np.int8)
    if cpus:
        cp = np.ascontiguousarray(cpus, dtype=np.int32)
        lib().oracle_verify_txns_pinned(arena.ctypes.data, txns.ctypes.data, len(txns), codes.ctypes.data,
                                        mapping, len(cp), cp.ctypes.data)
    else:
        lib().oracle_verify_txns(arena.ctypes.data, txns.ctypes.data, len(txns), codes.ctypes.data,
                                 mapping, nthreads)
    return codes
