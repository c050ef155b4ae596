"""Loader for the C-ABI engine library (libfd_ed25519_gpu.so).

The library is built in-tree (``make -C firedancer_amd/csrc`` or
``__graft_entry__.build()``).  There is deliberately no fallback: if the
library is missing or cannot be loaded, every entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FDGPU_LIB overrides the library path (A/B builds of kernel variants in one tree).
LIB_PATH = os.environ.get("FDGPU_LIB") or os.path.join(_HERE, "libfd_ed25519_gpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "fd_ed25519_gpu.h")

_LIB = None


class FdgpuTxn(ctypes.Structure):
    """fdgpu_txn_t (include/fd_ed25519_gpu.h)."""
    _fields_ = [("msg_off", ctypes.c_uint32), ("msg_sz", ctypes.c_uint32),
                ("sig_off", ctypes.c_uint32), ("pub_off", ctypes.c_uint32),
                ("sig_cnt", ctypes.c_uint32)]


class FdgpuCfg(ctypes.Structure):
    """fdgpu_cfg_t (include/fd_ed25519_gpu.h)."""
    _fields_ = [("max_txn", ctypes.c_uint64), ("max_sig", ctypes.c_uint64),
                ("max_arena", ctypes.c_uint64), ("ring_depth", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


def lib():
    """Load libfd_ed25519_gpu.so and declare prototypes.  Raises if absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"firedancer_amd: engine library not built: {LIB_PATH} "
                           "(run `make -C firedancer_amd/csrc`)")
    L = ctypes.CDLL(LIB_PATH)
    c = ctypes
    vp, u8p = c.c_void_p, c.c_char_p
    L.fd_ed25519_verify.argtypes = [u8p, c.c_uint64, u8p, u8p, vp]
    L.fd_ed25519_verify.restype = c.c_int
    L.fd_ed25519_verify_batch_single_msg.argtypes = [u8p, c.c_uint64, u8p, u8p, vp, c.c_uint8]
    L.fd_ed25519_verify_batch_single_msg.restype = c.c_int
    L.fd_ed25519_strerror.argtypes = [c.c_int]
    L.fd_ed25519_strerror.restype = c.c_char_p
    L.fdgpu_engine_open.argtypes = [c.c_int, c.POINTER(FdgpuCfg)]
    L.fdgpu_engine_open.restype = vp
    L.fdgpu_engine_reserve.argtypes = [vp, c.c_uint64]
    L.fdgpu_engine_reserve.restype = c.c_int
    L.fdgpu_engine_close.argtypes = [vp]
    L.fdgpu_engine_close.restype = None
    L.fdgpu_last_error.argtypes = []
    L.fdgpu_last_error.restype = c.c_char_p
    L.fdgpu_device_count.argtypes = []
    L.fdgpu_device_count.restype = c.c_int
    L.fdgpu_kernel_path.argtypes = []
    L.fdgpu_kernel_path.restype = c.c_char_p
    L.fdgpu_build_info.argtypes = []
    L.fdgpu_build_info.restype = c.c_char_p
    L.fdgpu_submit.argtypes = [vp, vp, c.c_uint64, vp, c.c_uint64]
    L.fdgpu_submit.restype = c.c_int64
    L.fdgpu_poll.argtypes = [vp, c.c_int64, vp, c.c_int]
    L.fdgpu_poll.restype = c.c_int
    L.fdgpu_stage_acquire.argtypes = [vp, c.POINTER(c.c_uint64)]
    L.fdgpu_stage_acquire.restype = vp
    L.fdgpu_stage_submit.argtypes = [vp, c.c_uint64, vp, c.c_uint64]
    L.fdgpu_stage_submit.restype = c.c_int64
    L.fdgpu_poll_keep.argtypes = [vp, c.c_int64, vp, c.c_int]
    L.fdgpu_poll_keep.restype = c.c_int
    L.fdgpu_release.argtypes = [vp, c.c_int64]
    L.fdgpu_release.restype = c.c_int
    L.fdgpu_stage_cancel.argtypes = [vp]
    L.fdgpu_stage_cancel.restype = c.c_int
    L.fdgpu_host_register.argtypes = [vp, vp, c.c_uint64]
    L.fdgpu_host_register.restype = c.c_int
    L.fdgpu_host_unregister.argtypes = [vp, vp]
    L.fdgpu_host_unregister.restype = c.c_int
    L.fdgpu_verify_device.argtypes = [vp, vp, vp, c.c_uint64, vp, c.c_uint64, vp, vp, vp]
    L.fdgpu_verify_device.restype = c.c_int
    L.fdgpu_engine_info.argtypes = [vp, c.POINTER(c.c_uint32), c.POINTER(c.c_uint32), c.POINTER(c.c_uint64)]
    L.fdgpu_engine_info.restype = c.c_int
    L.fdgpu_debug_fe_ops.argtypes = [vp, vp, c.c_uint64, vp]
    L.fdgpu_debug_decode.argtypes = [vp, vp, c.c_uint64, c.c_int, vp]
    L.fdgpu_debug_sha512.argtypes = [vp, vp, c.c_uint64, vp, c.c_uint64, vp]
    L.fdgpu_debug_hram.argtypes = [vp, vp, c.c_uint64, vp, c.c_uint64, vp]
    L.fdgpu_debug_sc_reduce.argtypes = [vp, vp, c.c_uint64, vp]
    L.fdgpu_debug_hs_split.argtypes = [vp, vp, c.c_uint64, vp]
    L.fdgpu_debug_sig_codes.argtypes = [vp, vp, c.c_uint64, vp, c.c_uint64, vp]
    L.fdgpu_dev_batch_upload.argtypes = [vp, vp, c.c_uint64, vp, c.c_uint64]
    L.fdgpu_dev_batch_upload.restype = vp
    L.fdgpu_dev_batch_verify.argtypes = [vp, vp]
    L.fdgpu_dev_batch_verify.restype = c.c_int
    L.fdgpu_dev_batch_own_queue.argtypes = [vp, vp]
    L.fdgpu_dev_batch_own_queue.restype = c.c_int
    L.fdgpu_dev_batch_codes.argtypes = [vp, vp, vp, vp]
    L.fdgpu_dev_batch_codes.restype = c.c_int
    L.fdgpu_dev_batch_upload_frags.argtypes = [vp, vp, c.c_uint64, vp, c.c_uint64]
    L.fdgpu_dev_batch_upload_frags.restype = vp
    L.fdgpu_dev_batch_txns.argtypes = [vp, vp, vp, vp]
    L.fdgpu_dev_batch_txns.restype = c.c_int
    L.fdgpu_dev_batch_time2.argtypes = [vp, vp, c.c_int] + [c.POINTER(c.c_double)] * 4
    L.fdgpu_dev_batch_time2.restype = c.c_int
    L.fdgpu_dev_batch_free.argtypes = [vp, vp]
    L.fdgpu_dev_batch_free.restype = None
    L.fdgpu_dev_batch_sig_cnt.argtypes = [vp]
    L.fdgpu_dev_batch_sig_cnt.restype = c.c_uint64
    L.fdgpu_dev_batch_device_ptrs.argtypes = [vp] + [vp] * 6
    L.fdgpu_dev_batch_device_ptrs.restype = c.c_int
    L.fdgpu_dev_batch_time.argtypes = [vp, vp, c.c_int, c.POINTER(c.c_double), c.POINTER(c.c_double),
                                       c.POINTER(c.c_double)]
    L.fdgpu_dev_batch_time.restype = c.c_int
    L.fdgpu_sync.argtypes = [vp]
    L.fdgpu_sync.restype = c.c_int
    L.fdgpu_submit_frags.argtypes = [vp, vp, c.c_uint64, vp, c.c_uint64, c.c_uint64]
    L.fdgpu_submit_frags.restype = c.c_int64
    L.fdgpu_poll_frags.argtypes = [vp, c.c_int64, vp, vp, c.c_int]
    L.fdgpu_poll_frags.restype = c.c_int
    L.fdgpu_submit_frags_io.argtypes = [vp, vp, c.c_uint64, vp, c.c_uint64, c.c_uint64, vp, c.c_uint64]
    L.fdgpu_submit_frags_io.restype = c.c_int64
    L.fdgpu_poll_frags_io.argtypes = [vp, c.c_int64, vp, vp, vp, c.c_int]
    L.fdgpu_poll_frags_io.restype = c.c_int
    L.fdgpu_debug_submit_times.argtypes = [vp, c.c_uint64]
    L.fdgpu_debug_submit_times.restype = c.c_uint64
    L.fdgpu_debug_h2d_gbps.argtypes = [vp, vp, c.c_uint64, c.c_int]
    L.fdgpu_debug_h2d_gbps.restype = c.c_double
    L.fdgpu_frag_out_cap.argtypes = [c.c_uint32]
    L.fdgpu_frag_out_cap.restype = c.c_uint32
    L.fdgpu_ed25519_verify.argtypes = [u8p, c.c_uint64, u8p, u8p]
    L.fdgpu_ed25519_verify.restype = c.c_int
    L.fdgpu_ed25519_verify_batch_single_msg.argtypes = [u8p, c.c_uint64, u8p, u8p, c.c_uint8]
    L.fdgpu_ed25519_verify_batch_single_msg.restype = c.c_int
    L.fdgpu_sync_stats.argtypes = [c.POINTER(c.c_uint64)] * 3
    L.fdgpu_sync_stats.restype = None
    L.fdgpu_sync_errors.argtypes = []
    L.fdgpu_sync_errors.restype = c.c_uint64
    for fn in ("fdgpu_debug_fe_ops", "fdgpu_debug_decode", "fdgpu_debug_sha512", "fdgpu_debug_hram",
               "fdgpu_debug_sc_reduce", "fdgpu_debug_hs_split", "fdgpu_debug_sig_codes"):
        getattr(L, fn).restype = c.c_int
    _LIB = L
    return L


def header_functions():
    """Names of the functions declared by include/fd_ed25519_gpu.h."""
    import re
    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \t\*]*?\b(fd\w+)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if not n.startswith("FD_")))


def build_info():
    """The loaded library's build switches (fdgpu_build_info) as a dict;
    "product" is 1 iff every one is at the shipped default."""
    import json
    return json.loads(lib().fdgpu_build_info().decode())


def require_product_build(allow_ab=False):
    """Raise unless the loaded library is the product build (every A/B and
    diagnostic switch off).  allow_ab: an A/B run says so and is let through;
    the returned dict goes into its record either way."""
    info = build_info()
    if not info.get("product") and not allow_ab:
        raise RuntimeError(f"firedancer_amd: {LIB_PATH} is not the product build: {info} "
                           "(rebuild with `make -C firedancer_amd/csrc`, or pass the A/B flag)")
    return info


def last_error():
    return lib().fdgpu_last_error().decode()
