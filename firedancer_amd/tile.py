"""Python mirror of the verify-stage integration (libfd_verify_tile.so,
include/fd_verify_tile.h): tango links (mcache + compact dcache), tcache,
fd_hash, fd_txn_parse, the verify tile over the GPU engine(s), the dedup
tile and a line-rate frag producer.

Reference interfaces restated (names follow the reference):
  fd_frag_meta_t / fd_mcache / fd_dcache   src/tango/fd_tango_base.h:146-203,
                                           mcache/fd_mcache.h:299-322,574-601,
                                           dcache/fd_dcache.h:198-269
  fd_tcache                                src/tango/tcache/fd_tcache.h:237-404
  fd_hash                                  src/util/fd_hash.c:12-73
  fd_txn_t / fd_txn_parse                  src/ballet/txn/fd_txn.h:122-335,
                                           fd_txn_parse.c:7-243
  fd_txn_verify + verify tile              src/app/fdctl/run/tiles/fd_verify.h:45-89,
                                           fd_verify.c:36-148
  dedup tile                               src/app/fdctl/run/tiles/fd_dedup.c:89-205
The library is required: there is no Python fallback for any of it.
"""
import ctypes
import mmap
import os

import numpy as np

from . import _lib
from .ed25519 import TXN_DTYPE

_HERE = os.path.dirname(os.path.abspath(__file__))
TILE_LIB_PATH = os.environ.get("FDGPU_TILE_LIB") or os.path.join(_HERE, "libfd_verify_tile.so")
TILE_HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "fd_verify_tile.h")

CHUNK_SZ = 64
TPU_MTU = 1232
TXN_MAX_SZ = 852
TPU_DCACHE_MTU = TPU_MTU + TXN_MAX_SZ + 2
TXN_VLEGACY, TXN_V0 = 0xFF, 0x00
VERIFY_SUCCESS, VERIFY_FAILED, VERIFY_DEDUP = 0, -1, -2
LOG_PARSE_FAIL, LOG_FILTERED, LOG_LOST = 1, 2, 3
VERIFY_TCACHE_DEPTH, VERIFY_TCACHE_MAP_CNT = 16, 64

FRAG_META_DTYPE = np.dtype([("seq", "<u8"), ("sig", "<u8"), ("chunk", "<u4"), ("sz", "<u2"), ("ctl", "<u2"),
                            ("tsorig", "<u4"), ("tspub", "<u4")])
assert FRAG_META_DTYPE.itemsize == 32

_TL = None
c = ctypes
vp = c.c_void_p


class FragMeta(c.Structure):
    _fields_ = [("seq", c.c_uint64), ("sig", c.c_uint64), ("chunk", c.c_uint32), ("sz", c.c_uint16),
                ("ctl", c.c_uint16), ("tsorig", c.c_uint32), ("tspub", c.c_uint32)]


class TxnInstr(c.Structure):
    _fields_ = [("program_id", c.c_uint8), ("_padding_reserved_1", c.c_uint8), ("acct_cnt", c.c_uint16),
                ("data_sz", c.c_uint16), ("acct_off", c.c_uint16), ("data_off", c.c_uint16)]


class TxnLut(c.Structure):
    _fields_ = [("addr_off", c.c_uint16), ("writable_cnt", c.c_uint8), ("readonly_cnt", c.c_uint8),
                ("writable_off", c.c_uint16), ("readonly_off", c.c_uint16)]


class TxnHdr(c.Structure):
    _fields_ = [("transaction_version", c.c_uint8), ("signature_cnt", c.c_uint8), ("signature_off", c.c_uint16),
                ("message_off", c.c_uint16), ("readonly_signed_cnt", c.c_uint8),
                ("readonly_unsigned_cnt", c.c_uint8), ("acct_addr_cnt", c.c_uint16), ("acct_addr_off", c.c_uint16),
                ("recent_blockhash_off", c.c_uint16), ("addr_table_lookup_cnt", c.c_uint8),
                ("addr_table_adtl_writable_cnt", c.c_uint8), ("addr_table_adtl_cnt", c.c_uint8),
                ("_padding_reserved_1", c.c_uint8), ("instr_cnt", c.c_uint16)]


class ParseCounters(c.Structure):
    _fields_ = [("success_cnt", c.c_uint64), ("failure_cnt", c.c_uint64), ("failure_ring", c.c_uint64 * 32)]


SUBMIT_FN = c.CFUNCTYPE(c.c_int64, vp, vp, c.c_uint64, vp, c.c_uint64)
POLL_FN = c.CFUNCTYPE(c.c_int, vp, c.c_int64, vp, c.c_int)
SUBMIT_FRAGS_FN = c.CFUNCTYPE(c.c_int64, vp, vp, c.c_uint64, vp, c.c_uint64, c.c_uint64)
POLL_FRAGS_FN = c.CFUNCTYPE(c.c_int, vp, c.c_int64, vp, vp, c.c_int)
SUBMIT_IO_FN = c.CFUNCTYPE(c.c_int64, vp, vp, c.c_uint64, vp, c.c_uint64, c.c_uint64, vp, c.c_uint64)
POLL_IO_FN = c.CFUNCTYPE(c.c_int, vp, c.c_int64, vp, vp, vp, c.c_int)
# fdgpu_frag_io_t: a payload where it lies and its out frag's room (fdgpu_submit_frags_io)
# (link = i + 1: the in link whose mcache line of seq is re-checked after the payload is read)
FRAG_IO_DTYPE = np.dtype([("src", "<u8"), ("sz", "<u4"), ("out_off", "<u4"), ("out_cap", "<u4"), ("link", "<u4"),
                          ("seq", "<u8")])
assert FRAG_IO_DTYPE.itemsize == 32
LINK_DTYPE = np.dtype([("mcache", "<u8"), ("depth", "<u8")])   # fdgpu_link_t
CODE_LAPPED = -66
# fdgpu_frag_ex_t: a payload and the place its parsed fd_txn_t goes (fdgpu_submit_frags)
FRAG_EX_DTYPE = np.dtype([("off", "<u4"), ("sz", "<u4"), ("tr_off", "<u4"), ("tr_cap", "<u4")])
CODE_PARSE_FAIL, CODE_TRAILER_CAP = -64, -65


class Verifier(c.Structure):
    """fdgpu_verifier_t: submit/poll, plus the optional zero-copy staging
    hooks (left NULL by PyVerifier; set by the GPU dispatcher)."""
    _fields_ = [("ctx", vp), ("submit", SUBMIT_FN), ("poll", POLL_FN), ("stage", vp), ("submit_staged", vp),
                ("poll_keep", vp), ("release", vp), ("stage_cancel", vp), ("submit_frags", SUBMIT_FRAGS_FN),
                ("poll_frags", POLL_FRAGS_FN), ("submit_io", SUBMIT_IO_FN), ("poll_io", POLL_IO_FN)]


class VTileCfg(c.Structure):
    _fields_ = [("in_mcache", vp), ("in_depth", c.c_uint64), ("in_seq0", c.c_uint64), ("in_base", vp),
                ("in_chunk0", c.c_uint64), ("in_wmark", c.c_uint64),
                ("out_mcache", vp), ("out_depth", c.c_uint64), ("out_seq0", c.c_uint64), ("out_base", vp),
                ("out_chunk0", c.c_uint64), ("out_wmark", c.c_uint64), ("out_fseq", vp),
                ("round_robin_idx", c.c_uint64), ("round_robin_cnt", c.c_uint64), ("hashmap_seed", c.c_uint64),
                ("tcache_depth", c.c_uint64), ("tcache_map_cnt", c.c_uint64), ("batch_txn_max", c.c_uint32),
                ("inflight_max", c.c_uint32), ("batch_wait_ns", c.c_uint64), ("batch_sig_max", c.c_uint64)]


class VTileStats(c.Structure):
    _fields_ = [(n, c.c_uint64) for n in ("in_frags", "filtered_rr", "corrupt", "overrun", "parse_fail",
                                          "verify_failed", "dedup", "published", "batches", "sigs",
                                          "backpressure", "lat_cnt", "verify_errors", "ingest_ns", "submit_ns",
                                          "poll_ns", "no_slot_steps", "polls", "poll_done_ns",
                                          "publish_ns", "batch_fill_ns", "batch_gpu_ns", "lapped", "rescued",
                                          "submit_max_ns", "stall_max_ns", "lap_margin_min")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class DTileCfg(c.Structure):
    _fields_ = [("in_cnt", c.c_uint32), ("in_mcache", vp * 16), ("in_depth", c.c_uint64 * 16),
                ("in_seq0", c.c_uint64 * 16), ("in_base", vp * 16), ("in_chunk0", c.c_uint64 * 16),
                ("in_wmark", c.c_uint64 * 16), ("unparsed_in_cnt", c.c_uint32),
                ("out_mcache", vp), ("out_depth", c.c_uint64), ("out_seq0", c.c_uint64), ("out_base", vp),
                ("out_chunk0", c.c_uint64), ("out_wmark", c.c_uint64), ("hashmap_seed", c.c_uint64),
                ("tcache_depth", c.c_uint64), ("tcache_map_cnt", c.c_uint64), ("in_fseq", vp * 16)]


class DTileStats(c.Structure):
    _fields_ = [(n, c.c_uint64) for n in ("in_frags", "dup", "published", "overrun", "corrupt", "parse_fail",
                                          "done_ns")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


MUX_FLAG_DEFAULT, MUX_FLAG_MANUAL_PUBLISH, MUX_FLAG_COPY = 0, 1, 2
MUX_IN_MAX = 16


class MuxCfg(c.Structure):
    """fdt_mux_cfg_t (the reference mux run loop's configuration)."""
    _fields_ = [("in_cnt", c.c_uint64), ("in_mcache", vp * MUX_IN_MAX), ("in_depth", c.c_uint64 * MUX_IN_MAX),
                ("in_seq0", c.c_uint64 * MUX_IN_MAX), ("in_fseq", vp * MUX_IN_MAX),
                ("out_mcache", vp), ("out_depth", c.c_uint64), ("out_seq0", c.c_uint64), ("out_cnt", c.c_uint64),
                ("out_fseq", vp * MUX_IN_MAX), ("flags", c.c_uint64), ("burst", c.c_uint64),
                ("cr_max", c.c_uint64), ("lazy_iters", c.c_uint64), ("metrics", vp)]


HISTF_BUCKET_CNT = 16


class Histf(c.Structure):
    """fdt_histf_t (the reference's fd_histf: 16 exponential buckets)."""
    _fields_ = [("counts", c.c_uint64 * HISTF_BUCKET_CNT), ("sum", c.c_uint64),
                ("left_edge", c.c_uint64 * (HISTF_BUCKET_CNT + 1))]

    def as_dict(self):
        return {"counts": list(self.counts), "sum": self.sum, "left_edge": list(self.left_edge)}


class LinkInMetrics(c.Structure):
    """fdt_link_in_metrics_t (metrics.xml <group name="Link" linkside="in">)."""
    _fields_ = [(n, c.c_uint64) for n in ("published_count", "published_size_bytes", "filtered_count",
                                          "filtered_size_bytes", "overrun_polling_count",
                                          "overrun_polling_frag_count", "overrun_reading_count")]


MUX_HISTS = ("loop_housekeeping_duration_ticks", "loop_backpressure_duration_ticks", "loop_caught_up_duration_ticks",
             "loop_overrun_polling_duration_ticks", "loop_overrun_reading_duration_ticks",
             "loop_filter_before_fragment_duration_ticks", "loop_filter_after_fragment_duration_ticks",
             "loop_finish_duration_ticks", "fragment_filtered_size_bytes", "fragment_handled_size_bytes")


class MuxMetrics(c.Structure):
    """fdt_mux_metrics_t: the reference's Tile, Stem and Link-in metrics of a mux tile."""
    _fields_ = ([("tile_pid", c.c_uint64), ("tile_tid", c.c_uint64), ("stem_in_backpressure", c.c_uint64),
                 ("stem_backpressure_count", c.c_uint64)] + [(n, Histf) for n in MUX_HISTS] +
                [("link_in", LinkInMetrics * MUX_IN_MAX), ("tick_per_ns", c.c_double),
                 ("housekeeping_cnt", c.c_uint64)])

    def as_dict(self, in_cnt=MUX_IN_MAX):
        d = {n: getattr(self, n) for n in ("tile_pid", "tile_tid", "stem_in_backpressure", "stem_backpressure_count",
                                           "tick_per_ns", "housekeeping_cnt")}
        d.update({n: getattr(self, n).as_dict() for n in MUX_HISTS})
        d["link_in"] = [{n: getattr(self.link_in[i], n) for n, _ in LinkInMetrics._fields_} for i in range(in_cnt)]
        return d


class MuxCallbacks(c.Structure):
    """fdt_mux_callbacks_t (fd_mux_callbacks_t, fd_mux.h:288-299)."""
    _fields_ = [(n, vp) for n in ("during_housekeeping", "before_credit", "after_credit", "before_frag",
                                  "during_frag", "after_frag", "metrics_write")]


class MuxStats(c.Structure):
    _fields_ = [(n, c.c_uint64) for n in ("in_frags", "filtered_before", "filtered_after", "overrun_polling",
                                          "overrun_reading", "backpressure", "published", "loops")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class VMuxCfg(c.Structure):
    """fdgpu_vmux_cfg_t (the verify tile as mux callbacks)."""
    _fields_ = [("in_cnt", c.c_uint64), ("in_base", vp * MUX_IN_MAX), ("in_chunk0", c.c_uint64 * MUX_IN_MAX),
                ("in_wmark", c.c_uint64 * MUX_IN_MAX), ("out_base", vp), ("out_chunk0", c.c_uint64),
                ("out_wmark", c.c_uint64), ("cr_max", c.c_uint64), ("round_robin_idx", c.c_uint64),
                ("round_robin_cnt", c.c_uint64), ("hashmap_seed", c.c_uint64), ("tcache_depth", c.c_uint64),
                ("tcache_map_cnt", c.c_uint64), ("batch_txn_max", c.c_uint32), ("inflight_max", c.c_uint32),
                ("batch_wait_ns", c.c_uint64), ("batch_sig_max", c.c_uint64), ("batch_bytes_max", c.c_uint64),
                ("gpu_parse", c.c_uint32), ("_pad", c.c_uint32), ("in_mcache", vp * MUX_IN_MAX),
                ("in_depth", c.c_uint64 * MUX_IN_MAX), ("lap_span_max", c.c_uint64), ("lap_margin", c.c_uint64)]


class LinkT(c.Structure):
    _fields_ = [("mcache", vp), ("depth", c.c_uint64), ("seq0", c.c_uint64), ("mtu", c.c_uint64),
                ("base", vp), ("chunk0", c.c_uint64), ("wmark", c.c_uint64), ("fseq", vp)]


def lib():
    """Load libfd_verify_tile.so (and through it libfd_ed25519_gpu.so). Raises if absent."""
    global _TL
    if _TL is not None:
        return _TL
    if not os.path.exists(TILE_LIB_PATH):
        raise RuntimeError(f"firedancer_amd: tile library not built: {TILE_LIB_PATH} "
                           "(run `make -C firedancer_amd/csrc`)")
    _lib.lib()      # the engine library first (the tile library links it)
    L = ctypes.CDLL(TILE_LIB_PATH)
    u64, i64 = c.c_uint64, c.c_int64
    sig = {
        "fdt_frag_meta_ctl": (u64, [u64, c.c_int, c.c_int, c.c_int]),
        "fdt_mcache_init": (None, [vp, u64, u64]),
        "fdt_mcache_publish": (None, [vp, u64, u64, u64, u64, u64, u64, u64, u64]),
        "fdt_mcache_poll": (c.c_int, [vp, u64, u64, vp, c.POINTER(u64)]),
        "fdt_mcache_query": (u64, [vp, u64, u64]),
        "fdt_dcache_chunk_mtu": (u64, [u64]),
        "fdt_dcache_data_sz": (u64, [u64, u64]),
        "fdt_dcache_wmark": (u64, [u64, u64, u64]),
        "fdt_dcache_compact_next": (u64, [u64, u64, u64, u64]),
        "fdt_tcache_map_cnt_default": (u64, [u64]),
        "fdt_tcache_footprint": (u64, [u64, u64]),
        "fdt_tcache_new": (vp, [vp, u64, u64]),
        "fdt_tcache_reset": (None, [vp]),
        "fdt_tcache_query": (c.c_int, [vp, u64]),
        "fdt_tcache_insert": (c.c_int, [vp, u64]),
        "fdt_tcache_insert_many": (u64, [vp, vp, u64]),
        "fdt_hash": (u64, [u64, vp, u64]),
        "fdt_txn_footprint": (u64, [u64, u64]),
        "fdt_txn_parse": (u64, [vp, u64, vp, c.POINTER(ParseCounters)]),
        "fdt_txn_peek": (u64, [vp, u64, c.POINTER(u64)]),
        "fdt_tagring_init": (None, [vp, u64]),
        "fdt_tagring_query": (c.c_int, [vp, u64]),
        "fdt_tagring_insert": (c.c_int, [vp, u64]),
        "fdgpu_dispatch_new": (vp, [c.POINTER(vp), c.c_uint32]),
        "fdgpu_dispatch_delete": (None, [vp]),
        "fdgpu_dispatch_verifier": (Verifier, [vp]),
        "fdgpu_vtile_new": (vp, [c.POINTER(VTileCfg), Verifier]),
        "fdgpu_vtile_delete": (None, [vp]),
        "fdgpu_vtile_step": (i64, [vp]),
        "fdgpu_vtile_run": (c.c_int, [vp, u64, c.c_double]),
        "fdgpu_vtile_flush": (c.c_int, [vp]),
        "fdgpu_vtile_stats": (None, [vp, c.POINTER(VTileStats)]),
        "fdgpu_vtile_latencies": (u64, [vp, vp, u64]),
        "fdgpu_vtile_tcache": (vp, [vp]),
        "fdgpu_vtile_log_enable": (None, [vp, u64]),
        "fdgpu_vtile_log": (u64, [vp, vp, vp, u64]),
        "fdgpu_dtile_new": (vp, [c.POINTER(DTileCfg)]),
        "fdgpu_dtile_delete": (None, [vp]),
        "fdgpu_dtile_step": (i64, [vp]),
        "fdgpu_dtile_stats": (None, [vp, c.POINTER(DTileStats)]),
        "fdgpu_dtile_tcache": (vp, [vp]),
        "fdgpu_producer_start": (vp, [vp, u64, u64, vp, u64, u64, vp, vp, vp, u64, c.c_double]),
        "fdgpu_replay_verify": (c.c_int, [Verifier, vp, vp, vp, u64, u64, u64, vp]),
        "fdgpu_fec_roots_verify": (c.c_int, [Verifier, vp, vp, vp, c.c_int, u64, u64, vp]),
        "fdt_tpu_reasm_footprint": (u64, [u64, u64]),
        "fdt_tpu_reasm_new": (vp, [vp, u64, u64, u64]),
        "fdt_tpu_reasm_reset": (None, [vp]),
        "fdt_tpu_reasm_chunk0": (u64, [vp, vp]),
        "fdt_tpu_reasm_wmark": (u64, [vp, vp]),
        "fdt_tpu_reasm_prepare": (c.c_uint32, [vp, u64]),
        "fdt_tpu_reasm_append": (c.c_int, [vp, c.c_uint32, vp, u64, u64]),
        "fdt_tpu_reasm_publish": (c.c_int, [vp, c.c_uint32, vp, vp, u64, u64]),
        "fdt_tpu_reasm_cancel": (None, [vp, c.c_uint32]),
        "fdt_tpu_reasm_slot_state": (c.c_int, [vp, c.c_uint32]),
        "fdt_link_footprint": (u64, [u64, u64]),
        "fdt_link_new": (c.c_int, [vp, u64, u64, u64]),
        "fdt_link_footprint_sz": (u64, [u64, u64, u64]),
        "fdt_link_new_sz": (c.c_int, [vp, u64, u64, u64, u64]),
        "fdt_link_join": (c.c_int, [vp, c.POINTER(LinkT)]),
        "fdt_sandbox_enter": (c.c_int, [c.c_int]),
        "fdt_sandbox_engine_enter": (c.c_int, [vp, c.c_int, c.c_int]),
        "fdt_sandbox_report": (u64, [vp]),
        "fdt_sandbox_driver_fds": (c.c_int, [vp, c.c_int]),
        "fdgpu_dtile_run_sandboxed": (None, [vp, u64, u64, c.POINTER(DTileStats), c.c_int]),
        "fdgpu_producer_join": (u64, [vp, c.POINTER(c.c_double)]),
        "fdgpu_producer_done": (c.c_int, [vp]),
        "fdt_histf_init": (None, [vp, u64, u64]),
        "fdt_histf_sample": (None, [vp, u64]),
        "fdt_mux_publish": (None, [vp, u64, u64, u64, u64, u64, u64]),
        "fdt_mux_run": (c.c_int, [c.POINTER(MuxCfg), c.POINTER(MuxCallbacks), vp, c.POINTER(u64),
                                  c.POINTER(MuxStats)]),
        "fdgpu_vmux_new": (vp, [c.POINTER(VMuxCfg), Verifier]),
        "fdgpu_vmux_delete": (None, [vp]),
        "fdgpu_vmux_callbacks": (MuxCallbacks, []),
        "fdgpu_vmux_dcache_data_sz": (u64, [u64, c.c_uint32, c.c_uint32]),
        "fdgpu_vmux_stats": (None, [vp, c.POINTER(VTileStats)]),
        "fdgpu_vmux_idle": (c.c_int, [vp]),
        "fdgpu_vmux_error": (c.c_int, [vp]),
        "fdgpu_vmux_final_cnt": (u64, [vp]),
        "fdgpu_vmux_latencies": (u64, [vp, vp, u64]),
        "fdgpu_vmux_log_enable": (None, [vp, u64]),
        "fdgpu_vmux_log": (u64, [vp, vp, vp, u64]),
        "fdt_mux_metrics_snapshot": (c.c_int, [c.POINTER(MuxMetrics), c.POINTER(MuxMetrics), u64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _TL = L
    return L


def header_functions():
    import re
    text = open(TILE_HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \t\*]*?\b(fd\w+)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if not n.startswith("FD_")))


def sandbox_enter(logfile_fd=2):
    """Enters the tiles' seccomp policy in this process (irreversible; only
    write to fd 2 / logfile_fd, fsync, clock_gettime and exit remain)."""
    r = lib().fdt_sandbox_enter(logfile_fd)
    if r:
        raise OSError(-r, "fdt_sandbox_enter failed")


def device_fds():
    """This process's open device fds of the GPU driver (/dev/kfd and the DRM
    render nodes; fdt_sandbox_driver_fds), the only fds the engine policy lets
    ioctl reach."""
    buf = (c.c_int * 64)()
    n = lib().fdt_sandbox_driver_fds(buf, 64)
    if n < 0:
        raise OSError(-n, "fdt_sandbox_driver_fds failed")
    return list(buf[:n])


_SYSCALL_NAMES = {}


def _syscall_names():
    """x86-64 syscall numbers -> names (read before a sandbox is entered)."""
    if not _SYSCALL_NAMES:
        import re
        for hdr in ("/usr/include/x86_64-linux-gnu/asm/unistd_64.h", "/usr/include/asm/unistd_64.h"):
            if os.path.exists(hdr):
                for m in re.finditer(r"#define __NR_(\w+)\s+(\d+)", open(hdr).read()):
                    _SYSCALL_NAMES[int(m.group(2))] = m.group(1)
                break
    return _SYSCALL_NAMES


def engine_sandbox_enter(report=False):
    """Enters the engine process's seccomp policy for every thread of this
    process (fdt_sandbox_engine_enter; irreversible): resource-neutral
    syscalls, ioctl on the GPU driver's fds held now, threads only; anything
    else kills the process -- or, with report=True, fails with EPERM and is
    recorded for engine_sandbox_report().  Returns the device fds allowed."""
    fds = device_fds()
    _syscall_names()
    arr = (c.c_int * max(1, len(fds)))(*fds)
    r = lib().fdt_sandbox_engine_enter(arr, len(fds), int(bool(report)))
    if r:
        raise OSError(-r, "fdt_sandbox_engine_enter failed")
    return fds


def engine_sandbox_report():
    """(refused call count, sorted names of the refused syscalls) in report mode"""
    bits = (c.c_uint64 * 8)()
    n = lib().fdt_sandbox_report(bits)
    names = _syscall_names()
    return int(n), sorted(names.get(k * 64 + j, str(k * 64 + j)) for k in range(8) for j in range(64)
                          if bits[k] >> j & 1)


def _aligned(nbytes, align):
    buf = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-buf.ctypes.data) % align
    return buf[off:off + nbytes]


def _page_buf(nbytes):
    """nbytes in whole pages of their own: a buffer the GPU engines may
    register (fdgpu_host_register pins whole pages) without sharing a page
    with another buffer."""
    return _aligned((nbytes + 4095) // 4096 * 4096, 4096)[:nbytes]


HUGE_PAGE = 2 << 20
PAGES = ("4k", "thp", "shm-thp", "hugetlb")


def _smaps_huge_bytes(addr, length):
    """Bytes of [addr, addr + length) this process maps with 2 MB pages
    (AnonHugePages + ShmemPmdMapped + FilePmdMapped of the overlapping
    mappings in /proc/self/smaps, scaled to the overlap)."""
    end, tot, cur = addr + length, 0, None
    try:
        f = open("/proc/self/smaps")
    except OSError:
        return 0
    with f:
        for line in f:
            head = line.split(None, 1)[0]
            if "-" in head and not head.endswith(":"):
                lo, hi = (int(x, 16) for x in head.split("-"))
                cur = (lo, hi) if lo < end and hi > addr else None
            elif cur and head in ("AnonHugePages:", "ShmemPmdMapped:", "FilePmdMapped:"):
                kb = int(line.split()[1])
                lo, hi = cur
                ov = min(hi, end) - max(lo, addr)
                tot += kb * 1024 * ov // (hi - lo)
    return tot


def hugepage_support():
    """What this host offers for 2 MB pages (the reference's workspaces sit on
    pre-allocated huge/gigantic pages, src/disco/topo/fd_topo.c:262-278):
    anonymous THP ("thp": in-process links), shmem THP ("shm-thp": links other
    processes join) and a hugetlbfs pool ("hugetlb")."""
    def rd(p):
        try:
            return open(p).read().strip()
        except OSError:
            return ""
    sel = lambda v: v[v.index("[") + 1:v.index("]")] if "[" in v else v   # noqa: E731
    thp, shm = sel(rd("/sys/kernel/mm/transparent_hugepage/enabled")), \
        sel(rd("/sys/kernel/mm/transparent_hugepage/shmem_enabled"))
    mi = {ln.split(":")[0]: ln.split(":")[1].split()[0] for ln in rd("/proc/meminfo").splitlines() if ":" in ln}
    mounts = [ln.split()[1] for ln in rd("/proc/mounts").splitlines() if ln.split()[2:3] == ["hugetlbfs"]]
    return {"thp": thp in ("always", "madvise"), "shm-thp": shm in ("always", "within_size", "advise", "force"),
            "hugetlb": int(mi.get("HugePages_Free", 0)) > 0 and bool(mounts),
            "thp_enabled": thp, "shmem_enabled": shm, "hugetlb_free": int(mi.get("HugePages_Free", 0)),
            "hugetlbfs_mounts": mounts}


class _Region:
    """A 4096-aligned byte region for link memory, faulted in (every page
    written) before it is used, so no first touch lands in a timed run.
    pages: "4k" (anonymous / the file's pages), "thp" (anonymous memory
    madvise'd MADV_HUGEPAGE: 2 MB pages when the host allows), "shm-thp" (a
    /dev/shm file madvise'd the same: other processes can join it), "hugetlb"
    (a file on a hugetlbfs mount)."""

    def __init__(self, nbytes, path=None, pages="4k", create=True):
        if pages not in PAGES:
            raise ValueError(f"pages must be one of {PAGES}")
        if pages == "thp" and path:
            raise ValueError("anonymous THP cannot back a shared link: use shm-thp or hugetlb")
        align = HUGE_PAGE if pages != "4k" else 4096
        self.pages, self.path = pages, path
        if path:
            size = (nbytes + align - 1) // align * align
            if create:
                fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o600)
            else:
                fd = os.open(path, os.O_RDWR)
            try:
                if create:
                    os.ftruncate(fd, size)
                else:
                    size = os.fstat(fd).st_size
                self._mm = mmap.mmap(fd, size, mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0),
                                     mmap.PROT_READ | mmap.PROT_WRITE)
            finally:
                os.close(fd)
            if pages == "shm-thp":
                self._mm.madvise(mmap.MADV_HUGEPAGE)
            self.buf = np.frombuffer(self._mm, dtype=np.uint8)
            self.size = size
        else:
            size = (nbytes + align - 1) // align * align
            self._mm = mmap.mmap(-1, size + align, mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS,
                                 mmap.PROT_READ | mmap.PROT_WRITE)
            raw = np.frombuffer(self._mm, dtype=np.uint8)
            off = (-raw.ctypes.data) % align
            if pages == "thp":
                self._mm.madvise(mmap.MADV_HUGEPAGE, off, size)
            self.buf = raw[off:off + size]
            self.size = size
        if create:
            self.buf[:] = 0                       # fault every page in now (the link's producer writes them later)
        else:
            _ = int(self.buf[::4096].sum())         # joiner: map every page (MAP_POPULATE did, where it exists)

    def huge_bytes(self):
        return _smaps_huge_bytes(self.buf.ctypes.data, self.size)


# ---------------------------------------------------------------- basics

def fd_hash(seed, data):
    data = bytes(data)
    return lib().fdt_hash(seed & (2**64 - 1), data, len(data))


def frag_meta_ctl(orig, som, eom, err):
    return lib().fdt_frag_meta_ctl(orig, som, eom, err)


def dcache_compact_next(chunk, sz, chunk0, wmark):
    return lib().fdt_dcache_compact_next(chunk, sz, chunk0, wmark)


class TCache:
    """fd_tcache: ring of the last `depth` unique tags + linear-probed map."""

    def __init__(self, depth, map_cnt=0):
        L = lib()
        fp = L.fdt_tcache_footprint(depth, map_cnt)
        if not fp:
            raise ValueError("bad tcache depth / map_cnt")
        self._mem = _aligned(fp, 128)
        self._p = L.fdt_tcache_new(self._mem.ctypes.data, depth, map_cnt)
        self.depth = depth
        self.map_cnt = int(self._mem[16:24].view("<u8")[0])

    @classmethod
    def attach(cls, ptr, owner):
        self = cls.__new__(cls)
        self._mem, self._p = owner, ptr
        hdr = (c.c_uint64 * 4).from_address(ptr)
        self.depth, self.map_cnt = hdr[1], hdr[2]
        return self

    def reset(self):
        lib().fdt_tcache_reset(self._p)

    def query(self, tag):
        return bool(lib().fdt_tcache_query(self._p, tag))

    def insert(self, tag):
        """returns True if tag was a duplicate (tcache unchanged)"""
        return bool(lib().fdt_tcache_insert(self._p, tag))

    def words(self):
        n = 4 + self.depth + self.map_cnt
        return np.ctypeslib.as_array((c.c_uint64 * n).from_address(self._p)).copy()


def txn_parse(payload, counters=None):
    """fd_txn_parse: returns (footprint, raw fd_txn_t bytes) or (0, None)."""
    payload = bytes(payload)
    out = c.create_string_buffer(TXN_MAX_SZ + 16)
    sz = lib().fdt_txn_parse(payload, len(payload), out, c.byref(counters) if counters is not None else None)
    return (sz, out.raw[:sz]) if sz else (0, None)


def txn_peek(payload):
    """fdt_txn_peek: (the footprint a successful parse would have, the
    leading signature count), read from the payload's counts."""
    payload = bytes(payload)
    sc = c.c_uint64()
    fp = lib().fdt_txn_peek(payload, len(payload), c.byref(sc))
    return int(fp), int(sc.value)


def txn_decode(raw):
    """fd_txn_t bytes -> dict (header fields, instr list, address tables)."""
    hdr = TxnHdr.from_buffer_copy(raw[:c.sizeof(TxnHdr)])
    d = {n: getattr(hdr, n) for n, _ in TxnHdr._fields_}
    off = c.sizeof(TxnHdr)
    d["instr"] = []
    for _ in range(hdr.instr_cnt):
        ins = TxnInstr.from_buffer_copy(raw[off:off + 10])
        d["instr"].append({n: getattr(ins, n) for n, _ in TxnInstr._fields_})
        off += 10
    d["luts"] = []
    for _ in range(hdr.addr_table_lookup_cnt):
        lut = TxnLut.from_buffer_copy(raw[off:off + 8])
        d["luts"].append({n: getattr(lut, n) for n, _ in TxnLut._fields_})
        off += 8
    return d


# ---------------------------------------------------------------- links

class Link:
    """One tango link: an mcache of `depth` frag metas and a compact dcache
    sized for `depth` frags of up to `mtu` bytes (chunk 0 = dcache start)."""

    def __init__(self, depth, mtu, seq0=0, data_sz=None, pages=None):
        """pages: None (numpy pages, faulted in on first use), or "4k" / "thp":
        the mcache and dcache in one region faulted in before use
        (_Region), on 2 MB pages for "thp" where the host allows."""
        L = lib()
        if depth & (depth - 1):
            raise ValueError("depth must be a power of 2")
        self.depth, self.mtu, self.seq0 = depth, mtu, seq0
        data_sz = data_sz or L.fdt_dcache_data_sz(mtu, depth)   # explicit: a dcache sized by its producer
        data_sz = (data_sz + CHUNK_SZ - 1) // CHUNK_SZ * CHUNK_SZ
        if pages:
            mo = (depth * 32 + 4095) // 4096 * 4096
            self._mem = _Region(mo + data_sz, pages=pages)
            self._region = self._mem.buf                       # one region: the engines register it whole
            self.mcache = self._region[:depth * 32].view(FRAG_META_DTYPE)
            self.dcache = self._region[mo:mo + data_sz]
        else:
            self.mcache = _page_buf(depth * 32).view(FRAG_META_DTYPE)
            self.dcache = _page_buf(data_sz)
        self.chunk0 = 0
        self.chunk1 = data_sz // CHUNK_SZ
        self.wmark = L.fdt_dcache_wmark(self.chunk0, self.chunk1, mtu)
        self.fseq = np.zeros(1, dtype=np.uint64)
        self.fseq[0] = seq0
        L.fdt_mcache_init(self.mcache.ctypes.data, depth, seq0)
        self._pub_seq, self._pub_chunk = seq0, 0

    @classmethod
    def shm_create(cls, path, depth, mtu, seq0=0, data_sz=0, pages="4k"):
        """A link formatted in a shared-memory file (fdt_link_new_sz),
        joinable by other processes with shm_join(path): the engine process
        and the sandboxed tiles share links this way (fd_wksp's role).  The
        whole region is faulted in before it is formatted (pages "4k", or
        "shm-thp" / "hugetlb" for 2 MB pages where the host offers them:
        hugepage_support())."""
        fp = lib().fdt_link_footprint_sz(depth, mtu, data_sz)
        if not fp:
            raise ValueError("bad link parameters")
        mem = _Region(fp, path=path, pages=pages)
        if lib().fdt_link_new_sz(mem.buf.ctypes.data, depth, mtu, seq0, data_sz):
            raise RuntimeError("fdt_link_new failed")
        return cls._from_region(mem, mem.buf)

    @classmethod
    def shm_join(cls, path, pages="4k"):
        """Joins a link another process formatted (every page mapped now)."""
        mem = _Region(0, path=path, pages=pages if pages != "thp" else "4k", create=False)
        return cls._from_region(mem, mem.buf)

    def huge_bytes(self):
        """Bytes of this link's memory on 2 MB pages in this process."""
        mem = getattr(self, "_mem", None) or getattr(self, "_mm", None)
        return mem.huge_bytes() if isinstance(mem, _Region) else 0

    @classmethod
    def _from_region(cls, mm, region):
        v = LinkT()
        if lib().fdt_link_join(region.ctypes.data, c.byref(v)):
            raise RuntimeError("not a formatted link region")
        base = region.ctypes.data
        self = cls.__new__(cls)
        self._mm, self._region = mm, region
        self.depth, self.mtu, self.seq0 = v.depth, v.mtu, v.seq0
        mo, do, fo = v.mcache - base, v.base - base, v.fseq - base
        self.mcache = region[mo:mo + v.depth * 32].view(FRAG_META_DTYPE)
        self.dcache = region[do:]
        self.fseq = region[fo:fo + 8].view(np.uint64)
        self.chunk0, self.wmark = v.chunk0, v.wmark
        self.chunk1 = len(self.dcache) // CHUNK_SZ
        self._pub_seq, self._pub_chunk = v.seq0, v.chunk0
        return self

    @property
    def mcache_ptr(self):
        return self.mcache.ctypes.data

    @property
    def base_ptr(self):
        return self.dcache.ctypes.data

    def publish(self, payload, sig=0, ctl=None):
        """Producer side (single-threaded): payload into the dcache, meta into the mcache."""
        L = lib()
        payload = bytes(payload)
        ch = self._pub_chunk
        self.dcache[ch * CHUNK_SZ: ch * CHUNK_SZ + len(payload)] = np.frombuffer(payload, dtype=np.uint8)
        ctl = frag_meta_ctl(0, 1, 1, 0) if ctl is None else ctl
        L.fdt_mcache_publish(self.mcache_ptr, self.depth, self._pub_seq, sig, ch, len(payload), ctl, 0, 0)
        self._pub_seq += 1
        self._pub_chunk = L.fdt_dcache_compact_next(ch, len(payload), self.chunk0, self.wmark)
        return self._pub_seq - 1

    def poll(self, seq):
        """Consumer side: (status, meta dict or None, seq_found)."""
        m = FragMeta()
        found = c.c_uint64()
        rc = lib().fdt_mcache_poll(self.mcache_ptr, self.depth, seq, c.byref(m), c.byref(found))
        meta = {n: getattr(m, n) for n, _ in FragMeta._fields_} if rc == 1 else None
        return rc, meta, found.value

    def payload(self, meta):
        o = meta["chunk"] * CHUNK_SZ
        return bytes(self.dcache[o:o + meta["sz"]])

    def drain(self, seq=None, max_frags=1 << 30):
        """Reads frags from `seq` (default seq0) until none is available: list of (meta, payload)."""
        seq = self.seq0 if seq is None else seq
        out = []
        while len(out) < max_frags:
            rc, meta, found = self.poll(seq)
            if rc != 1:
                break
            out.append((meta, self.payload(meta)))
            seq += 1
        return out


REASM_SUCCESS, REASM_ERR_SZ, REASM_ERR_SKIP, REASM_ERR_STATE = 0, 1, 2, 3
REASM_FREE, REASM_BUSY, REASM_PUB = 0, 1, 2
TPU_REASM_MTU = 1280


class TpuReasm:
    """The quic -> verify link as the reference builds it: TPU stream
    reassembly slots (fdt_tpu_reasm_*, fd_tpu.h:20-246) publishing into an
    mcache.  Has the attributes VerifyTile reads from a link (mcache_ptr,
    depth, seq0, base_ptr, chunk0, wmark): base is the region start, chunk0
    the first slot's chunk, wmark per fd_verify.c:186-191."""

    def __init__(self, depth, burst, orig=0, seq0=0):
        L = lib()
        fp = L.fdt_tpu_reasm_footprint(depth, burst)
        if not fp:
            raise ValueError("bad reasm parameters")
        self.depth, self.burst, self.seq0, self.mtu = depth, burst, seq0, TPU_REASM_MTU
        self.region = _page_buf(fp)
        self.dcache = self.region                    # the payloads' region (the verify tile registers it)
        self._r = L.fdt_tpu_reasm_new(self.region.ctypes.data, depth, burst, orig)
        if not self._r:
            raise RuntimeError("fdt_tpu_reasm_new failed")
        self.mcache = _page_buf(depth * 32).view(FRAG_META_DTYPE)
        L.fdt_mcache_init(self.mcache.ctypes.data, depth, seq0)
        self.chunk0 = L.fdt_tpu_reasm_chunk0(self._r, self.base_ptr)
        self.wmark = L.fdt_tpu_reasm_wmark(self._r, self.base_ptr)
        self.fseq = np.zeros(1, dtype=np.uint64)
        self.next_seq = seq0

    @property
    def mcache_ptr(self):
        return self.mcache.ctypes.data

    @property
    def base_ptr(self):
        return self.region.ctypes.data

    def prepare(self, tsorig=0):
        return lib().fdt_tpu_reasm_prepare(self._r, tsorig)

    def append(self, slot, data, off):
        data = bytes(data)
        return lib().fdt_tpu_reasm_append(self._r, slot, data, len(data), off)

    def publish(self, slot, tspub=0):
        rc = lib().fdt_tpu_reasm_publish(self._r, slot, self.mcache_ptr, self.base_ptr, self.next_seq, tspub)
        if rc == REASM_SUCCESS:
            self.next_seq += 1
        return rc

    def cancel(self, slot):
        lib().fdt_tpu_reasm_cancel(self._r, slot)

    def state(self, slot):
        return lib().fdt_tpu_reasm_slot_state(self._r, slot)

    def poll(self, seq):
        m = FragMeta()
        found = c.c_uint64()
        rc = lib().fdt_mcache_poll(self.mcache_ptr, self.depth, seq, c.byref(m), c.byref(found))
        meta = {n: getattr(m, n) for n, _ in FragMeta._fields_} if rc == 1 else None
        return rc, meta, found.value

    def payload(self, meta):
        o = meta["chunk"] * CHUNK_SZ
        return bytes(self.region[o:o + meta["sz"]])


def split_verify_output(frag_payload):
    """[payload][pad][fd_txn_t][u16 payload_sz] -> (payload, fd_txn_t bytes)."""
    b = bytes(frag_payload)
    psz = int.from_bytes(b[-2:], "little")
    toff = (psz + 1) & ~1
    return b[:psz], b[toff:-2]


# -------------------------------------------------------------- verifiers

class PyVerifier:
    """A verifier backed by a Python callable fn(arena uint8[], txns TXN_DTYPE[]) -> int8 codes.
    For tests of the tile logic without a GPU (the callable is the test's
    checker); `lag` makes each batch report PENDING for that many polls
    (`lag_fn(ticket)`, when given, sets it per batch: batches then complete
    out of order, as the engine's do on their own streams; `done` records
    the order the batches completed in)."""

    def __init__(self, fn, slots=2, lag=0, lag_fn=None, read_at_submit=False):
        self.fn, self.slots, self.lag, self.lag_fn = fn, slots, lag, lag_fn
        self.read_at_submit = read_at_submit          # gathered batches: payloads read at submit, not at the poll
        self.results, self.polls, self.next = {}, {}, 0
        self.batches, self.done, self.lags = [], [], {}

        def submit(ctx, arena, arena_sz, txns, n):
            if len(self.results) >= self.slots:
                return -12                                    # FDGPU_ERR_FULL
            a = np.ctypeslib.as_array((c.c_uint8 * max(arena_sz, 1)).from_address(arena))[:arena_sz].copy()
            t = np.frombuffer((c.c_uint8 * (20 * n)).from_address(txns), dtype=TXN_DTYPE).copy() if n else \
                np.zeros(0, dtype=TXN_DTYPE)
            self.batches.append(len(t))
            k = self.next
            self.next += 1
            self.results[k] = np.asarray(self.fn(a, t), dtype=np.int8)
            self.polls[k] = 0
            if self.lag_fn is not None:
                self.lags[k] = self.lag_fn(k)
            return k

        def poll(ctx, ticket, codes, blocking):
            if ticket not in self.results:
                return -13
            if not blocking and self.polls[ticket] < self.lags.get(ticket, self.lag):
                self.polls[ticket] += 1
                return 1                                      # FDGPU_PENDING
            r = self.results.pop(ticket)
            self.polls.pop(ticket)
            self.done.append(ticket)
            if len(r):
                c.memmove(codes, r.ctypes.data, len(r))
            return 0

        def submit_frags(ctx, arena, arena_sz, frags, n, trailer_sz):
            # the GPU engine's fdgpu_submit_frags on the host: fd_txn_parse of
            # every payload, codes from fn over the parsed txns, trailers
            # packed at the caller's reserved places
            if len(self.results) >= self.slots:
                return -12
            a = np.ctypeslib.as_array((c.c_uint8 * max(arena_sz, 1)).from_address(arena))[:arena_sz].copy()
            fx = np.frombuffer((c.c_uint8 * (16 * n)).from_address(frags), dtype=FRAG_EX_DTYPE).copy() if n else \
                np.zeros(0, dtype=FRAG_EX_DTYPE)
            codes = np.zeros(max(n, 1), dtype=np.int8)
            tr = bytearray(trailer_sz)
            txns, idx = [], []
            for i, f in enumerate(fx):
                off, sz = int(f["off"]), int(f["sz"])
                fp, raw = txn_parse(a[off:off + sz].tobytes())
                if not fp:
                    codes[i] = CODE_PARSE_FAIL
                    continue
                if fp != int(f["tr_cap"]):
                    codes[i] = CODE_TRAILER_CAP
                    continue
                tr[int(f["tr_off"]):int(f["tr_off"]) + fp] = raw
                h = txn_decode(raw)
                txns.append((off + h["message_off"], sz - h["message_off"], off + h["signature_off"],
                             off + h["acct_addr_off"], h["signature_cnt"]))
                idx.append(i)
            if txns:
                codes[idx] = np.asarray(self.fn(a, np.array(txns, dtype=TXN_DTYPE)), dtype=np.int8)
            self.batches.append(n)
            k = self.next
            self.next += 1
            self.results[k] = codes[:n]
            self.trailers[k] = bytes(tr)
            self.polls[k] = 0
            if self.lag_fn is not None:
                self.lags[k] = self.lag_fn(k)
            return k

        def poll_frags(ctx, ticket, codes, trailers, blocking):
            if ticket not in self.trailers:
                return -13
            rc = poll(ctx, ticket, codes, blocking)
            if rc == 0:
                t = self.trailers.pop(ticket)
                if t:
                    c.memmove(trailers, t, len(t))
            return rc

        def submit_io(ctx, frags, n, out, out_sz, seed, links, link_cnt):
            # fdgpu_submit_frags_io on the host: each payload read where it
            # lies -- late, when the batch completes (the first poll that
            # returns it), as the device reads it some time after submit --
            # its in-mcache line re-checked after the read, parsed, tagged,
            # its out frag written at its reserved place
            if len(self.results) >= self.slots:
                return -12
            fio = np.frombuffer((c.c_uint8 * (32 * n)).from_address(frags), dtype=FRAG_IO_DTYPE).copy() if n else \
                np.zeros(0, dtype=FRAG_IO_DTYPE)
            lk = np.frombuffer((c.c_uint8 * (16 * link_cnt)).from_address(links), dtype=LINK_DTYPE).copy() \
                if link_cnt else np.zeros(0, dtype=LINK_DTYPE)

            def work():
                codes = np.zeros(max(n, 1), dtype=np.int8)
                tags = np.zeros(max(n, 1), dtype=np.uint64)
                osz = np.zeros(max(n, 1), dtype=np.uint16)
                arena, txns, idx = bytearray(), [], []
                for i, f in enumerate(fio):
                    sz = int(f["sz"])
                    p = c.string_at(int(f["src"]), sz)
                    if int(f["link"]):
                        ln = lk[int(f["link"]) - 1]
                        line = int(ln["mcache"]) + (int(f["seq"]) & (int(ln["depth"]) - 1)) * 32
                        if c.c_uint64.from_address(line).value != int(f["seq"]):
                            codes[i] = CODE_LAPPED
                            continue
                    fp, raw = txn_parse(p)
                    if not fp:
                        codes[i] = CODE_PARSE_FAIL
                        continue
                    h = txn_decode(raw)
                    tags[i] = fd_hash(seed, p[h["signature_off"]:h["signature_off"] + 64])
                    toff = (sz + 1) & ~1
                    frag = p + b"\0" * (toff - sz) + raw + sz.to_bytes(2, "little")
                    if len(frag) > int(f["out_cap"]):
                        codes[i] = CODE_TRAILER_CAP
                        continue
                    c.memmove(out + int(f["out_off"]), frag, len(frag))
                    osz[i] = len(frag)
                    off = len(arena)
                    arena += p
                    txns.append((off + h["message_off"], sz - h["message_off"], off + h["signature_off"],
                                 off + h["acct_addr_off"], h["signature_cnt"]))
                    idx.append(i)
                if txns:
                    codes[idx] = np.asarray(self.fn(np.frombuffer(bytes(arena), dtype=np.uint8),
                                                    np.array(txns, dtype=TXN_DTYPE)), dtype=np.int8)
                return codes[:n], tags[:n], osz[:n]

            self.batches.append(n)
            k = self.next
            self.next += 1
            self.results[k] = None
            if self.read_at_submit:
                done = work()
                self.io[k] = lambda: done
            else:
                self.io[k] = work
            self.polls[k] = 0
            if self.lag_fn is not None:
                self.lags[k] = self.lag_fn(k)
            return k

        def poll_io(ctx, ticket, codes, tags, out_szs, blocking):
            if ticket not in self.io:
                return -13
            if not blocking and self.polls[ticket] < self.lags.get(ticket, self.lag):
                self.polls[ticket] += 1
                return 1                                      # FDGPU_PENDING
            r, t, o = self.io.pop(ticket)()
            self.results.pop(ticket)
            self.polls.pop(ticket)
            self.done.append(ticket)
            if len(r):
                c.memmove(codes, r.ctypes.data, len(r))
                c.memmove(tags, t.ctypes.data, 8 * len(t))
                c.memmove(out_szs, o.ctypes.data, 2 * len(o))
            return 0

        self.trailers, self.io = {}, {}
        self._submit_io, self._poll_io = SUBMIT_IO_FN(submit_io), POLL_IO_FN(poll_io)
        self._submit, self._poll = SUBMIT_FN(submit), POLL_FN(poll)
        self._submit_frags, self._poll_frags = SUBMIT_FRAGS_FN(submit_frags), POLL_FRAGS_FN(poll_frags)
        self.struct = Verifier(None, self._submit, self._poll)
        self.struct.submit_frags, self.struct.poll_frags = self._submit_frags, self._poll_frags
        self.struct.submit_io, self.struct.poll_io = self._submit_io, self._poll_io


class EngineVerifier:
    """Round-robin over GPU engines (fdgpu_dispatch; one engine per GPU)."""

    def __init__(self, engines):
        L = lib()
        self.engines = list(engines)
        self.sig_max = min(e.max_sig for e in self.engines)     # signatures per batch every engine accepts
        self.arena_max = min(e.max_arena for e in self.engines)
        arr = (vp * len(self.engines))(*[e._h for e in self.engines])
        self._d = L.fdgpu_dispatch_new(arr, len(self.engines))
        if not self._d:
            raise RuntimeError("fdgpu_dispatch_new failed")
        self.struct = L.fdgpu_dispatch_verifier(self._d)

    def close(self):
        if self._d:
            lib().fdgpu_dispatch_delete(self._d)
            self._d = None


# ------------------------------------------------------- other callers

REPLAY_PARSE_FAIL = 1


def replay_verify(verifier, payloads, batch_txn_max=4096, batch_bytes_max=4096 * 1232):
    """fd_executor_txn_verify over a block's raw txns, batched
    (fdgpu_replay_verify): one fd_ed25519 code per payload, or
    REPLAY_PARSE_FAIL."""
    n = len(payloads)
    sizes = np.array([len(p) for p in payloads], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(payloads) + b"\0", dtype=np.uint8)
    codes = np.zeros(max(n, 1), dtype=np.int8)
    r = lib().fdgpu_replay_verify(verifier.struct, arena.ctypes.data, offs.ctypes.data, sizes.ctypes.data, n,
                                  batch_txn_max, batch_bytes_max, codes.ctypes.data)
    if r:
        raise RuntimeError(f"fdgpu_replay_verify failed: {r}")
    return codes[:n]


def fec_roots_verify(verifier, roots, sigs, pubkeys, batch_max=65536):
    """fd_ed25519_verify(root, 32, sig, leader_pubkey) per FEC set
    (fdgpu_fec_roots_verify); pubkeys: one 32-B key (shared) or one per set."""
    roots = np.ascontiguousarray(np.frombuffer(bytes(roots), dtype=np.uint8))
    sigs = np.ascontiguousarray(np.frombuffer(bytes(sigs), dtype=np.uint8))
    pubkeys = np.ascontiguousarray(np.frombuffer(bytes(pubkeys), dtype=np.uint8))
    n = len(roots) // 32
    if len(sigs) != 64 * n or len(pubkeys) not in (32, 32 * n):
        raise ValueError("roots/sigs/pubkeys sizes disagree")
    codes = np.zeros(max(n, 1), dtype=np.int8)
    r = lib().fdgpu_fec_roots_verify(verifier.struct, roots.ctypes.data, sigs.ctypes.data, pubkeys.ctypes.data,
                                     1 if len(pubkeys) == 32 and n != 1 else 0, n, batch_max, codes.ctypes.data)
    if r:
        raise RuntimeError(f"fdgpu_fec_roots_verify failed: {r}")
    return codes[:n]


# ------------------------------------------------------------------ tiles

class VerifyTile:
    """The verify tile (fd_verify.c) over a verifier (GPU engines in the product)."""

    def __init__(self, in_link, out_link, verifier, hashmap_seed=0x5EEDF00D, batch_txn_max=4096, inflight_max=2,
                 batch_wait_us=200, round_robin_idx=0, round_robin_cnt=1, tcache_depth=0, tcache_map_cnt=0,
                 flow_control=False, log_max=0, batch_sig_max=0):
        L = lib()
        self.verifier, self.in_link, self.out_link = verifier, in_link, out_link
        cfg = VTileCfg()
        cfg.in_mcache, cfg.in_depth, cfg.in_seq0 = in_link.mcache_ptr, in_link.depth, in_link.seq0
        cfg.in_base, cfg.in_chunk0, cfg.in_wmark = in_link.base_ptr, in_link.chunk0, in_link.wmark
        cfg.out_mcache, cfg.out_depth, cfg.out_seq0 = out_link.mcache_ptr, out_link.depth, out_link.seq0
        cfg.out_base, cfg.out_chunk0, cfg.out_wmark = out_link.base_ptr, out_link.chunk0, out_link.wmark
        cfg.out_fseq = out_link.fseq.ctypes.data if flow_control else None
        cfg.round_robin_idx, cfg.round_robin_cnt = round_robin_idx, round_robin_cnt
        cfg.hashmap_seed = hashmap_seed
        cfg.tcache_depth, cfg.tcache_map_cnt = tcache_depth, tcache_map_cnt
        cfg.batch_txn_max, cfg.inflight_max = batch_txn_max, inflight_max
        cfg.batch_wait_ns = int(batch_wait_us * 1000)
        cfg.batch_sig_max = batch_sig_max or getattr(verifier, "sig_max", 0)
        self.cfg = cfg
        self._t = L.fdgpu_vtile_new(c.byref(cfg), verifier.struct)
        if not self._t:
            raise RuntimeError("fdgpu_vtile_new: bad configuration")
        if log_max:
            L.fdgpu_vtile_log_enable(self._t, log_max)
        self.tcache = TCache.attach(L.fdgpu_vtile_tcache(self._t), self)

    def step(self):
        r = lib().fdgpu_vtile_step(self._t)
        if r < 0:
            raise RuntimeError(f"verify tile step failed: {r} ({_lib.last_error()})")
        return r

    def run(self, in_frags, timeout_s=60.0):
        r = lib().fdgpu_vtile_run(self._t, in_frags, timeout_s)
        if r < 0:
            raise RuntimeError(f"verify tile run failed: {r} ({_lib.last_error()})")

    def flush(self):
        r = lib().fdgpu_vtile_flush(self._t)
        if r < 0:
            raise RuntimeError(f"verify tile flush failed: {r}")

    def stats(self):
        s = VTileStats()
        lib().fdgpu_vtile_stats(self._t, c.byref(s))
        return s.as_dict()

    def latencies_ns(self):
        n = self.stats()["lat_cnt"]
        out = np.zeros(max(n, 1), dtype=np.uint64)
        n = lib().fdgpu_vtile_latencies(self._t, out.ctypes.data, n)
        return out[:n]

    def log(self, max_entries=1 << 24):
        seqs = np.zeros(max_entries, dtype=np.uint64)
        codes = np.zeros(max_entries, dtype=np.int8)
        n = lib().fdgpu_vtile_log(self._t, seqs.ctypes.data, codes.ctypes.data, max_entries)
        order = np.argsort(seqs[:n], kind="stable")
        return seqs[:n][order], codes[:n][order]

    def close(self):
        if self._t:
            lib().fdgpu_vtile_delete(self._t)
            self._t = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class VerifyMuxTile:
    """The verify tile as the reference's mux callbacks (fdgpu_vmux, run by
    fdt_mux_run with FD_MUX_FLAG_COPY | FD_MUX_FLAG_MANUAL_PUBLISH, burst 1;
    fd_verify.c:232-246) on its own thread.  Frags are copied into the out
    link's dcache (registered with every engine of an EngineVerifier, so the
    GPU reads the batch from there with no staging copy) and published from
    there in order.  `flow_control`: the out link's fseq is the mux's one
    reliable consumer (otherwise published frags count as consumed)."""

    def __init__(self, in_links, out_link, verifier, hashmap_seed=0x5EEDF00D, batch_txn_max=4096, inflight_max=2,
                 batch_wait_us=200, round_robin_idx=0, round_robin_cnt=1, cr_max=0, log_max=0, batch_sig_max=0,
                 batch_bytes_max=0, lazy_iters=16, flow_control=False, register=True, gpu_parse=False,
                 lap_span_max=0, lap_margin=0, metrics=False):
        import threading
        L = lib()
        in_links = list(in_links) if isinstance(in_links, (list, tuple)) else [in_links]
        self.verifier, self.in_links, self.out_link = verifier, in_links, out_link
        self.cr_max = cr_max or out_link.depth
        vc = VMuxCfg()
        vc.in_cnt = len(in_links)
        for i, ln in enumerate(in_links):
            vc.in_base[i], vc.in_chunk0[i], vc.in_wmark[i] = ln.base_ptr, ln.chunk0, ln.wmark
        vc.out_base, vc.out_chunk0, vc.out_wmark = out_link.base_ptr, out_link.chunk0, out_link.wmark
        vc.cr_max, vc.round_robin_idx, vc.round_robin_cnt = self.cr_max, round_robin_idx, round_robin_cnt
        vc.hashmap_seed, vc.batch_txn_max, vc.inflight_max = hashmap_seed, batch_txn_max, inflight_max
        vc.batch_wait_ns = int(batch_wait_us * 1000)
        vc.batch_sig_max = batch_sig_max or getattr(verifier, "sig_max", 0)
        vc.batch_bytes_max = batch_bytes_max or getattr(verifier, "arena_max", 0)
        vc.gpu_parse = int(gpu_parse)            # False/True/0/1/2 (2: the GPU also gathers the payloads)
        for i, ln in enumerate(in_links):
            vc.in_mcache[i], vc.in_depth[i] = ln.mcache_ptr, ln.depth
        vc.lap_span_max, vc.lap_margin = lap_span_max, lap_margin   # 0: depth / 2, depth / 4; LAP_OFF: off
        self.vcfg = vc
        self._t = L.fdgpu_vmux_new(c.byref(vc), verifier.struct)
        if not self._t:
            raise RuntimeError("fdgpu_vmux_new: bad configuration")
        if log_max:
            L.fdgpu_vmux_log_enable(self._t, log_max)
        mc = MuxCfg()
        mc.in_cnt = len(in_links)
        for i, ln in enumerate(in_links):
            mc.in_mcache[i], mc.in_depth[i], mc.in_seq0[i] = ln.mcache_ptr, ln.depth, ln.seq0
        mc.out_mcache, mc.out_depth, mc.out_seq0 = out_link.mcache_ptr, out_link.depth, out_link.seq0
        if flow_control:
            mc.out_cnt, mc.out_fseq[0] = 1, out_link.fseq.ctypes.data
        mc.flags, mc.burst, mc.cr_max, mc.lazy_iters = MUX_FLAG_COPY | MUX_FLAG_MANUAL_PUBLISH, 1, self.cr_max, lazy_iters
        self._metrics = MuxMetrics() if metrics else None   # the reference's link / stem metrics, written by the loop
        mc.metrics = c.addressof(self._metrics) if metrics else None
        self.mcfg = mc
        self.cb = L.fdgpu_vmux_callbacks()
        self._halt = c.c_uint64(0)
        self._mstats = MuxStats()
        self._rc = None
        self._registered = []
        if register:
            # gather: the device reads the payloads in the in dcaches and
            # re-reads their mcache lines (a shared-memory link: its region)
            bufs = [out_link.dcache]
            if vc.gpu_parse == 2:
                for ln in in_links:
                    reg = getattr(ln, "_region", None)
                    bufs += [reg] if reg is not None else [ln.dcache, ln.mcache]
            for e in getattr(verifier, "engines", []):
                for b in bufs:
                    e.host_register(b)
                    self._registered.append((e, b))
        self._threading = threading
        self._th = None

    def start(self, cpu=None):
        """Runs the mux loop on a thread of its own (pinned to `cpu` by the
        thread itself, so the caller's own affinity is never touched)."""
        up = self._threading.Event()

        def body():
            if cpu is not None:
                os.sched_setaffinity(0, {cpu})
            up.set()
            self._rc = lib().fdt_mux_run(c.byref(self.mcfg), c.byref(self.cb), self._t, c.byref(self._halt),
                                         c.byref(self._mstats))
        self._halt.value = 0
        self._th = self._threading.Thread(target=body, daemon=True)
        self._th.start()
        # returns once the thread is entering the loop (as the reference's tiles
        # signal RUN on their cnc before their producers start): a producer
        # started next cannot lap a shallow link before the tile polls it
        up.wait(10.0)

    def stop(self):
        if self._th is not None:
            self._halt.value = 1
            self._th.join()
            self._th = None
            if self._rc:
                raise RuntimeError("fdt_mux_run: bad configuration")

    def final_cnt(self):
        return lib().fdgpu_vmux_final_cnt(self._t)

    def run(self, n_frags, timeout_s=60.0):
        """Runs the mux thread until the outcome of n_frags frags (all of this
        tile's in-link frags, its round-robin share included) is final."""
        import time
        self.start()
        t0 = time.time()
        try:
            while self.final_cnt() < n_frags:
                if lib().fdgpu_vmux_error(self._t):
                    raise RuntimeError(f"verify mux tile: verifier error {lib().fdgpu_vmux_error(self._t)}")
                if time.time() - t0 > timeout_s:
                    raise TimeoutError(f"verify mux tile: {self.final_cnt()}/{n_frags} frags final")
                time.sleep(0.0005)
        finally:
            self.stop()

    def stats(self):
        s = VTileStats()
        lib().fdgpu_vmux_stats(self._t, c.byref(s))
        return s.as_dict()

    def mux_stats(self):
        return self._mstats.as_dict()

    def metrics(self):
        """The reference's metrics (Tile, Stem, Link in) as the mux loop last
        wrote them (metrics=True), or None."""
        if self._metrics is None:
            return None
        snap = MuxMetrics()          # a consistent copy (the loop's writes are a seqlock)
        if lib().fdt_mux_metrics_snapshot(c.byref(self._metrics), c.byref(snap), 1 << 20):
            raise RuntimeError("fdt_mux_metrics_snapshot: no stable copy")
        d = snap.as_dict(len(self.in_links))
        d["housekeeping_cnt"] //= 2            # the sequence word counts two per write
        return d

    def latencies_ns(self):
        n = self.stats()["lat_cnt"]
        out = np.zeros(max(n, 1), dtype=np.uint64)
        n = lib().fdgpu_vmux_latencies(self._t, out.ctypes.data, n)
        return out[:n]

    def idle(self):
        return bool(lib().fdgpu_vmux_idle(self._t))

    def log(self, max_entries=1 << 24):
        seqs = np.zeros(max_entries, dtype=np.uint64)
        codes = np.zeros(max_entries, dtype=np.int8)
        n = lib().fdgpu_vmux_log(self._t, seqs.ctypes.data, codes.ctypes.data, max_entries)
        order = np.argsort(seqs[:n], kind="stable")
        return seqs[:n][order], codes[:n][order]

    def close(self):
        self.stop()
        if self._t:
            lib().fdgpu_vmux_delete(self._t)
            self._t = None
        for e, b in self._registered:
            e.host_unregister(b)
        self._registered = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


LAP_OFF = (1 << 64) - 1      # lap_span_max / lap_margin: that part of the lap guard off


def vmux_dcache_data_sz(cr_max, batch_txn_max, inflight_max=2):
    """Out dcache bytes the verify mux tile wants (fdgpu_vmux_dcache_data_sz)."""
    return lib().fdgpu_vmux_dcache_data_sz(cr_max, batch_txn_max, inflight_max)


class DedupTile:
    """The dedup tile (fd_dedup.c) over one or more verify outputs."""

    def __init__(self, in_links, out_link, hashmap_seed=0xDED0, tcache_depth=4194302, tcache_map_cnt=0,
                 unparsed_in_cnt=0, reliable=False):
        """reliable: the tile writes its progress into each in link's fseq (the
        producer -- a verify tile with flow_control -- waits for it) instead of
        being lapped when it falls behind."""
        L = lib()
        cfg = DTileCfg()
        cfg.in_cnt = len(in_links)
        for i, lk in enumerate(in_links):
            cfg.in_mcache[i], cfg.in_depth[i], cfg.in_seq0[i] = lk.mcache_ptr, lk.depth, lk.seq0
            cfg.in_base[i], cfg.in_chunk0[i], cfg.in_wmark[i] = lk.base_ptr, lk.chunk0, lk.wmark
            if reliable:
                cfg.in_fseq[i] = lk.fseq.ctypes.data
        cfg.unparsed_in_cnt = unparsed_in_cnt
        cfg.out_mcache, cfg.out_depth, cfg.out_seq0 = out_link.mcache_ptr, out_link.depth, out_link.seq0
        cfg.out_base, cfg.out_chunk0, cfg.out_wmark = out_link.base_ptr, out_link.chunk0, out_link.wmark
        cfg.hashmap_seed, cfg.tcache_depth, cfg.tcache_map_cnt = hashmap_seed, tcache_depth, tcache_map_cnt
        self.cfg, self.links = cfg, (in_links, out_link)
        self._t = L.fdgpu_dtile_new(c.byref(cfg))
        if not self._t:
            raise RuntimeError("fdgpu_dtile_new: bad configuration")

    def step(self):
        return lib().fdgpu_dtile_step(self._t)

    def run_until_idle(self, max_idle=4):
        idle, n = 0, 0
        while idle < max_idle:
            k = self.step()
            n += k
            idle = idle + 1 if k == 0 else 0
        return n

    def stats(self):
        s = DTileStats()
        lib().fdgpu_dtile_stats(self._t, c.byref(s))
        return s.as_dict()

    def tcache_fill(self, n, seed=1):
        """Insert n pseudo-random tags into the tile's tcache (a long-running
        tile's steady state: the ring full, every insert evicting); returns
        the dups among them."""
        tags = np.random.default_rng(seed).integers(1, 2 ** 63, size=n, dtype=np.uint64)
        return int(lib().fdt_tcache_insert_many(lib().fdgpu_dtile_tcache(self._t), tags.ctypes.data, n))

    def fork_sandboxed(self, frag_target, idle_s=10.0, logfile_fd=2):
        """Runs this tile in a forked child process inside the tiles' seccomp
        sandbox (fdgpu_dtile_run_sandboxed).  Its links must live in shared
        memory (Link.shm_create).  Returns (pid, stats_fn): stats_fn() reads
        the stats the child left behind once it has exited."""
        shared = mmap.mmap(-1, c.sizeof(DTileStats), mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        st = DTileStats.from_buffer(shared)
        pid = os.fork()
        if pid == 0:                                             # child: never returns
            try:
                lib().fdgpu_dtile_run_sandboxed(self._t, frag_target, int(idle_s * 1e9), c.byref(st), logfile_fd)
            finally:
                os._exit(4)

        def stats():
            return DTileStats.from_buffer_copy(shared).as_dict()
        return pid, stats

    def close(self):
        if self._t:
            lib().fdgpu_dtile_delete(self._t)
            self._t = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Producer:
    """Line-rate producer thread (stands in for the quic tile)."""

    def __init__(self, link, payloads_arena, offs, sizes, rate_tps=0.0):
        L = lib()
        self._keep = (np.ascontiguousarray(payloads_arena, dtype=np.uint8),
                      np.ascontiguousarray(offs, dtype=np.uint64), np.ascontiguousarray(sizes, dtype=np.uint32))
        a, o, s = self._keep
        self._p = L.fdgpu_producer_start(link.mcache_ptr, link.depth, link.seq0, link.base_ptr, link.chunk0,
                                         link.wmark, a.ctypes.data, o.ctypes.data, s.ctypes.data, len(o),
                                         float(rate_tps))
        if not self._p:
            raise RuntimeError("fdgpu_producer_start failed")

    def running(self):
        return self._p is not None and not lib().fdgpu_producer_done(self._p)

    def join(self):
        el = c.c_double()
        n = lib().fdgpu_producer_join(self._p, c.byref(el))
        self._p = None
        return n, el.value
