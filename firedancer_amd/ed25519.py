"""Python mirror of the reference's Ed25519 verify interface, served by the
MI355X engine through the C ABI (include/fd_ed25519_gpu.h).

Reference interface (src/ballet/ed25519/fd_ed25519.h):
  FD_ED25519_SUCCESS / ERR_SIG / ERR_PUBKEY / ERR_MSG       :11-14
  fd_ed25519_verify(msg, msg_sz, sig, public_key, sha)      :96-101
  fd_ed25519_verify_batch_single_msg(msg, msg_sz, signatures, pubkeys, shas, batch_sz)  :124-130
  fd_ed25519_strerror(err)                                  :132-136

Same names (without the fd_ed25519_ prefix), argument meaning and codes;
the SHA-512 scratch objects are accepted and ignored (hashing is on the GPU).
The batched engine (VerifyEngine) is the throughput path used by the verify
stage; per-transaction results equal fd_ed25519_verify_batch_single_msg.
"""
import ctypes

import numpy as np

from . import _lib

SUCCESS, ERR_SIG, ERR_PUBKEY, ERR_MSG = 0, -1, -2, -3

FLAG_REF_MAPPING = 1
FLAG_NO_BUCKET = 2      # verify in transaction order instead of grouped by SHA-512 block count
FLAG_FULL_PATH = 4      # diagnostics: every signature through the full-length fallback kernel
FLAG_KEY_CACHE = 8      # one A decode + table per distinct public key of a batch (signer reuse)
FLAG_PAIR = 16          # two lanes per signature: a shorter verify for batches that leave the GPU idle
FLAG_PAIR_AUTO = 32     # the two-lane kernel for small ring batches while the engine is otherwise idle
FLAG_MERGE = 64         # gathered batches' verifies merged into shared launches
FLAG_SPREAD = 128       # one verify block per CU
FLAG_SPREAD_AUTO = 256  # ... while the engine's batches fit the chip that way

# fdgpu_txn_t as a numpy record (msg_off, msg_sz, sig_off, pub_off, sig_cnt)
TXN_DTYPE = np.dtype([("msg_off", "<u4"), ("msg_sz", "<u4"), ("sig_off", "<u4"),
                      ("pub_off", "<u4"), ("sig_cnt", "<u4")])
SIG_DESC_DTYPE = np.dtype([("msg_off", "<u4"), ("msg_sz", "<u4"), ("sig_off", "<u4"), ("pub_off", "<u4")])
TXN_DESC_DTYPE = np.dtype([("sig0", "<u4"), ("sig_cnt", "<u4")])
ARENA_SLACK = 160


def verify(msg, sig, public_key, sha=None):
    """fd_ed25519_verify: returns SUCCESS or an ERR_* code."""
    msg = bytes(msg)
    sig, public_key = bytes(sig), bytes(public_key)
    if len(sig) != 64 or len(public_key) != 32:
        raise ValueError("sig must be 64 bytes and public_key 32 bytes")
    return _lib.lib().fd_ed25519_verify(msg, len(msg), sig, public_key, None)


def verify_batch_single_msg(msg, signatures, pubkeys, shas, batch_sz):
    """fd_ed25519_verify_batch_single_msg: batch_sz in [1,16] else ERR_SIG."""
    msg = bytes(msg)
    signatures, pubkeys = bytes(signatures), bytes(pubkeys)
    n = int(batch_sz)
    if n < 0 or n > 255:
        raise ValueError("batch_sz is a uchar")
    if 1 <= n <= 16 and (len(signatures) < 64 * n or len(pubkeys) < 32 * n):
        raise ValueError("signatures/pubkeys shorter than batch_sz records")
    return _lib.lib().fd_ed25519_verify_batch_single_msg(msg, len(msg), signatures, pubkeys, None, n)


def sync_stats():
    """Counters of the synchronous API (fdgpu_sync_stats): calls, the GPU
    batches concurrent calls were coalesced into, engine failures answered
    with ERR_SIG."""
    import ctypes as c
    v = [c.c_uint64() for _ in range(3)]
    _lib.lib().fdgpu_sync_stats(*[c.byref(x) for x in v])
    return {"calls": v[0].value, "batches": v[1].value, "errors": v[2].value}


def strerror(err):
    """fd_ed25519_strerror."""
    return _lib.lib().fd_ed25519_strerror(int(err)).decode()


def expand_txns(txns):
    """Per-signature and per-transaction descriptors for the device path
    (the same expansion the engine's submit performs on the host)."""
    txns = np.asarray(txns, dtype=TXN_DTYPE)
    cnt = txns["sig_cnt"].astype(np.int64)
    valid = (cnt >= 1) & (cnt <= 16)
    used = np.where(valid, cnt, 0)
    sig0 = np.zeros(len(txns), dtype=np.int64)
    if len(txns):
        sig0[1:] = np.cumsum(used)[:-1]
    n_sig = int(used.sum())
    tdesc = np.zeros(len(txns), dtype=TXN_DESC_DTYPE)
    tdesc["sig0"] = sig0
    tdesc["sig_cnt"] = used
    sdesc = np.zeros(n_sig, dtype=SIG_DESC_DTYPE)
    t_of_sig = np.repeat(np.arange(len(txns)), used)
    j = np.arange(n_sig) - sig0[t_of_sig]
    sdesc["msg_off"] = txns["msg_off"][t_of_sig]
    sdesc["msg_sz"] = txns["msg_sz"][t_of_sig]
    sdesc["sig_off"] = txns["sig_off"][t_of_sig] + 64 * j
    sdesc["pub_off"] = txns["pub_off"][t_of_sig] + 32 * j
    return sdesc, tdesc


class VerifyEngine:
    """One engine per GPU: pinned double-buffered rings, HIP streams, and the
    verify kernels.  submit()/poll() is the asynchronous batch API;
    verify_txns() is submit + blocking poll."""

    def __init__(self, device=0, max_txn=1 << 16, max_sig=None, max_arena=None, ring_depth=2, ref_mapping=False,
                 bucket=True, full_path=False, key_cache=False, pair=False, pair_auto=False, merge=False,
                 spread=False, spread_auto=False):
        L = _lib.lib()
        # max_sig default: 12 signatures per txn (FD_TXN_ACTUAL_SIG_MAX), as the engine's own default
        self.max_sig = max_sig or 12 * max_txn
        flags = ((FLAG_REF_MAPPING if ref_mapping else 0) | (0 if bucket else FLAG_NO_BUCKET) |
                 (FLAG_FULL_PATH if full_path else 0) | (FLAG_KEY_CACHE if key_cache else 0) |
                 (FLAG_PAIR if pair else 0) | (FLAG_PAIR_AUTO if pair_auto else 0) | (FLAG_MERGE if merge else 0) |
                 (FLAG_SPREAD if spread else 0) | (FLAG_SPREAD_AUTO if spread_auto else 0))
        cfg = _lib.FdgpuCfg(max_txn, self.max_sig, max_arena or 1232 * max_txn, ring_depth, flags)
        self._cfg = cfg
        self.max_arena = cfg.max_arena
        self._h = L.fdgpu_engine_open(int(device), ctypes.byref(cfg))
        if not self._h:
            raise RuntimeError(f"fdgpu_engine_open({device}) failed: {_lib.last_error()}")
        self.device = device
        self._pending = {}

    def reserve(self, n_sig=0):
        """fdgpu_engine_reserve: size every ring slot for batches of up to
        n_sig signatures (0: max_sig) now, so no batch allocates inside the
        pipeline (call with nothing in flight)."""
        r = _lib.lib().fdgpu_engine_reserve(self._h, int(n_sig))
        if r:
            raise RuntimeError(f"fdgpu_engine_reserve failed: {r} ({_lib.last_error()})")

    def host_register(self, buf):
        """Registers a long-lived host buffer (numpy array) for direct DMA:
        batches whose arena lies inside it upload with no staging copy
        (fdgpu_host_register)."""
        arr = np.asarray(buf)
        r = _lib.lib().fdgpu_host_register(self._h, arr.ctypes.data, arr.nbytes)
        if r:
            raise RuntimeError(f"fdgpu_host_register failed: {r} ({_lib.last_error()})")

    def host_unregister(self, buf):
        r = _lib.lib().fdgpu_host_unregister(self._h, np.asarray(buf).ctypes.data)
        if r:
            raise RuntimeError(f"fdgpu_host_unregister failed: {r} ({_lib.last_error()})")

    def close(self):
        if self._h:
            _lib.lib().fdgpu_engine_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        g, b, w = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
        _lib.lib().fdgpu_engine_info(self._h, ctypes.byref(g), ctypes.byref(b), ctypes.byref(w))
        return {"resident_blocks": g.value, "block_threads": b.value, "ws_bytes": w.value}

    def submit(self, arena, txns):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        txns = np.ascontiguousarray(txns, dtype=TXN_DTYPE)
        tk = _lib.lib().fdgpu_submit(self._h, arena.ctypes.data, arena.size, txns.ctypes.data, len(txns))
        if tk < 0:
            raise RuntimeError(f"fdgpu_submit failed ({tk}): {_lib.last_error()}")
        self._pending[tk] = len(txns)
        return tk

    def poll(self, ticket, blocking=True):
        n = self._pending.get(ticket)
        if n is None:
            raise KeyError(ticket)
        out = np.zeros(max(n, 1), dtype=np.int8)
        rc = _lib.lib().fdgpu_poll(self._h, ticket, out.ctypes.data, 1 if blocking else 0)
        if rc == 1:
            return None
        if rc != 0:
            raise RuntimeError(f"fdgpu_poll failed ({rc}): {_lib.last_error()}")
        del self._pending[ticket]
        return out[:n]

    def verify_txns(self, arena, txns):
        return self.poll(self.submit(arena, txns), blocking=True)

    def submit_frags(self, arena, frags, trailer_sz):
        """fdgpu_submit_frags: raw payloads parsed on the GPU; frags is a
        FRAG_EX_DTYPE array ({off, sz, tr_off, tr_cap})."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        frags = np.ascontiguousarray(frags, dtype=FRAG_EX_DTYPE)
        tk = _lib.lib().fdgpu_submit_frags(self._h, arena.ctypes.data, arena.size, frags.ctypes.data, len(frags),
                                           int(trailer_sz))
        if tk < 0:
            raise RuntimeError(f"fdgpu_submit_frags failed ({tk}): {_lib.last_error()}")
        self._pending[tk] = (len(frags), int(trailer_sz))
        return tk

    def poll_frags(self, ticket, blocking=True):
        """-> (codes int8[n], trailers uint8[trailer_sz]) or None while pending."""
        n, tsz = self._pending[ticket]
        codes = np.zeros(max(n, 1), dtype=np.int8)
        tr = np.zeros(max(tsz, 1), dtype=np.uint8)
        rc = _lib.lib().fdgpu_poll_frags(self._h, ticket, codes.ctypes.data, tr.ctypes.data, 1 if blocking else 0)
        if rc == 1:
            return None
        if rc != 0:
            raise RuntimeError(f"fdgpu_poll_frags failed ({rc}): {_lib.last_error()}")
        del self._pending[ticket]
        return codes[:n], tr[:tsz]

    def submit_frags_io(self, frags, out, out_sz, hash_seed, links=None):
        """fdgpu_submit_frags_io: payloads read by the device where they lie
        (frags: FRAG_IO_DTYPE {src host address, sz, out_off, out_cap, link,
        seq}, every src inside a registered buffer), out frags written to
        `out` (a registered numpy buffer) [0, out_sz).  links: (mcache
        address, depth) per in link; a frag with link = i + 1 has links[i]'s
        line of its seq re-read by the device after its payload
        (FDGPU_CODE_LAPPED when republished)."""
        frags = np.ascontiguousarray(frags, dtype=FRAG_IO_DTYPE)
        out = np.asarray(out)
        if out_sz > out.nbytes:
            raise ValueError("out_sz exceeds the out buffer")
        lk = np.array(list(links or []), dtype=LINK_DTYPE)
        tk = _lib.lib().fdgpu_submit_frags_io(self._h, frags.ctypes.data, len(frags), out.ctypes.data, int(out_sz),
                                              int(hash_seed), lk.ctypes.data if len(lk) else None, len(lk))
        if tk < 0:
            raise RuntimeError(f"fdgpu_submit_frags_io failed ({tk}): {_lib.last_error()}")
        self._pending[tk] = (len(frags), frags)
        return tk

    def poll_frags_io(self, ticket, blocking=True):
        """-> (codes int8[n], tags uint64[n], out_szs uint16[n]) or None while pending."""
        n, _ = self._pending[ticket]
        codes = np.zeros(max(n, 1), dtype=np.int8)
        tags = np.zeros(max(n, 1), dtype=np.uint64)
        osz = np.zeros(max(n, 1), dtype=np.uint16)
        rc = _lib.lib().fdgpu_poll_frags_io(self._h, ticket, codes.ctypes.data, tags.ctypes.data, osz.ctypes.data,
                                            1 if blocking else 0)
        if rc == 1:
            return None
        if rc != 0:
            raise RuntimeError(f"fdgpu_poll_frags_io failed ({rc}): {_lib.last_error()}")
        del self._pending[ticket]
        return codes[:n], tags[:n], osz[:n]

    def verify_device(self, d_arena, d_sig_desc, n_sig, d_txn_desc, n_txn, d_sig_codes, d_txn_codes, stream=0):
        """Device-resident path; all pointers are device addresses (ints)."""
        rc = _lib.lib().fdgpu_verify_device(self._h, d_arena, d_sig_desc, n_sig, d_txn_desc, n_txn,
                                            d_sig_codes, d_txn_codes, stream or None)
        if rc != 0:
            raise RuntimeError(f"fdgpu_verify_device failed ({rc}): {_lib.last_error()}")

    def upload(self, arena, txns):
        """Stage a batch in HBM once (DeviceBatch); verify it any number of times."""
        return DeviceBatch(self, arena, txns)

    def upload_frags(self, arena, frags):
        """Raw transaction payloads in HBM (FragBatch): each verify parses
        them on the GPU (fdgpu_dev_batch_upload_frags)."""
        return FragBatch(self, arena, frags)

    def sync(self):
        self._chk(_lib.lib().fdgpu_sync(self._h), "fdgpu_sync")

    # ---- per-stage diagnostics (parity tests) ----
    def _chk(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc}): {_lib.last_error()}")

    def debug_fe_ops(self, ab):
        ab = np.ascontiguousarray(ab, dtype=np.uint8).reshape(-1, 64)
        out = np.zeros((len(ab), 8, 32), dtype=np.uint8)
        self._chk(_lib.lib().fdgpu_debug_fe_ops(self._h, ab.ctypes.data, len(ab), out.ctypes.data), "debug_fe_ops")
        return out

    def debug_decode(self, enc, ref_mapping=False):
        enc = np.ascontiguousarray(enc, dtype=np.uint8).reshape(-1, 32)
        out = np.zeros((len(enc), 72), dtype=np.uint8)
        self._chk(_lib.lib().fdgpu_debug_decode(self._h, enc.ctypes.data, len(enc), 1 if ref_mapping else 0,
                                                out.ctypes.data), "debug_decode")
        rc = out[:, 0:4].copy().view(np.int32)[:, 0]
        so = out[:, 4:8].copy().view(np.int32)[:, 0]
        return rc, so, out[:, 8:40], out[:, 40:72]

    def debug_sha512(self, arena, txns):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        txns = np.ascontiguousarray(txns, dtype=TXN_DTYPE)
        out = np.zeros((len(txns), 64), dtype=np.uint8)
        self._chk(_lib.lib().fdgpu_debug_sha512(self._h, arena.ctypes.data, arena.size, txns.ctypes.data, len(txns),
                                                out.ctypes.data), "debug_sha512")
        return out

    def debug_hram(self, arena, txns):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        txns = np.ascontiguousarray(txns, dtype=TXN_DTYPE)
        out = np.zeros((len(txns), 32), dtype=np.uint8)
        self._chk(_lib.lib().fdgpu_debug_hram(self._h, arena.ctypes.data, arena.size, txns.ctypes.data, len(txns),
                                              out.ctypes.data), "debug_hram")
        return out

    def debug_sc_reduce(self, x):
        x = np.ascontiguousarray(x, dtype=np.uint8).reshape(-1, 64)
        out = np.zeros((len(x), 32), dtype=np.uint8)
        self._chk(_lib.lib().fdgpu_debug_sc_reduce(self._h, x.ctypes.data, len(x), out.ctypes.data), "debug_sc_reduce")
        return out

    def debug_hs_split(self, k):
        """k: uint8[n, 32] scalars < L -> uint32[n, 16] (|u|, |v|, ok, u_neg, v_neg, bits)"""
        k = np.ascontiguousarray(k, dtype=np.uint8).reshape(-1, 32)
        out = np.zeros((len(k), 16), dtype=np.uint32)
        self._chk(_lib.lib().fdgpu_debug_hs_split(self._h, k.ctypes.data, len(k), out.ctypes.data), "debug_hs_split")
        return out

    def debug_sig_codes(self, arena, txns):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        txns = np.ascontiguousarray(txns, dtype=TXN_DTYPE)
        cnt = txns["sig_cnt"].astype(np.int64)
        n = int(np.where((cnt >= 1) & (cnt <= 16), cnt, 0).sum())
        out = np.zeros(max(n, 1), dtype=np.int8)
        self._chk(_lib.lib().fdgpu_debug_sig_codes(self._h, arena.ctypes.data, arena.size, txns.ctypes.data,
                                                   len(txns), out.ctypes.data), "debug_sig_codes")
        return out[:n]


class DeviceBatch:
    """A batch resident in HBM (fdgpu_dev_batch_t)."""

    def __init__(self, engine, arena, txns):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        txns = np.ascontiguousarray(txns, dtype=TXN_DTYPE)
        self._e = engine
        self.n_txn = len(txns)
        self._b = _lib.lib().fdgpu_dev_batch_upload(engine._h, arena.ctypes.data, arena.size, txns.ctypes.data,
                                                    len(txns))
        if not self._b:
            raise RuntimeError(f"fdgpu_dev_batch_upload failed: {_lib.last_error()}")
        self.n_sig = int(_lib.lib().fdgpu_dev_batch_sig_cnt(self._b))

    def own_queue(self):
        """Give this batch its own HIP stream + workspace (verifies of
        different batches then overlap on the GPU, like ring slots)."""
        rc = _lib.lib().fdgpu_dev_batch_own_queue(self._e._h, self._b)
        if rc != 0:
            raise RuntimeError(f"fdgpu_dev_batch_own_queue failed ({rc}): {_lib.last_error()}")
        return self

    def verify(self):
        """Enqueue one verify (async on the batch's queue: the engine's
        compute stream unless own_queue() was called)."""
        rc = _lib.lib().fdgpu_dev_batch_verify(self._e._h, self._b)
        if rc != 0:
            raise RuntimeError(f"fdgpu_dev_batch_verify failed ({rc}): {_lib.last_error()}")

    def codes(self, sig_codes=False):
        t = np.zeros(max(self.n_txn, 1), dtype=np.int8)
        s = np.zeros(max(self.n_sig, 1), dtype=np.int8) if sig_codes else None
        rc = _lib.lib().fdgpu_dev_batch_codes(self._e._h, self._b, t.ctypes.data,
                                              s.ctypes.data if s is not None else None)
        if rc != 0:
            raise RuntimeError(f"fdgpu_dev_batch_codes failed ({rc}): {_lib.last_error()}")
        return (t[:self.n_txn], s[:self.n_sig]) if sig_codes else t[:self.n_txn]

    def time(self, iters):
        """HIP-event timing of `iters` back-to-back verifies: (wall_ms,
        mean verify-kernel ms, mean combine-kernel ms)."""
        import ctypes as c
        w, v, k = c.c_double(), c.c_double(), c.c_double()
        rc = _lib.lib().fdgpu_dev_batch_time(self._e._h, self._b, int(iters), c.byref(w), c.byref(v), c.byref(k))
        if rc != 0:
            raise RuntimeError(f"fdgpu_dev_batch_time failed ({rc}): {_lib.last_error()}")
        return w.value, v.value, k.value

    def free(self):
        if self._b:
            _lib.lib().fdgpu_dev_batch_free(self._e._h, self._b)
            self._b = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


FRAG_DTYPE = np.dtype([("off", "<u4"), ("sz", "<u4")])
FRAG_EX_DTYPE = np.dtype([("off", "<u4"), ("sz", "<u4"), ("tr_off", "<u4"), ("tr_cap", "<u4")])
FRAG_IO_DTYPE = np.dtype([("src", "<u8"), ("sz", "<u4"), ("out_off", "<u4"), ("out_cap", "<u4"), ("link", "<u4"),
                          ("seq", "<u8")])
LINK_DTYPE = np.dtype([("mcache", "<u8"), ("depth", "<u8")])   # fdgpu_link_t
CODE_LAPPED = -66             # FDGPU_CODE_LAPPED
CODE_TRAILER_CAP = -65        # FDGPU_CODE_TRAILER_CAP
CODE_PARSE_FAIL = -64          # FDGPU_CODE_PARSE_FAIL
TXN_MAX_SZ = 852               # FD_TXN_MAX_SZ: stride of the parsed fd_txn_t records


class FragBatch(DeviceBatch):
    """Raw payloads resident in HBM (fdgpu_dev_batch_upload_frags): verify()
    runs fd_txn_parse, the signature-count scan and the descriptor expansion
    on the GPU before the verify kernels."""

    def __init__(self, engine, arena, frags):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        frags = np.ascontiguousarray(frags, dtype=FRAG_DTYPE)
        self._e = engine
        self.n_txn = len(frags)
        self._b = _lib.lib().fdgpu_dev_batch_upload_frags(engine._h, arena.ctypes.data, arena.size,
                                                          frags.ctypes.data, len(frags))
        if not self._b:
            raise RuntimeError(f"fdgpu_dev_batch_upload_frags failed: {_lib.last_error()}")
        sz = frags["sz"].astype(np.int64)
        self.sig_bound = int(np.where(sz >= 134, np.minimum(16, (sz - 38) // 96), 0).sum())   # fdgpu_frag_sig_bound
        self.n_sig = self.sig_bound

    def codes(self, sig_codes=False):
        out = super().codes(sig_codes)
        self.n_sig = int(_lib.lib().fdgpu_dev_batch_sig_cnt(self._b))
        if sig_codes:
            return out[0], out[1][:self.n_sig]
        return out

    def txns(self, records=True):
        """(parsed fd_txn_t records uint8[n, 852] or None, footprints uint16[n]; 0 = not a txn)"""
        out = np.zeros((max(self.n_txn, 1), TXN_MAX_SZ), dtype=np.uint8) if records else None
        sz = np.zeros(max(self.n_txn, 1), dtype=np.uint16)
        rc = _lib.lib().fdgpu_dev_batch_txns(self._e._h, self._b, out.ctypes.data if records else None,
                                             sz.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"fdgpu_dev_batch_txns failed ({rc}): {_lib.last_error()}")
        return (out[:self.n_txn] if records else None), sz[:self.n_txn]

    def time2(self, iters):
        """HIP-event timing: (wall_ms, mean ingest ms (parse + scan + expand),
        mean verify-kernel ms, mean combine ms)."""
        import ctypes as c
        w, g, v, k = c.c_double(), c.c_double(), c.c_double(), c.c_double()
        rc = _lib.lib().fdgpu_dev_batch_time2(self._e._h, self._b, int(iters), c.byref(w), c.byref(g), c.byref(v),
                                              c.byref(k))
        if rc != 0:
            raise RuntimeError(f"fdgpu_dev_batch_time2 failed ({rc}): {_lib.last_error()}")
        return w.value, g.value, v.value, k.value
