"""Sequential models of the reference's verify-stage tiles, used as the
checker for the batched tile (test infrastructure).

verify_tile_model restates the per-frag loop of src/app/fdctl/run/tiles/
fd_verify.c:36-148 + fd_verify.h:45-89 one frag at a time:
  round robin filter -> fd_txn_parse -> tag = fd_hash(seed, sig0, 64) ->
  tcache query (DEDUP) -> fd_ed25519_verify_batch_single_msg (FAILED) ->
  tcache insert -> publish.
The tcache model is a plain ring + set with the reference's non-LRU insert
(fd_tcache.h:344-404)."""
from collections import deque

import numpy as np

from firedancer_amd import tile


class TCacheModel:
    def __init__(self, depth):
        self.depth = depth
        self.ring = deque()
        self.set = set()

    def query(self, tag):
        return tag in self.set

    def insert(self, tag):
        if tag in self.set:
            return True
        self.ring.append(tag)
        self.set.add(tag)
        if len(self.ring) > self.depth:
            self.set.discard(self.ring.popleft())
        return False

    def reset(self):
        self.ring.clear()
        self.set.clear()


def txn_descriptor(payload, raw):
    d = tile.txn_decode(raw)
    return (d["message_off"], len(payload) - d["message_off"], d["signature_off"], d["acct_addr_off"],
            d["signature_cnt"])


def verify_tile_model(payloads, seed, verify_fn, rr_idx=0, rr_cnt=1, tcache=None, seq0=0, seqs=None):
    """payloads: list of bytes (one frag each, seq0+i; or seqs[i] when given:
    the frags a tile saw when others were lost to overrun).  verify_fn(arena,
    txns) -> codes (the oracle).  Returns (outcomes list, published list of
    (payload, raw fd_txn_t, tag))."""
    tc = tcache if tcache is not None else TCacheModel(tile.VERIFY_TCACHE_DEPTH)
    outcomes, published = [], []
    for i, p in enumerate(payloads):
        seq = seqs[i] if seqs is not None else seq0 + i
        if rr_cnt > 1 and seq % rr_cnt != rr_idx:
            outcomes.append(tile.LOG_FILTERED)
            continue
        sz, raw = tile.txn_parse(p)
        if not sz:
            outcomes.append(tile.LOG_PARSE_FAIL)
            continue
        mo, ms, so, po, sc = txn_descriptor(p, raw)
        tag = tile.fd_hash(seed, p[so:so + 64])
        if tc.query(tag):
            outcomes.append(tile.VERIFY_DEDUP)
            continue
        arena = np.frombuffer(p, dtype=np.uint8)
        txns = np.array([(mo, ms, so, po, sc)], dtype=tile.TXN_DTYPE)
        if int(verify_fn(arena, txns)[0]) != 0:
            outcomes.append(tile.VERIFY_FAILED)
            continue
        tc.insert(tag)
        outcomes.append(tile.VERIFY_SUCCESS)
        published.append((p, raw, tag))
    return outcomes, published


def dedup_model(frags, seed, depth):
    """frags: verify-tile output payloads in dedup service order."""
    tc = TCacheModel(depth)
    out = []
    for f in frags:
        payload, raw = tile.split_verify_output(f)
        so = tile.txn_decode(raw)["signature_off"]
        if not tc.insert(tile.fd_hash(seed, payload[so:so + 64])):
            out.append(f)
    return out
