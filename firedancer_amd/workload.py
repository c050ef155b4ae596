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
        g.fdgen_txns_ex.argtypes = [c.c_uint64, c.c_uint64, c.c_int, c.c_uint32, c.c_uint32, c.c_uint32, c.c_double,
                                    c.c_int, c.c_uint64, c.c_uint32, c.c_void_p, c.c_void_p, c.c_void_p, c.c_int]
        g.fdgen_txns_ex.restype = c.c_int
        g.fdgen_sign.argtypes = [c.c_char_p, c.c_char_p, c.c_uint64, c.c_char_p, c.c_char_p]
        g.fdgen_sign.restype = c.c_int
        _GEN = g
    return _GEN


def cpu_share_evidence():
    """What bounds this process's CPU use, as read on the host: the cgroup v2
    quota (/sys/fs/cgroup/cpu.max, quota/period CPUs), the affinity mask, and
    the thread limit the environment sets (a GPU box sets OMP_NUM_THREADS to
    its one-GPU share, 16, while os.cpu_count() and the affinity mask show the
    whole machine).  share = the quota when one is set, else
    OMP_NUM_THREADS, else 16; never more than the affinity mask."""
    ev = {}
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        ev["cgroup_cpu_max"] = " ".join(q)
        if q and q[0] != "max":
            ev["cgroup_quota_cpus"] = int(q[0]) / int(q[1])
    except (OSError, ValueError, IndexError):
        ev["cgroup_cpu_max"] = None
    try:
        ev["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        ev["affinity_cpus"] = os.cpu_count() or 1
    ev["os_cpu_count"] = os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS", "")
    ev["OMP_NUM_THREADS"] = omp or None
    if ev.get("cgroup_quota_cpus"):
        share, src = int(ev["cgroup_quota_cpus"]), "cgroup cpu.max quota"
    elif omp.isdigit() and int(omp) > 0:
        share, src = int(omp), "OMP_NUM_THREADS"
    else:
        share, src = 16, "default one-GPU share (16)"
    ev["share"] = max(1, min(share, ev["affinity_cpus"]))
    ev["share_source"] = src
    return ev


# A GPU box gives one GPU's share of the host (cpu_share_evidence): worker
# pools stay within it.
BOX_CPU_SHARE = cpu_share_evidence()["share"]


def default_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, BOX_CPU_SHARE))


def _cpu_busy_ticks():
    """{cpu: busy jiffies} from /proc/stat (total minus idle and iowait)"""
    out = {}
    try:
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3:4].isdigit():
                    v = line.split()
                    t = [int(x) for x in v[1:]]
                    out[int(v[0][3:])] = sum(t) - t[3] - (t[4] if len(t) > 4 else 0)
    except OSError:
        pass
    return out


def _smt_siblings(cpu):
    """The logical CPUs sharing `cpu`'s physical core (itself included)."""
    try:
        txt = open(f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list").read().strip()
    except OSError:
        return [cpu]
    out = []
    for part in txt.split(","):
        lo, _, hi = part.partition("-")
        out.extend(range(int(lo), int(hi or lo) + 1))
    return out or [cpu]


def idle_first(cpus, sample_s=0.2):
    """`cpus` reordered least busy first over a short sample of /proc/stat
    (ties keep their order).  On a box whose cores other tenants share, a
    pinned tile or producer thread on a busy core runs at a fraction of its
    speed; the benches pin to the quietest cores they may use.  A core's
    busy time counts all of its SMT siblings: another tenant on the sibling
    hyperthread shares the core (one tile at ~0.7 of its rate in alternating
    runs on such a box, profiles/r05/tab_traffic/tcap3_*)."""
    import time
    a = _cpu_busy_ticks()
    time.sleep(sample_s)
    b = _cpu_busy_ticks()
    if not a or not b:
        return list(cpus)
    core = {c: sum(b.get(s, 0) - a.get(s, 0) for s in _smt_siblings(c)) for c in cpus}
    return sorted(cpus, key=lambda c: (core[c], cpus.index(c)))


def _l3_of(cpu):
    """(package, L3 id) of a logical CPU, from /sys (None when unknown)"""
    base = f"/sys/devices/system/cpu/cpu{cpu}/"
    try:
        return (open(base + "topology/physical_package_id").read().strip(),
                open(base + "cache/index3/id").read().strip())
    except OSError:
        return None


def same_l3_first(cpus, need):
    """`cpus` (least busy first, idle_first) reordered so that the first
    `need` share one L3 (one CCD of an EPYC): the quietest L3 group that has
    `need` of them, in their order, then the rest.  A tile reads every
    mcache line its producers write, so a producer and a tile on different
    CCDs (or sockets) move every line across the fabric.  Unchanged when no
    group has `need` or the topology is unknown."""
    groups = {}
    for rank, c in enumerate(cpus):
        groups.setdefault(_l3_of(c), []).append((rank, c))
    best = None
    for key, members in groups.items():
        if key is None or len(members) < need:
            continue
        score = sum(r for r, _ in members[:need])          # lower: quieter (earlier in idle order)
        if best is None or score < best[0]:
            best = (score, [c for _, c in members[:need]])
    if best is None:
        return list(cpus)
    head = best[1]
    return head + [c for c in cpus if c not in head]


def physical_cpus(limit=BOX_CPU_SHARE):
    """One logical CPU per physical core among the CPUs this process may run
    on (SMT siblings skipped; /sys topology), at most `limit`: the CPU
    baseline pins one thread to each (BASELINE.md "one pinned thread per
    physical core", within the box's CPU share)."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        allowed = list(range(os.cpu_count() or 1))
    seen, out = set(), []
    for cpu in allowed:
        base = f"/sys/devices/system/cpu/cpu{cpu}/topology/"
        try:
            key = (open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip())
        except OSError:
            key = ("cpu", str(cpu))
        if key in seen:
            continue
        seen.add(key)
        out.append(cpu)
        if len(out) >= limit:
            break
    return out or [0]


# corruption modes (modes[i]): which bit the generator flipped
MODE_NONE, MODE_SIG, MODE_MSG, MODE_PUB, MODE_R = 0, 1, 2, 3, 4


def make_txns(n, seed, multi=False, msg_lo=180, msg_hi=220, max_sigs=12, corrupt=0.10, nthreads=None,
              corrupt_mode=0, key_pool=0):
    """Returns (arena uint8[n*stride + slack], txns TXN_DTYPE[n], modes uint8[n]).
    corrupt_mode 0 flips a bit of a random one of signature / message /
    public key (test_ed25519.c:920-951's bad-sig/msg/pub modes); MODE_* forces
    one (MODE_R: a bit of R).  key_pool K > 0 draws signers from K seeded key
    pairs instead of a fresh pair per signer."""
    stride = 1232 + 16 if multi else ((1 + 64 + max(msg_hi, 256) + 15) // 16) * 16
    arena = np.zeros(n * stride + 256, dtype=np.uint8)
    txns = np.zeros(n, dtype=TXN_DTYPE)
    modes = np.zeros(n, dtype=np.uint8)
    rc = gen().fdgen_txns_ex(n, seed, 1 if multi else 0, msg_lo, msg_hi, max_sigs, corrupt, corrupt_mode, key_pool,
                             stride, arena.ctypes.data, txns.ctypes.data, modes.ctypes.data,
                             nthreads or default_threads())
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


_P = 2**255 - 19
_L = 2**252 + 27742317777372353535851937790883648493

# The eight small-order encodings (fd_curve25519.h:87-94 lists the points;
# these are their canonical encodings with both sign bits where x == 0).
SMALL_ORDER_ENC = [
    "0100000000000000000000000000000000000000000000000000000000000000",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0000000000000000000000000000000000000000000000000000000000000080",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa"]


def small_order_cross_product(msg=b"cross"):
    """SURVEY §8(d) cfg4 adversarial set: the small-order encodings, their
    y+p variants (where y+p < 2^255) with both sign bits, plus one valid
    (R, A), as A x R, with S in {0, 1, L-1, L, L+1, 2^253-1, 2^256-1, valid S}.
    Returns a list of (msg, sig, pub) records."""
    le = lambda x: int(x % (1 << 256)).to_bytes(32, "little")  # noqa: E731
    encs = set()
    for h in SMALL_ORDER_ENC:
        y = int.from_bytes(bytes.fromhex(h), "little") & (2**255 - 1)
        for yy in (y, y + _P):
            if yy < 2**255:
                for s in (0, 1):
                    encs.add(le(yy + (s << 255)))
    pub_ok, sig_ok = sign(bytes(range(32)), msg)
    encs.add(pub_ok)
    encs.add(sig_ok[:32])
    encs = sorted(encs)
    Ss = [0, 1, _L - 1, _L, _L + 1, 2**253 - 1, 2**256 - 1, int.from_bytes(sig_ok[32:], "little")]
    return [(msg, Renc + le(S), Aenc) for Aenc in encs for Renc in encs for S in Ss]


def explode_sigs(txns):
    """One single-signature descriptor per signature of each transaction (the
    signature's own R||S and public key, the transaction's shared message):
    the per-signature view of fd_ed25519_verify_batch_single_msg's inputs."""
    cnt = txns["sig_cnt"].astype(np.int64)
    cnt = np.where((cnt >= 1) & (cnt <= 16), cnt, 0)
    owner = np.repeat(np.arange(len(txns)), cnt)
    j = np.arange(len(owner)) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    out = np.zeros(len(owner), dtype=TXN_DTYPE)
    t = txns[owner]
    out["msg_off"], out["msg_sz"] = t["msg_off"], t["msg_sz"]
    out["sig_off"] = t["sig_off"] + 64 * j
    out["pub_off"] = t["pub_off"] + 32 * j
    out["sig_cnt"] = 1
    return out, owner


def payloads(arena, txns):
    """Raw Solana wire payloads ([sig_cnt][sigs][message]) of generated txns."""
    return [bytes(arena[int(t["sig_off"]) - 1: int(t["msg_off"]) + int(t["msg_sz"])]) for t in txns]


def pack_payloads(payload_list):
    """payload bytes list -> (arena uint8, offs uint64, sizes uint32) for the frag producer."""
    sizes = np.array([len(p) for p in payload_list], dtype=np.uint32)
    offs = np.zeros(len(payload_list), dtype=np.uint64)
    if len(payload_list):
        offs[1:] = np.cumsum(sizes.astype(np.uint64))[:-1]
    arena = np.frombuffer(b"".join(payload_list) or b"\0", dtype=np.uint8).copy()
    return arena, offs, sizes
