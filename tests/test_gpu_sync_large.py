"""The synchronous API on messages larger than one batch arena (VERDICT r05
item 5): the reference hashes any msg_sz
(src/ballet/ed25519/fd_ed25519_user.c:205-207), so such a call must get the
reference's code, not an abort.  The engine hashes SHA-512(R || A || M) of
such a message on the device in arena-sized pieces
(fdgpu_sha512_stream_kernel) and verifies from the digests.  The real limit
is ~2 GB; FDGPU_SYNC_ARENA_MAX lowers it (read when the library loads, so the
calls run in a child process) so that small messages take the piecewise path
and cross many piece boundaries.  Every code is compared with the oracle's."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import os, random, sys
sys.path.insert(0, {repo!r})
from firedancer_amd import _lib
from oracle import oracle as orc
L = _lib.lib()
rng = random.Random(0x1A46E)
keys = []
for _ in range(16):
    prv = bytes(rng.getrandbits(8) for _ in range(32))
    keys.append((prv, orc.public_from_private(prv)))
limit = int(os.environ["FDGPU_SYNC_ARENA_MAX"])
bad = 0
checked = 0
for sz in (0, 100, limit - 200, limit - 96, limit - 95, limit + 1, 2 * limit - 64, 2 * limit - 63, 3 * limit + 17,
           16 * limit + 111, 40000, 40000 + 127, 40000 + 128):
    for n in (1, 2, 5, 16):
        for mode in range(5):
            msg = bytearray(rng.getrandbits(8) for _ in range(sz))
            sigs, pubs = b"", b""
            for i in range(n):
                prv, pub = keys[i]
                sigs += orc.sign(bytes(msg), pub, prv)
                pubs += pub
            sigs, pubs = bytearray(sigs), bytearray(pubs)
            if mode == 1 and sz:                      # the message changed after signing
                msg[rng.randrange(sz)] ^= 1 << rng.randrange(8)
            elif mode == 2:                           # one signature's R
                sigs[64 * rng.randrange(n) + rng.randrange(32)] ^= 1 << rng.randrange(8)
            elif mode == 3:                           # one signature's S (often >= L)
                sigs[64 * rng.randrange(n) + 63] |= 0xF0
            elif mode == 4:                           # one public key
                pubs[32 * rng.randrange(n) + rng.randrange(32)] ^= 1 << rng.randrange(8)
            msg, sigs, pubs = bytes(msg), bytes(sigs), bytes(pubs)
            exp = orc.verify_batch_single_msg(msg, sigs, pubs, n)
            got = L.fd_ed25519_verify_batch_single_msg(msg, len(msg), sigs, pubs, None, n)
            checked += 1
            if got != exp:
                bad += 1
                print("mismatch", sz, n, mode, got, exp, flush=True)
            if n == 1:
                exp1 = orc.verify(msg, sigs, pubs)
                got1 = L.fd_ed25519_verify(msg, len(msg), sigs, pubs, None)
                checked += 1
                if got1 != exp1:
                    bad += 1
                    print("mismatch single", sz, mode, got1, exp1, flush=True)
print("checked", checked, "bad", bad, "errors", L.fdgpu_sync_errors(), flush=True)
"""


@pytest.mark.gpu
def test_sync_api_message_beyond_arena_gets_reference_code():
    env = dict(os.environ, FDGPU_SYNC_ARENA_MAX="4096")
    env.pop("FDGPU_SYNC_FAIL_CLOSED", None)
    r = subprocess.run([sys.executable, "-c", _CHILD.format(repo=REPO)], capture_output=True, text=True, env=env,
                       timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    last = r.stdout.strip().splitlines()[-1].split()
    assert last[0] == "checked" and int(last[1]) > 300, r.stdout[-2000:]
    assert last[3] == "0" and last[5] == "0", r.stdout[-3000:]


def test_sync_arena_override_is_bounded():
    """The override only lowers the limit (values below 1 KiB or above the
    32-bit arena are ignored): checked on the source, no GPU needed."""
    src = open(os.path.join(REPO, "firedancer_amd", "csrc", "fdgpu_engine.cpp")).read()
    assert 'getenv("FDGPU_SYNC_ARENA_MAX")' in src
    assert "m >= 1024 && m < SYNC_ARENA_LIMIT" in src
    assert "sync_run_prehashed" in src and "call too large" not in src
