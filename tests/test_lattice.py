"""fdgpu_lattice.h (half-size scalars for the verify equation) on the CPU,
against Python integers: for every k the split (u, v) must satisfy
u = v k (mod 8L), v odd, 0 < |v| < L and |u|, |v| < 2^bits <= 2^159 whenever
it reports ok -- the conditions under which [w]B - [u]A - [v]R = O decides
the reference's cofactorless [S]B - [k]A == R exactly (file comment)."""
import ctypes
import os
import random
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = 2**252 + 27742317777372353535851937790883648493
N = 8 * L


@pytest.fixture(scope="module")
def hs(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("lat") / "liblattice.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                    os.path.join(REPO, "tests", "native", "lattice_host.cpp"), "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.hs_split_host.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int]

    def split(k, which=0):
        kb = (ctypes.c_uint32 * 8)(*[(k >> (32 * i)) & 0xffffffff for i in range(8)])
        u, v, f = (ctypes.c_uint32 * 5)(), (ctypes.c_uint32 * 5)(), (ctypes.c_uint32 * 4)()
        lib.hs_split_host(kb, u, v, f, which)
        uu = sum(x << (32 * i) for i, x in enumerate(u))
        vv = sum(x << (32 * i) for i, x in enumerate(v))
        return (-uu if f[1] else uu), (-vv if f[2] else vv), bool(f[0]), f[3]
    return split


def _check(split, k):
    u, v, ok, bits = split(k)
    if not ok:
        return False
    assert (u - v * k) % N == 0, k
    assert v % 2 == 1 and 0 < abs(v) < L
    assert max(abs(u).bit_length(), abs(v).bit_length()) == bits <= 159
    return True


def test_random_scalars(hs):
    rnd = random.Random(0x1A7)
    oks = sum(_check(hs, rnd.randrange(L)) for _ in range(20000))
    assert oks >= 19990                       # fallback rate ~1e-5 (file comment)


def test_edge_scalars(hs):
    ks = [0, 1, 2, 3, 7, 8, 2**64, 2**127 - 1, 2**127, 2**128 - 1, 2**128, 2**128 + 1, L - 1, L - 2, L // 2,
          L // 3, L // 8, (N // 2) % L, 2**252, 2**252 - 1, 2**200, (1 << 253) % L]
    for k in ks:
        u, v, ok, bits = hs(k)
        if ok:
            _check(hs, k)
        else:
            assert k == 0 or k >= 2**100, k     # tiny k: (k, 1) is the split
    # k < 2^128: the loop never runs and (u, v) = (k, 1)
    for k in (1, 5, 2**100 + 3, 2**128 - 1):
        assert hs(k)[:3] == (k, 1, True)


def test_scalars_with_large_quotients(hs):
    """k near rationals with small denominators give huge partial quotients
    (k ~ N m / n): the split must stay exact, or report not-ok (full path)."""
    rnd = random.Random(9)
    for _ in range(3000):
        n = rnd.randrange(1, 1 << 40)
        m = rnd.randrange(1, n + 1)
        k = (N * m // n + rnd.randrange(-1000, 1000)) % L
        _check(hs, k)


def test_lehmer_matches_euclid(hs):
    """hs_split (Lehmer: Euclid simulated on 52-bit leading parts, matrix
    applied to the full values) stops where the one-step-at-a-time Euclid
    stops, so both return the same split -- except that a quotient >= 2^31
    inside a simulated run is exact in Lehmer (ok) where the full-precision
    step gives up (not ok)."""
    rnd = random.Random(0x1E4)
    ks = [rnd.randrange(L) for _ in range(20000)]
    ks += [rnd.randrange(2**128, 2**140) for _ in range(500)]          # short runs, the stop near the top
    ks += [(N * m // n + rnd.randrange(-50, 50)) % L                    # large partial quotients
           for n, m in ((rnd.randrange(1, 1 << 36), rnd.randrange(1, 1 << 20)) for _ in range(3000)) if m < n]
    ks += [2**128 + i for i in range(50)] + [2**129 - i for i in range(1, 50)] + [L - i for i in range(1, 50)]
    for k in ks:
        a, b = hs(k, 0), hs(k, 1)
        if b[2]:
            assert a == b, k
        elif a[2]:
            _check(hs, k)
