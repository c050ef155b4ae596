"""The committed device constants (firedancer_amd/csrc/fdgpu_consts.h) equal
their definitions, re-derived here with Python integers."""
import os
import re

import pyref_ed25519 as pyref

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "firedancer_amd", "csrc",
                   "fdgpu_consts.h")
P, L = pyref.P, pyref.L
WIDTHS = [26, 25] * 5


def _parse():
    out = {}
    for m in re.finditer(r"#define (FDGPU_\w+) \{ ([^}]*) \}", open(HDR).read()):
        out[m.group(1)] = [int(x.strip().rstrip("u"), 16) for x in m.group(2).split(",")]
    return out


def _fe(limbs):
    v, pos = 0, 0
    for x, w in zip(limbs, WIDTHS):
        v += x << pos
        pos += w
    return v


def test_field_constants():
    c = _parse()
    D = (-121665 * pow(121666, P - 2, P)) % P
    assert _fe(c["FDGPU_FE_D"]) == D
    assert _fe(c["FDGPU_FE_D2"]) == 2 * D % P
    s = _fe(c["FDGPU_FE_SQRTM1"])
    assert s * s % P == P - 1
    bx, by = _fe(c["FDGPU_FE_BX"]), _fe(c["FDGPU_FE_BY"])
    assert (by, bx) == (pyref.B[1], pyref.B[0])
    assert by == 4 * pow(5, P - 2, P) % P and bx % 2 == 0
    assert _fe(c["FDGPU_FE_BT"]) == bx * by % P
    assert (-bx * bx + by * by - 1 - D * bx * bx * by * by) % P == 0
    for name in ("FDGPU_FE_Y0", "FDGPU_FE_Y1"):
        y = _fe(c[name])
        enc = y.to_bytes(32, "little")
        pt = pyref.decode(enc, "ref")
        assert pt is not None and pyref._small_order(pt)
    assert {_fe(c["FDGPU_FE_Y0"]).to_bytes(32, "little").hex()[:8], _fe(c["FDGPU_FE_Y1"]).to_bytes(32, "little").hex()[:8]} == {"26e8958f", "c7176a70"}
    assert _fe(c["FDGPU_FE_2P"]) == 2 * P and _fe(c["FDGPU_FE_4P"]) == 4 * P


def test_scalar_constants():
    c = _parse()
    l = sum(x << (32 * i) for i, x in enumerate(c["FDGPU_SC_L"]))
    mu = sum(x << (32 * i) for i, x in enumerate(c["FDGPU_SC_MU"]))
    assert l == L and mu == (1 << 512) // L
