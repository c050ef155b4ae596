"""The C-ABI boundary (CPU only: loading and symbol checks, no GPU calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from firedancer_amd import _lib
import firedancer_amd as fa

REF_API = ["fd_ed25519_verify", "fd_ed25519_verify_batch_single_msg", "fd_ed25519_strerror"]


def test_library_loads():
    L = _lib.lib()
    assert isinstance(L, ctypes.CDLL)


def test_exports_every_header_function():
    names = _lib.header_functions()
    for fn in REF_API:
        assert fn in names
    assert len(names) == 47, names
    L = _lib.lib()
    for n in names:
        assert hasattr(L, n), n


def test_dynamic_symbol_table_lists_exports():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = set(re.findall(r"\s[TW]\s(\w+)$", out, flags=re.M))
    for n in _lib.header_functions():
        assert n in syms, n


def test_header_is_plain_c():
    """The boundary header compiles as C11 with no HIP/torch includes."""
    src = f'#include "{_lib.HEADER_PATH}"\nint main(void){{ fdgpu_txn_t t; (void)t; return FD_ED25519_ERR_MSG + 3; }}\n'
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-x", "c", "-", "-fsyntax-only"], input=src,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    text = open(_lib.HEADER_PATH).read()
    code = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    includes = re.findall(r"#include\s*[<\"]([^>\"]+)", code)
    assert set(includes) <= {"stddef.h", "stdint.h"}, includes
    assert "hipStream_t" not in code and "torch" not in code


def test_strerror_matches_reference_table():
    """fd_ed25519_user.c:312-322 (pure host function, no GPU needed)."""
    assert fa.strerror(0) == "success"
    assert fa.strerror(-1) == "bad signature"
    assert fa.strerror(-2) == "bad public key"
    assert fa.strerror(-3) == "bad message"
    assert fa.strerror(7) == "unknown"


def test_codes_match_reference_values():
    assert (fa.SUCCESS, fa.ERR_SIG, fa.ERR_PUBKEY, fa.ERR_MSG) == (0, -1, -2, -3)


def test_txn_struct_layout():
    assert ctypes.sizeof(_lib.FdgpuTxn) == 20
    assert fa.TXN_DTYPE.itemsize == 20
    assert ctypes.sizeof(_lib.FdgpuCfg) == 32


def test_engine_open_without_gpu_fails_loudly():
    """No silent CPU fallback: opening an engine with no visible device raises."""
    if os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "") != "-1":
        pytest.skip("a GPU may be present; covered by the gpu tests")
    with pytest.raises(RuntimeError):
        fa.VerifyEngine(0, max_txn=16)


def test_product_does_not_reference_oracle():
    """The shipped package never imports or links the oracle."""
    pkg = os.path.dirname(fa.__file__)
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", "Makefile")):
                text = open(os.path.join(root, f)).read()
                for bad in ("import oracle", "from oracle", "liboracle", "fd_ed25519_oracle"):
                    assert bad not in text, (f, bad)
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out


def test_engine_flags_match_header():
    """The Python engine flags are the header's FDGPU_FLAG_* values."""
    from firedancer_amd import ed25519 as ed
    text = open(_lib.HEADER_PATH).read()
    hdr = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+FDGPU_FLAG_(\w+)\s+(\d+)u", text)}
    py = {"REF_MAPPING": ed.FLAG_REF_MAPPING, "NO_BUCKET": ed.FLAG_NO_BUCKET, "FULL_PATH": ed.FLAG_FULL_PATH,
          "KEY_CACHE": ed.FLAG_KEY_CACHE}
    assert hdr == py, (hdr, py)


def test_stamps_variant_builds():
    """The one kernel variant kept (per-phase stamps for tools/phase_stamps.py)
    still compiles for gfx950 and exports its stamp reader."""
    csrc = os.path.join(os.path.dirname(_lib.HEADER_PATH), "..", "firedancer_amd", "csrc")
    r = subprocess.run(["make", "-C", csrc, "stamps"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    so = os.path.join(os.path.dirname(_lib.HEADER_PATH), "..", "build", "stamps", "libfd_ed25519_gpu.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    assert "fdgpu_debug_stamps" in out and "fdgpu_submit" in out
