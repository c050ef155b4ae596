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
    assert len(names) == 51, names          # + fdgpu_build_info (round 6)
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
          "KEY_CACHE": ed.FLAG_KEY_CACHE, "PAIR": ed.FLAG_PAIR, "PAIR_AUTO": ed.FLAG_PAIR_AUTO,
          "MERGE": ed.FLAG_MERGE, "SPREAD": ed.FLAG_SPREAD, "SPREAD_AUTO": ed.FLAG_SPREAD_AUTO}
    assert hdr == py, (hdr, py)


def test_shipped_library_is_product_build():
    """fdgpu_build_info() of the library smoke() and bench.py load: every A/B
    switch at its shipped default, no fault injection; the stamps variant is
    reported as not a product build (so the guard is not vacuous)."""
    info = _lib.build_info()
    assert info["product"] == 1, info
    assert (info["verify_waves"], info["atab_words"], info["tab_store_nt"], info["tab_load_cpol"], info["ws_slot"],
            info["phase_stamps"], info["debug_drop_flag"]) == (2, 40, 0, 0, 0, 0, 0), info
    assert _lib.require_product_build() == info
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = ("import json, sys; sys.path.insert(0, {r!r}); from firedancer_amd import _lib; "
             "print(json.dumps(_lib.build_info()))").format(r=repo)
    stamps = os.path.join(repo, "build", "stamps", "libfd_ed25519_gpu.so")
    if os.path.exists(stamps):
        r = subprocess.run(["python", "-c", probe], capture_output=True, text=True, env={**os.environ, "FDGPU_LIB": stamps})
        assert r.returncode == 0, r.stderr
        import json
        st = json.loads(r.stdout)
        assert st["phase_stamps"] == 1 and st["product"] == 0, st
    r = subprocess.run(["python", "-c", probe], capture_output=True, text=True,
                       env={**os.environ, "FDGPU_DEBUG_DROP_FLAG": "1"})
    assert '"product": 0' in r.stdout and '"debug_drop_flag": 1' in r.stdout, r.stdout + r.stderr
    # no wrong-code diagnostic switch is left in the product sources
    csrc = os.path.join(repo, "firedancer_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h", ".cpp")):
            assert "FDGPU_DIAG_" not in open(os.path.join(csrc, f)).read(), f


def test_stamps_variant_builds():
    """The one kernel variant kept (per-phase stamps for tools/phase_stamps.py)
    still compiles for gfx950 and exports its stamp reader."""
    csrc = os.path.join(os.path.dirname(_lib.HEADER_PATH), "..", "firedancer_amd", "csrc")
    r = subprocess.run(["make", "-C", csrc, "stamps"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    so = os.path.join(os.path.dirname(_lib.HEADER_PATH), "..", "build", "stamps", "libfd_ed25519_gpu.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    assert "fdgpu_debug_stamps" in out and "fdgpu_submit" in out


_SYNC_CALL = r"""
import ctypes, os, sys
sys.path.insert(0, {repo!r})
from firedancer_amd import _lib
L = _lib.lib()
rc = L.fd_ed25519_verify(b"abc", 3, bytes(64), bytes(32), None)
print("rc", rc, "errors", L.fdgpu_sync_errors(), flush=True)
"""


def _sync_child(env_extra):
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k != "FDGPU_SYNC_FAIL_CLOSED"}
    env.update(FDGPU_SYNC_DEVICE="99", **env_extra)
    return subprocess.run(["python", "-c", _SYNC_CALL.format(repo=repo)], capture_output=True, text=True, env=env,
                          timeout=120)


def test_sync_api_engine_failure_aborts_by_default():
    """The reference's fd_ed25519_verify never answers a good signature with
    an error, so an engine failure (here: no device 99, on any machine) aborts
    the process with the reason on stderr rather than returning a verdict."""
    r = _sync_child({})
    assert r.returncode == -6, (r.returncode, r.stdout, r.stderr[-500:])
    assert "fd_ed25519_gpu:" in r.stderr and "FDGPU_SYNC_FAIL_CLOSED" in r.stderr
    assert "rc" not in r.stdout


def test_sync_api_fail_closed_opt_in():
    """FDGPU_SYNC_FAIL_CLOSED=1: the failed call returns FD_ED25519_ERR_SIG
    and fdgpu_sync_errors() counts it."""
    r = _sync_child({"FDGPU_SYNC_FAIL_CLOSED": "1"})
    assert r.returncode == 0, r.stderr[-500:]
    assert r.stdout.split() == ["rc", "-1", "errors", "1"]


def test_frag_io_structs_layout():
    """fdgpu_frag_io_t (32 B: src, sz, out_off, out_cap, link, seq) and
    fdgpu_link_t (16 B) as C sees them match the Python dtypes."""
    from firedancer_amd import ed25519 as ed, tile
    src = (f'#include "{_lib.HEADER_PATH}"\n#include <stddef.h>\n'
           '_Static_assert(sizeof(fdgpu_frag_io_t) == 32, "io");\n'
           '_Static_assert(offsetof(fdgpu_frag_io_t, link) == 20 && offsetof(fdgpu_frag_io_t, seq) == 24, "io");\n'
           '_Static_assert(sizeof(fdgpu_link_t) == 16, "link");\nint main(void){ return 0; }\n')
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-x", "c", "-", "-fsyntax-only"], input=src,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert ed.FRAG_IO_DTYPE.itemsize == tile.FRAG_IO_DTYPE.itemsize == 32
    assert ed.FRAG_IO_DTYPE.fields["seq"][1] == 24 and ed.LINK_DTYPE.itemsize == 16
