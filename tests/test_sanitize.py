"""The host tile library -- the code that parses untrusted frags (fd_txn_parse,
TPU reassembly, tcache, the verify / dedup / mux tiles) -- built with
AddressSanitizer + UndefinedBehaviorSanitizer (make -C firedancer_amd/csrc
sanitize; the reference's config/extra/with-asan.mk and with-ubsan.mk), and
the CPU tests of those layers re-run against it in a child process with the
sanitizer runtimes preloaded.  Any ASan report or UBSan runtime error fails
the child (halt_on_error)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_LIB = os.path.join(REPO, "build", "asan", "libfd_verify_tile.so")


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.slow
def test_tile_layers_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "firedancer_amd", "csrc"), "sanitize"], check=True)
    env = dict(os.environ, LD_PRELOAD=f"{asan} {ubsan}", FDGPU_TILE_LIB=ASAN_LIB,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    tests = [os.path.join(REPO, "tests", t) for t in
             ("test_tile.py", "test_reasm.py", "test_mux.py", "test_callers.py", "test_engine_proc.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider"]
                       + tests, env=env, cwd=REPO, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
