"""The engine's parallel descriptor expansion (expand_par, used by
fdgpu_submit for batches of >= 65,536 txns) against its serial expand():
byte-identical signature descriptors, txn descriptors and block-count
permutation on random batches (skipped 0 / >16-signature txns included),
and the same error -- the first failing txn in order -- for out-of-bounds
descriptors and max_sig overflows.  CPU only: tools/expand_check.cpp
compiles the engine source for the host (hipcc) and calls both."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_expand_par_equals_expand(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    lib = os.path.join(REPO, "firedancer_amd", "libfd_ed25519_gpu.so")
    if not os.path.exists(hipcc) or not os.path.exists(lib):
        pytest.skip("hipcc or the engine library is missing")
    exe = str(tmp_path / "expand_check")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-x", "hip", os.path.join(REPO, "tools", "expand_check.cpp"), "-o", exe,
                    "-L", os.path.dirname(lib), "-l:libfd_ed25519_gpu.so",
                    "-Wl,-rpath," + os.path.dirname(lib)], check=True, capture_output=True, timeout=600)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-3000:]
    assert "DIFFER" not in r.stdout
