"""the native C++ runtime (keccak, PNG, H.264 I_PCM, secp256k1) built with
AddressSanitizer + UBSan on the CPU, every entry point exercised against its Python reference."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_native_runtime_clean_under_asan_ubsan(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "sanitize_native.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "all entry points clean" in r.stdout
