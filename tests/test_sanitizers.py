"""the native runtime (engine batcher, HTTP server, load generator) under
AddressSanitizer+UBSan and ThreadSanitizer, host-side, on the CPU backend (tools/sanitize.sh)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(not (os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("hipcc")), reason="needs hipcc")
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_native_runtime_under_sanitizer(kind):
    out = subprocess.run(["bash", str(ROOT / "tools" / "sanitize.sh"), kind], capture_output=True, text=True,
                         timeout=900, cwd=ROOT)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "stress OK" in out.stdout
