"""Host AddressSanitizer + UndefinedBehaviorSanitizer run (SURVEY.md 5 "Race detection /
sanitizers"): `make san` instruments the scene stage, octree builder, layout compilers, host
ABI, the kernel's per-pixel code compiled for the host, the group row map and the oracle
(clang, -fsanitize=address,undefined, leak detection on) and runs tests/cpp/san_check.cpp,
which renders small frames through the emulation and the oracle and compares bits.  CPU only:
GPU sanitizers are not available on this pool."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.slow
def test_asan_ubsan_host_build():
    r = subprocess.run(["make", "-C", str(ROOT), "-j8", "san"], capture_output=True, text=True, timeout=1200)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "san_check: all cases passed" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out
