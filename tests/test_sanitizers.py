"""Race / memory-error detection for the native host runtime: the TCPStore server+clients,
comm watchdog and host tracer, hammered from many threads by csrc/runtime/stress/runtime_stress.cpp, built
with ThreadSanitizer and with AddressSanitizer+UBSan (paddle2_amd._build.build_sanitized).  Host code only
(GPU sanitizers are not used on this hardware).  Any sanitizer report fails the test."""
import shutil
import subprocess

import pytest

from paddle2_amd import _build


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("kind", ["thread", "address"])
def test_runtime_under_sanitizer(kind):
    exe = _build.build_sanitized(kind)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    reports = [ln for ln in r.stderr.splitlines() if "SUMMARY:" in ln or "ERROR: AddressSanitizer" in ln]
    assert r.returncode == 0 and not reports, "\n".join(reports) or r.stderr[-3000:]
    assert "runtime_stress OK" in r.stdout
