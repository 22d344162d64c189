"""ASan/UBSan and TSan builds of the host native code run their self-test."""
from __future__ import annotations

import os
import subprocess

import pytest

from downloader_amd.ops import build


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_native_selftest_under_sanitizer(kind):
    exe = build.build_selftest(kind, verbose=False)
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan
    # runtime; that is tolerated rather than changing the environment.
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "selftest ok" in r.stdout
