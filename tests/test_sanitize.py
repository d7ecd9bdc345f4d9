"""ASan + UBSan over the host C/C++ code: the library's host sources
(csrc/pack.cpp, csrc/abi.cpp) and the oracle's C restatement, driven by
tools/sanitize/host_check.cpp on random and edge-case inputs (empty graphs, one-row /
one-column graphs, duplicates and out-of-range ids rejected, strided FC operands).  Any
sanitizer report aborts the harness (-fno-sanitize-recover=all)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="no host toolchain")
def test_host_code_under_asan_ubsan():
    d = os.path.join(ROOT, "tools", "sanitize")
    b = subprocess.run(["make", "-C", d, "all"], capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    # verify_asan_link_order=0: the environment may preload a library of its own ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(d, "build", "host_check")], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host sanitizer checks: ok" in r.stdout
