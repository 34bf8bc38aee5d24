"""Host-side sanitizers: the oracle's C restatement built with
clang's AddressSanitizer + UBSan (`make asan`), then (1) a deliberate
overflow proves the instrumentation is live and (2) the oracle's golden and
known-answer tests, including the full-grid respawn path, run clean under
it.  `make asan-test` runs the whole CPU suite this way, with libdronerl's
host code (C ABI validation) instrumented too."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang"


def _asan_env():
    rt = subprocess.run([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True, text=True,
                        check=True).stdout.strip()
    if not os.path.exists(rt):
        pytest.skip("clang ASan runtime not found")
    subprocess.run(["make", "-s", "-C", REPO, "build/asan/liboracle.so"], check=True, capture_output=True)
    return dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1",
                DRL_ORACLE_LIB=os.path.join(REPO, "build", "asan", "liboracle.so"), PYTHONPATH=REPO)


@pytest.fixture(scope="module")
def asan_env():
    if not os.path.exists(CLANG):
        pytest.skip("no ROCm clang")
    return _asan_env()


def test_asan_instrumentation_is_live(asan_env):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "asan_probe.py")], env=asan_env,
                       capture_output=True, text=True, timeout=120)
    assert "AddressSanitizer: heap-buffer-overflow" in r.stderr and "orc_set_state" in r.stderr
    assert "no report" not in r.stdout


def test_oracle_suite_clean_under_asan_ubsan(asan_env):
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_oracle_golden.py")], env=asan_env, capture_output=True,
                       text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert "passed" in r.stdout and "Sanitizer" not in r.stderr
