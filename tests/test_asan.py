"""Host AddressSanitizer + UBSan runs of the CPU code (SURVEY.md §5
sanitizer row; no GPU code is instrumented): tools/asan/Makefile builds
csrc/layout_graph.cpp and oracle/grl_oracle.c with
-fsanitize=address,undefined, then
  * tools/asan/run_layout.py drives the layout builder over every fixture
    page and edge type (outputs equal to the reference's), and
  * the oracle test suite (tests/test_oracle.py) runs on the ASan oracle,
each in a child Python with LD_PRELOAD=libasan (leak checks off: the
interpreter itself leaks by design).  Any memory error or UB aborts the
child, and the test fails with its report."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _runtime(name):
    cc = shutil.which("gcc")
    if cc is None:
        return None
    p = subprocess.run([cc, f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def asan_env():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc's ASan/UBSan runtimes are not installed")
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "tools", "asan")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=87",
               GRL_ORACLE_LIB=os.path.join(ROOT, "build", "asan", "libgrl_oracle_asan.so"),
               PYTHONDONTWRITEBYTECODE="1")
    return env


def _check(r):
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]


def test_layout_builder_under_asan(asan_env):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asan", "run_layout.py")], env=asan_env,
                       capture_output=True, text=True, timeout=600)
    _check(r)
    assert "adjacencies equal the reference" in r.stdout


def test_oracle_suite_under_asan(asan_env):
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-x",
                        os.path.join(ROOT, "tests", "test_oracle.py")], env=asan_env, cwd=ROOT,
                       capture_output=True, text=True, timeout=900)
    _check(r)
    assert " passed" in r.stdout
