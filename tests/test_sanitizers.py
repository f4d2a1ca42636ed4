"""Sanitizer builds of libtsg's host code and the oracle, on the CPU (the
reference runs `go test -race`, /root/reference/Makefile:27). GPU sanitizers are not available on
the MI355X pool, so the HIP entry points are replaced by tests/sanitize/host_stub.cpp (test
infrastructure, never in libtsg.so) and the host code runs under:

- AddressSanitizer + UBSan: the search-block loader on synthetic blocks and under a corruption
  fuzz of all four files; the reference's v2 blocks (tests/golden) index and data pages, snappy
  and zstd, fuzzed; snappy round trips (san_host);
- ThreadSanitizer and ASan: many threads through tsg_search (the coalescer's leaders and parked
  waiters, park.hpp), limit waves, tsg_search_batch's workers, the result-holder pool and the
  frontend merge, every result checked against the same search run alone (san_coal);
- ASan + UBSan under the CPU tests that drive the library and the oracle (a subprocess with the
  sanitized libtsg.so and liboracle.so).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "build", "san")
CLANG = "/opt/rocm/llvm/bin/clang++"

pytestmark = pytest.mark.skipif(not os.path.exists(CLANG), reason="no clang++ with the sanitizer runtimes")


@pytest.fixture(scope="module")
def built():
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.check_call(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "tests", "sanitize"), "all"])
    return SAN


def _run(cmd, env=None, timeout=600):
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run(cmd, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-6000:]
    for bad in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer"):
        assert bad not in p.stdout, p.stdout[-6000:]
    return p.stdout


def test_loader_and_decoders_under_asan(built, tmp_path):
    out = _run([os.path.join(built, "san_host"), str(tmp_path), os.path.join(ROOT, "tests", "golden"), "150"],
               {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert "san_host: ok" in out
    assert "tempo_cli: 611 records, 611 pages decoded" in out


def test_concurrent_searches_under_tsan(built, tmp_path):
    out = _run([os.path.join(built, "san_coal_tsan"), str(tmp_path), "10", "20"],
               {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    assert "0 mismatches" in out


def test_concurrent_searches_under_asan(built, tmp_path):
    out = _run([os.path.join(built, "san_coal_asan"), str(tmp_path), "8", "20"],
               {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})
    assert "0 mismatches" in out


def test_cpu_tests_under_asan(built):
    rt = subprocess.check_output([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], text=True).strip()
    assert os.path.exists(rt), rt
    env = {"LD_PRELOAD": rt, "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1",
           "TSG_LIB_PATH": os.path.join(built, "lib", "libtsg.so"),
           "ORACLE_LIB_PATH": os.path.join(built, "liboracle_asan.so")}
    tests = ["tests/test_abi.py", "tests/test_oracle_golden.py", "tests/test_live_oracle.py", "tests/test_wal_oracle.py",
             "tests/test_zstd_host.py"]
    out = _run([sys.executable, "-m", "pytest", "-x", "-q", "-s", "-m", "not gpu", "-p", "no:cacheprovider"] + tests,
               env, timeout=900)
    assert " passed" in out and "failed" not in out
