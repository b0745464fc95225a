"""ASan + UBSan builds: the oracle driven over random schemas,
truncated and corrupted streams (oracle/san_driver.c), and the product's
host-only code — the C-ABI schema compiler / argument validation and the C++
mirror's XdrBuffer growth (tests/cpp/san_host.cpp).  CPU only; GPU kernels are
not instrumented (no GPU sanitizer on this pool)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build_and_run(make_dir, binary, args=()):
    subprocess.run(["make", "-s", "-C", make_dir, "sanitize"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([binary, *args], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


def test_oracle_under_asan_ubsan():
    out = _build_and_run(os.path.join(ROOT, "oracle"), os.path.join(ROOT, "oracle", "_san", "san_driver"),
                         ["400"])
    assert "400 batch rounds ok" in out


def test_host_code_under_asan_ubsan():
    out = _build_and_run(os.path.join(ROOT, "oncrpc4j_amd", "csrc"),
                         os.path.join(ROOT, "oncrpc4j_amd", "csrc", "build", "san", "san_host"))
    assert "san_host: ok" in out


def test_host_staging_pipeline_under_asan_ubsan():
    """XDRG_HOST_PTRS bookkeeping (oncrpc4j_amd/csrc/host_stage.h): chunking,
    slot layout, bounce copies, rebasing, ring growth, CAPACITY and first-bad
    errors, run with the oracle as the kernels and checked against the oracle
    on whole batches (tests/cpp/san_stage.cpp)."""
    out = _build_and_run(os.path.join(ROOT, "oncrpc4j_amd", "csrc"),
                         os.path.join(ROOT, "oncrpc4j_amd", "csrc", "build", "san", "san_stage"), ["400"])
    assert "400 rounds ok" in out
