"""The C++ host mirror (include/xdrg_host.hpp, libxdrg_host.so) and its test
program tests/cpp/test_xdr_host.cpp, which restates the reference's XDR unit
tests (XdrIntTest, XdrLongTest, XdrOpaqueTest, XdrTest) against the GPU engine."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTLIB = os.path.join(ROOT, "oncrpc4j_amd", "libxdrg_host.so")
TESTBIN = os.path.join(ROOT, "tests", "cpp", "build", "test_xdr_host")


def test_host_library_exports_the_mirror():
    out = subprocess.run(["nm", "-DC", "--defined-only", HOSTLIB], capture_output=True, text=True,
                         check=True).stdout
    for sym in ("oncrpc4j::xdr::BatchXdrEncoder::flush", "oncrpc4j::xdr::BatchXdrDecoder::load",
                "oncrpc4j::xdr::BatchXdrEncoder::xdrEncodeInt", "oncrpc4j::xdr::BatchXdrDecoder::xdrDecodeString",
                "oncrpc4j::xdr::schemaOf", "oncrpc4j::xdr::Engine::Engine"):
        assert sym in out, sym
    assert os.access(TESTBIN, os.X_OK)


@pytest.mark.gpu
def test_reference_unit_tests_in_cpp():
    r = subprocess.run([TESTBIN], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
