"""The crypto-kernel plugin ABI (srtp.def:46-69): tests/c/plugin_test.c,
built by build() / `make -C libsrtp_amd relay`, run against the GPU-backed
built-in types, the published vectors, the reference's own known answers
(its srtp_aes_* / srtp_hmac test_data, read from oracle/_ref), replacement
semantics and the packet path after a replacement."""
import os
import subprocess

import pytest

import libsrtp_amd as L

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c", "plugin_test")
REF = os.path.join(ROOT, "oracle", "_ref", "libsrtp_ref_ossl.so")


def test_plugin_abi():
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")
    assert os.path.exists(BIN), "build() makes tests/c/plugin_test"
    args = [BIN] + ([REF] if os.path.exists(REF) else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout
    if os.path.exists(REF):
        assert r.stdout.count("through the GPU type: ok") == 7
