"""Session keys derived on the GPU (k_kdf, srtp_gpu_kdf: the SRTP KDF of
srtp.c:1070-1142 and the key setup of srtp_stream_init_keys 1233-1607 for
every stream of a srtp_create / srtp_update in one launch) against the same
keys derived on the host (SRTP_MI355X_HOST_KDF=1, host_crypto.c): the
device key records must be identical, which every packet shows -- RTP and
SRTCP outputs of both sessions are compared byte for byte, for every cipher
family and key size, MKI, RFC 6904 (its AES-GCM PRF with the padded salt),
and a 4096-stream session rekeyed by srtp_update.  The golden-fixture tests
(tests/test_gpu_parity.py etc.) run on GPU-derived keys as well."""
import os
import random

import pytest

import libsrtp_amd as L
from tests.test_gpu_parity import policy, rtp_packet

pytestmark = pytest.mark.gpu


def _gpu():
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")


def _session(pols, host):
    old = os.environ.get("SRTP_MI355X_HOST_KDF")
    os.environ["SRTP_MI355X_HOST_KDF"] = "1" if host else "0"
    try:
        return L.Session(pols)
    finally:
        if old is None:
            del os.environ["SRTP_MI355X_HOST_KDF"]
        else:
            os.environ["SRTP_MI355X_HOST_KDF"] = old


def _traffic(s, ssrcs, rng, n=6):
    out = []
    for ssrc in ssrcs:
        for k in range(n):
            p = rtp_packet(rng, ssrc, 100 + k, rng.choice([0, 17, 160, 1400]),
                           cc=k % 2, xwords=1 if k % 3 == 0 else -1)
            out.append(s.protect(p))
            rtcp = bytes([0x81, 0xc8, 0, 6]) + ssrc.to_bytes(4, "big") + \
                rng.randbytes(20)
            out.append(s.protect_rtcp(rtcp))
    return out


NAMES = ["icm128_hmac80", "icm128_hmac32", "icm128_nullauth", "null_hmac80",
         "icm192_hmac80", "icm256_hmac80", "icm128_authonly", "gcm128_16",
         "gcm256_16", "gcm256_8"]


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("variant", ["plain", "mki", "xtn"])
def test_gpu_kdf_matches_host_kdf(name, variant):
    _gpu()
    kw = {}
    if variant == "mki":
        kw = dict(mki=4, nkeys=3)
    pol = policy(name, seed=7, **kw)
    if variant == "xtn":
        pol["enc_xtn_hdr"] = [1, 2, 3, 4, 5]
    a, b = _session([pol], False), _session([pol], True)
    ra, rb = random.Random(1), random.Random(1)
    ta, tb = _traffic(a, [0xcafebabe], ra), _traffic(b, [0xcafebabe], rb)
    assert ta == tb
    # (random extension bytes are often malformed RFC 8285 elements: the
    # header-extension walk reports parse_err for them, identically)
    ok = {L.Status.ok, L.Status.no_such_op} | \
        ({L.Status.parse_err} if variant == "xtn" else set())
    assert all(st in ok for st, _ in ta)
    assert sum(st == 0 for st, _ in ta) >= len(ta) // 3


def test_gpu_kdf_mass_rekey():
    """4096 streams with distinct keys created in one call, then all rekeyed
    by one srtp_update: GPU- and host-derived sessions agree on every
    stream."""
    _gpu()
    n = 4096
    ssrcs = [0x10000 + i for i in range(n)]
    pols = [policy("icm128_hmac80", ssrc=s, seed=s) for s in ssrcs]
    a, b = _session(pols, False), _session(pols, True)
    rng = random.Random(3)
    pick = rng.sample(ssrcs, 64)
    assert _traffic(a, pick, random.Random(4), 2) == \
        _traffic(b, pick, random.Random(4), 2)
    new = [policy("gcm256_16", ssrc=s, seed=s + 1) for s in ssrcs]
    # srtp_update keeps the streams' index: same pending state in both
    assert a.update_all(new) == 0 and b.update_all(new) == 0
    assert _traffic(a, pick, random.Random(5), 2) == \
        _traffic(b, pick, random.Random(5), 2)
