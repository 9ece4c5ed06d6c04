"""Packets longer than one counter-cache epoch.

The kernels cache AES rounds 1-2 for the blocks of a packet that share
counter bytes 0..14 (256 keystream blocks = 4 KiB of payload; GCM's BE32
counter starts at 2); past that the steady / cooperative paths hand the
rest of the packet to the general path with full AES.  These batches cross
that boundary -- mixed sizes, and a uniform batch (all 64 lanes of a wave
alike, so the wave-cooperative path runs up to the boundary) -- and are
compared byte for byte with the oracle, then unprotected back.
"""
import random

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.test_gpu_parity import _gpu, policy, rtp_packet

pytestmark = pytest.mark.gpu

NAMES = ["icm128_hmac80", "icm256_hmac32", "gcm128_16", "gcm256_16"]


def _roundtrip(name, pkts):
    pol = policy(name, seed=3)
    lib_s, orc_s = L.Session([pol]), O.Session([pol])
    st, out = lib_s.protect_batch(pkts)
    srtp = []
    for i, p in enumerate(pkts):
        rc, ref = orc_s.protect(p, len(p) + 144)
        assert st[i] == rc == 0, (i, st[i], rc)
        assert out[i] == ref, i
        srtp.append(ref)
    lib_r = L.Session([pol])
    st, back = lib_r.unprotect_batch(srtp)
    for i in range(len(srtp)):
        assert st[i] == 0 and back[i] == pkts[i], i


@pytest.mark.parametrize("name", NAMES)
def test_jumbo_mixed_sizes(name):
    _gpu()
    rng = random.Random(name)
    sizes = [4064, 4079, 4080, 4095, 4096, 4100, 5000, 8191, 9000, 1400]
    pkts = [rtp_packet(rng, 0xcafebabe, 0x100 + i, sizes[i % len(sizes)],
                       rng.choice([0, 1]), rng.choice([-1, 0]))
            for i in range(80)]
    _roundtrip(name, pkts)


@pytest.mark.parametrize("name", NAMES)
def test_jumbo_uniform_wave(name):
    _gpu()
    rng = random.Random(name + "u")
    pkts = [rtp_packet(rng, 0xcafebabe, (0xfff0 + i) & 0xffff, 5000)
            for i in range(128)]
    _roundtrip(name, pkts)
