"""The per-call path (srtp_one.hip k_one): an unchanged libsrtp caller's
srtp_protect / srtp_unprotect of ONE packet (srtp/srtp.c:2493-2818,
2820-3172; AEAD 2088-2267, 2276-2491) runs one workgroup over a pinned copy
of the packet.  Every status and byte against the oracle's per-packet calls:
every built-in policy, payloads 0..1400 B with CSRCs and extensions, MKI
streams with several master keys, in place and not, then forged tags, a
bad MKI, replays and old packets on the receive side (a rejected packet's
buffer keeps its ciphertext), packets past the kernel's 4 KiB limit (the
batch path), and key usage."""
import random

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.test_gpu_parity import POLICIES, _gpu, policy, rtp_packet


def _packets(rng, ssrc, seq0, n, sizes=(0, 1, 15, 16, 17, 160, 1000, 1400)):
    out = []
    for k in range(n):
        out.append(rtp_packet(rng, ssrc, (seq0 + k) & 0xffff, rng.choice(sizes),
                              cc=rng.choice((0, 0, 1, 3)),
                              xwords=rng.choice((-1, -1, 0, 2))))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(POLICIES))
def test_single_calls_every_policy(name):
    _gpu()
    rng = random.Random(801 + len(name))
    ssrc = 0x31000000
    pols = [policy(name, ssrc=ssrc, seed=9)]
    lib, orc = L.Session(pols), O.Session(pols)
    rcv, orc_r = L.Session(pols), O.Session(pols)
    tag = POLICIES[name][4]
    pk = _packets(rng, ssrc, 0xffff - 20, 60)
    sent = []
    for k, p in enumerate(pk):
        inplace = k % 2 == 0
        rc, out = lib.protect(p, len(p) + 64, inplace=inplace)
        rc_o, ref = orc.protect(p, len(p) + 64)
        assert rc == rc_o == 0 and out == ref, (k, rc, rc_o)
        sent.append(ref)
    # the receive side: accepted, forged, replayed
    for k, p in enumerate(sent):
        if tag and k % 7 == 3:
            b = bytearray(p)
            b[-1] ^= 0x04
            p = bytes(b)
        inplace = k % 2 == 1
        rc, out = rcv.unprotect(p, len(p), inplace=inplace)
        rc_o, ref = orc_r.unprotect(p, len(p))
        assert rc == rc_o, (k, rc, rc_o)
        assert rc or out == ref, k
    # replays of accepted packets (replay_fail); a forged packet's original
    # is still new (accepted now)
    for k in (55, 56, 57, 58, 59, 0, 1):
        p = sent[k]
        rc, out = rcv.unprotect(p, len(p))
        rc_o, ref = orc_r.unprotect(p, len(p))
        assert rc == rc_o, (k, rc, rc_o)
        assert (rc != 0) == (not tag or k % 7 != 3), (k, rc)
        assert rc or out == ref, k
    assert lib.debug_key_left(ssrc) == (0, orc.key_left(ssrc)[1])
    assert rcv.debug_key_left(ssrc) == (0, orc_r.key_left(ssrc)[1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_single_calls_mki_keys_and_bad_mki(name):
    """MKI streams: each call's mki_index on protect, the packet's MKI on
    unprotect (srtp.c:1961-2016), an unknown MKI is bad_mki; per-key uses"""
    _gpu()
    rng = random.Random(803)
    ssrc = 0x31100000
    pols = [policy(name, ssrc=ssrc, seed=11, mki=4, nkeys=3)]
    lib, orc = L.Session(pols), O.Session(pols)
    rcv, orc_r = L.Session(pols), O.Session(pols)
    pk = _packets(rng, ssrc, 500, 30)
    sent = []
    for k, p in enumerate(pk):
        j = k % 3
        rc, out = lib.protect(p, len(p) + 64, mki_index=j)
        rc_o, ref = orc.protect(p, len(p) + 64, j)
        assert rc == rc_o == 0 and out == ref, (k, j)
        sent.append(ref)
    tag = POLICIES[name][4]
    back = 4 + (0 if name.startswith("gcm") else tag)
    for k, p in enumerate(sent):
        if k % 5 == 2:   # an MKI no key has
            b = bytearray(p)
            b[len(b) - back:len(b) - back + 4] = b"\xee" * 4
            p = bytes(b)
        rc, out = rcv.unprotect(p, len(p), inplace=k % 2 == 0)
        rc_o, ref = orc_r.unprotect(p, len(p))
        assert rc == rc_o, (k, rc, rc_o)
        assert rc or out == ref, k
    for j in range(3):
        assert lib.debug_key_left(ssrc, j) == (0, orc.key_left(ssrc, j)[1])
        assert rcv.debug_key_left(ssrc, j) == (0, orc_r.key_left(ssrc, j)[1])


@pytest.mark.gpu
def test_single_calls_in_place_rejected_buffer_kept_and_large_packets():
    """in place, a rejected packet's buffer keeps the ciphertext; packets
    past SRTP_ONE_MAX (4 KiB) take the batch path, with the same bytes"""
    import ctypes as C
    _gpu()
    rng = random.Random(805)
    ssrc = 0x31200000
    for name in ("icm128_hmac80", "gcm128_16"):
        pols = [policy(name, ssrc=ssrc, seed=13)]
        lib, orc = L.Session(pols), O.Session(pols)
        rcv, orc_r = L.Session(pols), O.Session(pols)
        pk = _packets(rng, ssrc, 77, 6, sizes=(1400, 4000, 5000, 9000))
        for p in pk:
            rc, out = lib.protect(p, len(p) + 64)
            rc_o, ref = orc.protect(p, len(p) + 64)
            assert rc == rc_o == 0 and out == ref, len(p)
            b = bytearray(ref)
            b[-1] ^= 1
            forged = bytes(b)
            buf = C.create_string_buffer(forged, len(forged))
            n = C.c_size_t(len(forged))
            st = rcv.L.srtp_unprotect(rcv.h, buf, len(forged), buf, C.byref(n))
            assert st == orc_r.unprotect(forged, len(forged))[0] == 7
            assert buf.raw[:len(forged)] == forged, "rejected packet changed"
            rc, out = rcv.unprotect(ref, len(ref), inplace=True)
            rc_o, back = orc_r.unprotect(ref, len(ref))
            assert rc == rc_o == 0 and out == back == p
