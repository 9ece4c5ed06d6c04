"""Adversarial receive path: forged packets inside unprotect batches.

The reference authenticates each packet before it moves the replay window
(srtp.c:2994-3053, then 3157-3167), so a forged packet must change nothing.
The GPU library speculates that packets authenticate and re-runs those whose
index estimate moved; these tests check that forged traffic with advancing
sequence numbers (the case that defeats speculation) gives the reference's
statuses and bytes (through the oracle, one call per packet), that the number
of post-pass rounds / launches stays bounded, and that the buffer of every
rejected packet holds its ciphertext again -- never unauthenticated
plaintext."""
import random

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.test_gpu_parity import _gpu, policy, rtp_packet

pytestmark = pytest.mark.gpu
SSRC = 0x0badcafe


def _traffic(rng, name, n, forge_rate, forge_seq):
    """genuine packets (protected by the oracle sender) in order with forged
    ones inserted; forge_seq(cur_seq, k) gives the k-th forgery's seq"""
    pol = policy(name, ssrc=SSRC, seed=7)
    snd = O.Session([pol])
    out, plain, kinds, seq, nf = [], [], [], 0xff00, 0
    for i in range(n):
        p = rtp_packet(rng, SSRC, seq & 0xffff, rng.choice([20, 160, 1200]))
        rc, s = snd.protect(p, len(p) + 64)
        assert rc == 0
        out.append(s)
        plain.append(p)
        kinds.append("genuine")
        if rng.random() < forge_rate:
            fs = forge_seq(seq, nf) & 0xffff
            f = rtp_packet(rng, SSRC, fs, 160) + rng.randbytes(16)
            out.append(f)
            plain.append(None)
            kinds.append("forged")
            nf += 1
        seq += 1
    return pol, out, plain, kinds


def _oracle_recv(pol, pkts):
    rcv = O.Session([pol])
    return [rcv.unprotect(p, len(p)) for p in pkts]


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_forged_10pct_advancing_seq(name):
    _gpu()
    rng = random.Random(11)
    pol, pk, plain, kinds = _traffic(
        rng, name, 4000, 0.10, lambda cur, k: cur + rng.randrange(1, 3000))
    ref = _oracle_recv(pol, pk)
    lib = L.Session([pol])
    st, out = lib.unprotect_batch(pk)
    for i, (rc, o) in enumerate(ref):
        assert int(st[i]) == rc, (i, kinds[i], int(st[i]), rc)
        if rc == 0:
            assert out[i] == o, i
    assert sum(1 for k, s in zip(kinds, st) if k == "forged" and s == 0) == 0
    rounds, launches, _ = lib.unprotect_stats()
    assert rounds <= 5 and launches <= 5, (rounds, launches)


def test_forged_chain_is_bounded():
    """each forgery makes the next one look old (30000, 29800, ...): with
    optimistic speculation alone every forgery costs a round"""
    _gpu()
    rng = random.Random(12)
    pol, pk, plain, kinds = _traffic(
        rng, "icm128_hmac80", 3000, 0.05,
        lambda cur, k: 0xff00 + 30000 - 200 * k)
    ref = _oracle_recv(pol, pk)
    lib = L.Session([pol])
    st, out = lib.unprotect_batch(pk)
    assert [int(s) for s in st] == [rc for rc, _ in ref]
    for i, (rc, o) in enumerate(ref):
        if rc == 0:
            assert out[i] == o, i
    rounds, launches, _ = lib.unprotect_stats()
    assert rounds <= 6 and launches <= 6, (rounds, launches)


def _device_unprotect(lib, pkts, inplace):
    import torch
    offs, pos = [], 0
    for p in pkts:
        offs.append(pos)
        pos += (len(p) + 15) & ~15
    buf = bytearray(pos + 16)
    for o, p in zip(offs, pkts):
        buf[o:o + len(p)] = p
    arena = torch.frombuffer(buf, dtype=torch.uint8).cuda()
    dst = arena if inplace else torch.full_like(arena, 0x3c)
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    cap = ln.clone()
    st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    assert lib.unprotect_device(arena, off, ln, dst, off, cap, st) == 0
    host = dst.cpu().numpy().tobytes()
    return st.cpu().tolist(), cap.cpu().tolist(), host, offs


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm128_16"])
@pytest.mark.parametrize("inplace", [True, False], ids=["inplace", "outofplace"])
def test_rejected_buffers_hold_no_plaintext(name, inplace):
    _gpu()
    rng = random.Random(13)
    pol, pk, plain, kinds = _traffic(
        rng, name, 2000, 0.10, lambda cur, k: cur + rng.randrange(1, 40))
    # tamper 5% of the genuine packets too (payload bit flip)
    for i in range(len(pk)):
        if kinds[i] == "genuine" and rng.random() < 0.05:
            b = bytearray(pk[i])
            b[len(b) // 2] ^= 0x10
            pk[i] = bytes(b)
            kinds[i] = "tampered"
    ref = _oracle_recv(pol, pk)
    lib = L.Session([pol])
    st, olen, host, offs = _device_unprotect(lib, pk, inplace)
    tag = 16 if name.startswith("gcm") else 10
    nrej = 0
    for i, (rc, o) in enumerate(ref):
        assert st[i] == rc, (i, kinds[i], st[i], rc)
        got = host[offs[i]:offs[i] + len(pk[i])]
        if rc == 0:
            assert olen[i] == len(o) and got[:len(o)] == o, i
            continue
        nrej += 1
        body = len(pk[i]) - tag
        if inplace:
            assert got == pk[i], (i, kinds[i])    # ciphertext restored
        elif kinds[i] == "tampered":
            # never the plaintext; where the crypto ran, the ciphertext
            assert got[12:body] != plain[i][12:body], i
            assert got[12:body] in (pk[i][12:body], bytes([0x3c]) * (body - 12))
    assert nrej > 100


# --------------------------------------------------------------------------
# the device unprotect pre-pass (srtp_gpu_pp_unprotect): receive batches of
# known streams stay on the GPU, forged / tampered packets included

def _multi_stream_batches(rng, name, ns, per, nbatch, tamper):
    ssrcs = [0x30000000 + 11 * k for k in range(ns)]
    pols = [policy(name, ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    snd = O.Session(pols)
    seq = {s: rng.randrange(1, 0x10000) for s in ssrcs}
    batches = []
    for _ in range(nbatch):
        order = [s for s in ssrcs for _ in range(per)]
        rng.shuffle(order)
        pk, kinds = [], []
        for s in order:
            p = rtp_packet(rng, s, seq[s] & 0xffff, rng.choice([0, 20, 160]))
            seq[s] += 1
            rc, sp = snd.protect(p, len(p) + 64)
            assert rc == 0
            if rng.random() < tamper:
                b = bytearray(sp)
                b[-1] ^= 0x40
                sp = bytes(b)
                kinds.append("tampered")
            else:
                kinds.append("genuine")
            pk.append(sp)
        batches.append((pk, kinds))
    return pols, batches


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16", "null_hmac80"])
@pytest.mark.parametrize("inplace", [True, False], ids=["inplace", "outofplace"])
def test_device_unprotect_prepass(name, inplace):
    _gpu()
    rng = random.Random(14)
    pols, batches = _multi_stream_batches(rng, name, 40, 30, 3, 0.05)
    lib, orc = L.Session(pols), O.Session(pols)
    for bi, (pk, kinds) in enumerate(batches):
        ref = [orc.unprotect(p, len(p)) for p in pk]
        st, olen, host, offs = _device_unprotect(lib, pk, inplace)
        for i, (rc, o) in enumerate(ref):
            assert st[i] == rc, (bi, i, kinds[i], st[i], rc)
            got = host[offs[i]:offs[i] + len(pk[i])]
            if rc == 0:
                assert olen[i] == len(o) and got[:len(o)] == o, (bi, i)
            elif inplace:
                assert got == pk[i], (bi, i)     # ciphertext restored
    assert lib.prepass_stats() == (3, 0), lib.prepass_last_abort()
    # state left by the device is what the host path continues from
    _, more = _multi_stream_batches(random.Random(15), name, 40, 2, 1, 0)
    for p in more[0][0][:20]:
        assert lib.unprotect(p, len(p))[0] == orc.unprotect(p, len(p))[0]


def test_device_unprotect_replayed_batch_goes_to_host():
    _gpu()
    rng = random.Random(16)
    pols, batches = _multi_stream_batches(rng, "icm128_hmac80", 8, 20, 2, 0)
    lib, orc = L.Session(pols), O.Session(pols)
    pk = batches[0][0]
    for p in pk:
        orc.unprotect(p, len(p))
    st, _, _, _ = _device_unprotect(lib, pk, False)
    assert st == [0] * len(pk)
    # the same packets again: every one a replay (host path decides)
    ref = [orc.unprotect(p, len(p))[0] for p in pk]
    st, _, _, _ = _device_unprotect(lib, pk, False)
    assert st == ref and set(ref) == {9}
    assert lib.prepass_stats() == (1, 1)


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
@pytest.mark.parametrize("inplace", [True, False], ids=["inplace", "outofplace"])
def test_device_unprotect_chain_one_stream(name, inplace):
    """one stream, more packets than the replay window: the chain form
    (stream order, advances, segmented sum; acceptance checked against the
    highest authenticated index before each packet)"""
    _gpu()
    rng = random.Random(17)
    pols, batches = _multi_stream_batches(rng, name, 1, 3000, 2, 0.05)
    lib, orc = L.Session(pols), O.Session(pols)
    for bi, (pk, kinds) in enumerate(batches):
        ref = [orc.unprotect(p, len(p)) for p in pk]
        st, olen, host, offs = _device_unprotect(lib, pk, inplace)
        for i, (rc, o) in enumerate(ref):
            assert st[i] == rc, (bi, i, kinds[i], st[i], rc)
            got = host[offs[i]:offs[i] + len(pk[i])]
            if rc == 0:
                assert got[:len(o)] == o, (bi, i)
            elif inplace:
                assert got == pk[i], (bi, i)
    assert lib.prepass_stats() == (2, 0), lib.prepass_last_abort()
    assert lib.get_roc(0x30000000)[1] == orc.get_roc(0x30000000)[1]


def test_device_unprotect_chain_long_rejected_run_goes_to_host():
    """forged packets advancing the chain by 3 x 20000 indices: from the
    second one on, the reference's guess from the last accepted index
    (above 2^15, so with ROC inference) differs from the chain's -- the
    host path decides"""
    _gpu()
    rng = random.Random(18)
    pol = policy("icm128_hmac80", ssrc=SSRC, seed=3)
    snd, orc, lib = O.Session([pol]), O.Session([pol]), L.Session([pol])
    pk, seq = [], 40000
    for k in range(200):
        p = rtp_packet(rng, SSRC, seq & 0xffff, 40)
        pk.append(snd.protect(p, len(p) + 64)[1])
        seq += 1
    for _ in range(3):
        seq += 20000
        p = rtp_packet(rng, SSRC, seq & 0xffff, 40)
        snd.protect(p, len(p) + 64)         # the sender's index moves on
        pk.append(p + rng.randbytes(10))    # what arrives is forged
    for k in range(50):
        seq += 1
        p = rtp_packet(rng, SSRC, seq & 0xffff, 40)
        pk.append(snd.protect(p, len(p) + 64)[1])
    ref = [orc.unprotect(p, len(p))[0] for p in pk]
    st, _, _, _ = _device_unprotect(lib, pk, True)
    assert st == ref
    assert lib.prepass_stats() == (0, 1)
