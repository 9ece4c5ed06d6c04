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
