"""One-stream receive batches as a network delivers them -- reordered,
duplicated, late across batch boundaries, old, forged -- stay on the device
pre-pass (srtp_prepass.hip k_pu_chain1 .. k_pu_commit1) and give exactly
the statuses and bytes of the reference's receive loop (test/rtp.c:104-149,
srtp.c:2884-2903 estimate + replay check, 3157-3167 replay add after the tag
check; crypto/replay/rdbx.c:112-145, 227-270), here the C oracle's
srtp_unprotect called once per packet in arrival order.

Round 3 sent any non-advancing sequence number in a one-stream batch to the
host path for the whole batch; these tests assert the device path ran
(prepass_stats: no host batch)."""
import random

import numpy as np
import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.test_gpu_parity import _gpu, policy

pytestmark = pytest.mark.gpu
SSRC = 0x0badcafe


def _sent(pol, n, seq0, payloads, seed):
    """n packets of one stream protected in send order by the oracle:
    (arena (n, slot) uint8, srtp lengths)"""
    rng = np.random.default_rng(seed)
    slot = (12 + max(payloads) + 16 + 15) & ~15
    a = rng.integers(0, 256, (n, slot), dtype=np.uint8)
    plen = rng.choice(np.array(payloads), n)
    seq = (np.arange(n) + seq0) & 0xffff
    a[:, 0], a[:, 1] = 0x80, 96
    a[:, 2], a[:, 3] = seq >> 8, seq & 0xff
    a[:, 8:12] = np.frombuffer(SSRC.to_bytes(4, "big"), dtype=np.uint8)
    snd = O.Session([pol])
    bad, out, olen = snd.protect_many(a.reshape(-1),
                                      np.arange(n, dtype=np.uint64) * slot,
                                      (12 + plen).astype(np.uint32), slot)
    assert bad == 0
    return out, olen


def _network(n, rng, reorder, dup, old, forge):
    """arrival order as (sent index, forged) pairs: local displacements of up
    to 32 places, duplicates of recent packets, old copies 200..400 behind
    (past a 128-bit window), forgeries (a copy with a flipped tag bit that
    arrives just before the genuine packet)"""
    order = list(range(n))
    for i in range(n - 1):
        if rng.random() < reorder:
            j = min(n - 1, i + rng.randrange(1, 33))
            order[i], order[j] = order[j], order[i]
    out = []
    for i, s in enumerate(order):
        r = rng.random()
        if dup + old <= r < dup + old + forge:
            out.append((s, True))   # arrives first: auth_fail, not a replay
        out.append((s, False))
        if r < dup:
            out.append((order[max(0, i - rng.randrange(0, 64))], False))
        elif r < dup + old and i > 400:
            out.append((order[i - rng.randrange(200, 400)], False))
    return out


def _receive(name, n, seq0, nbatch, reorder, dup, old, forge, inplace=True,
             payloads=(0, 20, 160, 1200), seed=1):
    import torch
    _gpu()
    pol = policy(name, ssrc=SSRC, seed=seed)
    sent, slen = _sent(pol, n, seq0, payloads, seed)
    arr = _network(n, random.Random(seed), reorder, dup, old, forge)
    src = np.array([s for s, _ in arr])
    forged = np.array([f for _, f in arr])
    recv = sent[src].copy()
    rlen = slen[src].astype(np.uint32)
    fi = np.nonzero(forged)[0]
    recv[fi, rlen[fi] - 1] ^= 0x40          # the tag's last byte
    m, slot = recv.shape
    # the oracle's receive loop, one srtp_unprotect per packet in order
    orc = O.Session([pol])
    ref_st, ref_out, ref_len = orc.unprotect_many(
        recv.reshape(-1), np.arange(m, dtype=np.uint64) * slot, rlen, slot)
    lib = L.Session([pol])
    bounds = np.linspace(0, m, nbatch + 1).astype(int)
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        k = b1 - b0
        d = torch.from_numpy(recv[b0:b1].copy()).cuda().view(-1)
        dst = d if inplace else torch.full_like(d, 0x3c)
        off = (torch.arange(k, dtype=torch.int64) * slot).cuda()
        ln = torch.from_numpy(rlen[b0:b1].astype(np.int32)).cuda()
        cap = ln.clone()
        st = torch.full((k,), -1, dtype=torch.int32).cuda()
        assert lib.unprotect_device(d, off, ln, dst, off, cap, st) == 0
        st, cap = st.cpu().numpy(), cap.cpu().numpy()
        got = dst.cpu().numpy().reshape(k, slot)
        bad = np.nonzero(st != ref_st[b0:b1])[0]
        assert len(bad) == 0, [(int(b0 + i), int(st[i]), int(ref_st[b0 + i]))
                               for i in bad[:10]]
        ok = st == 0
        assert (cap[ok] == ref_len[b0:b1][ok]).all()
        for i in np.nonzero(ok)[0]:
            assert (got[i, :cap[i]] == ref_out[b0 + i, :cap[i]]).all(), b0 + i
        rej = np.nonzero(~ok)[0]
        if inplace:   # a rejected packet's buffer holds its ciphertext again
            for i in rej:
                assert (got[i, :rlen[b0 + i]] ==
                        recv[b0 + i, :rlen[b0 + i]]).all(), b0 + i
    assert lib.prepass_stats()[1] == 0, lib.prepass_last_abort()
    assert lib.prepass_stats()[0] == nbatch
    # the state the device left is what the host path continues from
    assert lib.get_roc(SSRC)[1] == orc.get_roc(SSRC)[1]
    return ref_st


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
@pytest.mark.parametrize("inplace", [True, False], ids=["inplace", "outofplace"])
def test_reordered_duplicated_old_forged(name, inplace):
    st = _receive(name, 40000, 0xff00, 3, reorder=0.05, dup=0.01, old=0.005,
                  forge=0.01, inplace=inplace)
    for code in (0, 7, 9, 10):           # every verdict occurs
        assert (st == code).any(), code


def test_reorders_across_rollover_and_batches():
    """sequence numbers wrap twice inside the run; packets reordered across
    the batch boundaries arrive after the stream's index moved past them
    (the stored window decides)"""
    st = _receive("icm128_hmac80", 150000, 0xfff0, 8, reorder=0.2, dup=0.02,
                  old=0.0, forge=0.0, payloads=(0, 40))
    assert (st == 9).any()


def test_in_order_batch_is_plain():
    """strictly advancing: no duplicate pass, every packet accepted"""
    st = _receive("gcm256_16", 20000, 5, 2, 0, 0, 0, 0)
    assert (st == 0).all()


def test_configs1_receive_1pct_reorder_01pct_dup():
    """the verdict's bar: a 2^20-packet one-stream batch with 1 % reorders
    and 0.1 % duplicates stays on the device, bit-exact against the oracle"""
    _receive("icm128_hmac80", 1 << 20, 0x1234, 1, reorder=0.01, dup=0.001,
             old=0.0, forge=0.0, payloads=(160,))


def test_host_buffer_unprotect_batch_on_device_prepass():
    """srtp_unprotect_batch (per-packet host pointers, the socket receive
    path of srtp.c:2820-3172 / test/rtp.c:104-149) gathers the batch into the
    pinned staging arena and runs the device pre-pass: reordered, duplicated
    and forged packets included, no host-path batch"""
    _gpu()
    pol = policy("icm128_hmac80", ssrc=SSRC, seed=5)
    sent, slen = _sent(pol, 3000, 0xfff0, (0, 20, 160, 1200), 5)
    arr = _network(3000, random.Random(5), 0.05, 0.01, 0.005, 0.01)
    pk = []
    for s, f in arr:
        b = bytearray(sent[s, :slen[s]].tobytes())
        if f:
            b[-1] ^= 0x40
        pk.append(bytes(b))
    orc, lib = O.Session([pol]), L.Session([pol])
    ref = [orc.unprotect(p, len(p)) for p in pk]
    st, out = lib.unprotect_batch(pk)
    for i, (rc, o) in enumerate(ref):
        assert int(st[i]) == rc, (i, int(st[i]), rc)
        if rc == 0:
            assert out[i] == o, i
    assert lib.prepass_stats() == (1, 0), lib.prepass_last_abort()
