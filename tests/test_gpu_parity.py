"""GPU parity: libsrtp_mi355x (HIP kernels through the C ABI) against the
reference's golden fixtures and against the CPU oracle on random batches.

Bit-exact equality is required for every output byte and status code.
"""
import random

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.golden_util import all_cases, case_ids, kat_cases, replay_ops

pytestmark = pytest.mark.gpu
H = bytes.fromhex


def _gpu():
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")


# --------------------------------------------------------------------------
# golden fixtures (outputs of the reference itself)

@pytest.mark.parametrize("case", all_cases(), ids=case_ids())
def test_golden_single_packet_api(case):
    _gpu()
    snd = L.Session([case["snd"]])
    rcv = L.Session([case["rcv"]])
    for i, op in enumerate(case["ops"]):
        s = snd if op["sess"] == "snd" else rcv
        if op["op"] == "protect":
            st, out = s.protect(H(op["in"]), op["cap"], op["mki_index"])
        else:
            st, out = s.unprotect(H(op["in"]), op["cap"])
        assert st == op["status"], (i, op["op"], st, op["status"])
        if st == 0:
            assert out.hex() == op["out"], (i, op["op"])


@pytest.mark.parametrize("case", all_cases(), ids=case_ids())
def test_golden_batched(case):
    """Consecutive ops of one session/direction go through ONE batch call:
    in-batch ordering (replays, wraps, tamper-then-genuine) must match the
    reference's one-call-per-packet results."""
    _gpu()
    sess = {"snd": L.Session([case["snd"]]), "rcv": L.Session([case["rcv"]])}
    ops = case["ops"]
    i = 0
    while i < len(ops):
        j = i
        while (j < len(ops) and ops[j]["sess"] == ops[i]["sess"]
               and ops[j]["op"] == ops[i]["op"]):
            j += 1
        grp = ops[i:j]
        s = sess[ops[i]["sess"]]
        pk = [H(o["in"]) for o in grp]
        caps = [o["cap"] for o in grp]
        if ops[i]["op"] == "protect":
            st, out = s.protect_batch(pk, caps, [o["mki_index"] for o in grp])
        else:
            st, out = s.unprotect_batch(pk, caps)
        for k, o in enumerate(grp):
            assert st[k] == o["status"], (i + k, o["op"], st[k], o["status"])
            if st[k] == 0:
                assert out[k].hex() == o["out"], (i + k, o["op"])
        i = j


@pytest.mark.parametrize("case", kat_cases(), ids=[c["name"] for c in kat_cases()])
def test_published_kats(case):
    """test/srtp_driver.c's published packets (srtp_validate*, empty
    payload), RTP and RTCP, through the single-packet C ABI."""
    _gpu()
    replay_ops(case, L.Session([case["snd"]]), L.Session([case["rcv"]]))


@pytest.mark.parametrize("case", kat_cases(), ids=[c["name"] for c in kat_cases()])
def test_published_kats_batched(case):
    _gpu()
    snd, rcv = L.Session([case["snd"]]), L.Session([case["rcv"]])
    for op in case["ops"]:
        s = snd if op["sess"] == "snd" else rcv
        fn = {"protect": s.protect_batch, "unprotect": s.unprotect_batch,
              "protect_rtcp": s.protect_rtcp_batch,
              "unprotect_rtcp": s.unprotect_rtcp_batch}[op["op"]]
        st, out = fn([H(op["in"])], [op["cap"]])
        assert st[0] == op["status"], (case["name"], op["op"])
        assert out[0].hex() == op["out"], (case["name"], op["op"])


# --------------------------------------------------------------------------
# random batches vs the oracle

POLICIES = {
    "icm128_hmac80": (1, 30, 3, 20, 10, 3),
    "icm128_hmac32": (1, 30, 3, 20, 4, 3),
    "icm192_hmac80": (4, 38, 3, 20, 10, 3),
    "icm256_hmac80": (5, 46, 3, 20, 10, 3),
    "icm256_hmac32": (5, 46, 3, 20, 4, 3),
    "icm128_nullauth": (1, 30, 0, 0, 0, 1),
    "null_hmac80": (0, 30, 3, 20, 10, 2),
    "null_null": (0, 0, 0, 0, 0, 0),
    "icm128_authonly": (1, 30, 3, 20, 10, 2),
    "gcm128_16": (6, 28, 0, 0, 16, 3),
    "gcm256_16": (7, 44, 0, 0, 16, 3),
    "gcm256_8": (7, 44, 0, 0, 8, 3),
}


def policy(name, ssrc=0xcafebabe, ssrc_type=1, seed=1, mki=0, nkeys=1,
           window=128, repeat=0):
    c, ckl, a, akl, tag, sv = POLICIES[name]
    rng = random.Random(seed)
    d = dict(ssrc_type=ssrc_type, ssrc=ssrc, cipher_type=c, cipher_key_len=ckl,
             auth_type=a, auth_key_len=akl, auth_tag_len=tag, sec_serv=sv,
             window_size=window, allow_repeat_tx=repeat,
             keys=[bytes(rng.randrange(256) for _ in range(46)).hex()
                   for _ in range(nkeys)],
             use_mki=1 if mki else 0, mki_size=mki,
             mki_ids=[bytes(rng.randrange(256) for _ in range(mki)).hex()
                      for _ in range(nkeys)] if mki else [])
    return d


def rtp_packet(rng, ssrc, seq, payload, cc=0, xwords=-1, ts=0):
    b0 = 0x80 | (0x10 if xwords >= 0 else 0) | cc
    hdr = bytes([b0, 96, seq >> 8, seq & 0xff]) + ts.to_bytes(4, "big") + \
        ssrc.to_bytes(4, "big")
    hdr += bytes(rng.randrange(256) for _ in range(4 * cc))
    if xwords >= 0:
        hdr += bytes([0xbe, 0xde, xwords >> 8, xwords & 0xff])
        hdr += bytes(rng.randrange(256) for _ in range(4 * xwords))
    return hdr + rng.randbytes(payload)


def random_stream(rng, n, ssrc, seq0=0x1234, sizes=(0, 1, 15, 16, 17, 31, 160,
                                                     1388, 1400, 1452, 57)):
    out, seq = [], seq0
    for i in range(n):
        cc = rng.choice([0, 0, 0, 1, 3])
        xw = rng.choice([-1, -1, -1, 0, 2])
        out.append(rtp_packet(rng, ssrc, seq & 0xffff, rng.choice(sizes), cc,
                              xw, ts=i * 160))
        seq += rng.choice([1, 1, 1, 1, 2, 0, -3])
    return out


@pytest.mark.parametrize("name", sorted(POLICIES))
def test_random_protect_unprotect_batches(name):
    _gpu()
    rng = random.Random(name)
    pol = policy(name, seed=len(name))
    lib_s, orc_s = L.Session([pol]), O.Session([pol])
    pkts = random_stream(rng, 300, 0xcafebabe, seq0=0xff00)
    caps = [len(p) + 20 for p in pkts]
    st, out = lib_s.protect_batch(pkts, caps)
    srtp = []
    for i, p in enumerate(pkts):
        rc, ref = orc_s.protect(p, caps[i])
        assert st[i] == rc, (i, st[i], rc)
        if rc == 0:
            assert out[i] == ref, i
            srtp.append(ref)
    # receiver: reorder a little, duplicate, tamper
    rx = []
    for i, p in enumerate(srtp):
        rx.append(p)
        r = rng.random()
        if r < 0.05:
            rx.append(p)                                  # replay
        elif r < 0.10:
            b = bytearray(p)
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
            rx.append(bytes(b))                           # tamper
        elif r < 0.15 and len(rx) > 2:
            rx[-1], rx[-2] = rx[-2], rx[-1]               # reorder
    lib_r, orc_r = L.Session([pol]), O.Session([pol])
    st, out = lib_r.unprotect_batch(rx)
    for i, p in enumerate(rx):
        rc, ref = orc_r.unprotect(p, len(p))
        assert st[i] == rc, (i, st[i], rc)
        if rc == 0:
            assert out[i] == ref, i


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_mki_batches(name):
    _gpu()
    rng = random.Random(7)
    pol = policy(name, mki=4, nkeys=3)
    lib_s, orc_s = L.Session([pol]), O.Session([pol])
    pkts = random_stream(rng, 60, 0xcafebabe)
    mk = [rng.randrange(4) for _ in pkts]   # 3 is a bad index
    st, out = lib_s.protect_batch(pkts, None, mk)
    good = []
    for i, p in enumerate(pkts):
        rc, ref = orc_s.protect(p, len(p) + 144, mk[i])
        assert st[i] == rc
        if rc == 0:
            assert out[i] == ref
            good.append(ref)
    lib_r, orc_r = L.Session([pol]), O.Session([pol])
    st, out = lib_r.unprotect_batch(good)
    for i, p in enumerate(good):
        rc, ref = orc_r.unprotect(p, len(p))
        assert st[i] == rc and (rc or out[i] == ref)


def test_template_many_ssrcs():
    _gpu()
    rng = random.Random(11)
    snd_p = policy("icm128_hmac80", ssrc_type=3, seed=5)
    rcv_p = dict(snd_p, ssrc_type=2)
    lib_s, orc_s = L.Session([snd_p]), O.Session([snd_p])
    pkts = []
    for r in range(8):
        for s in range(40):
            pkts.append(rtp_packet(rng, 0x1000 + s, (s * 977 + r) & 0xffff,
                                   rng.choice([20, 160, 1400])))
    st, out = lib_s.protect_batch(pkts)
    srtp = []
    for i, p in enumerate(pkts):
        rc, ref = orc_s.protect(p, len(p) + 144)
        assert st[i] == rc and out[i] == ref, i
        srtp.append(ref)
    # receiver: the first packet of some SSRCs is forged -> provisional
    # stream must not be created, later genuine packets still pass
    rx = []
    for i, p in enumerate(srtp):
        if i < 40 and i % 3 == 0:
            b = bytearray(p)
            b[-1] ^= 0x55
            rx.append(bytes(b))
        rx.append(p)
    lib_r, orc_r = L.Session([rcv_p]), O.Session([rcv_p])
    st, out = lib_r.unprotect_batch(rx)
    for i, p in enumerate(rx):
        rc, ref = orc_r.unprotect(p, len(p))
        assert st[i] == rc, (i, st[i], rc)
        if rc == 0:
            assert out[i] == ref


def test_multi_stream_distinct_keys():
    _gpu()
    rng = random.Random(3)
    pols = [policy(n, ssrc=0x100 + k, seed=k)
            for k, n in enumerate(["icm128_hmac80", "icm256_hmac80",
                                   "gcm128_16", "icm128_hmac32",
                                   "gcm256_8", "null_hmac80"])]
    lib_s, orc_s = L.Session(pols), O.Session(pols)
    pkts = [rtp_packet(rng, 0x100 + rng.randrange(6), i, rng.choice(
        [0, 33, 160, 1400])) for i in range(400)]
    st, out = lib_s.protect_batch(pkts)
    for i, p in enumerate(pkts):
        rc, ref = orc_s.protect(p, len(p) + 144)
        assert st[i] == rc, i
        if rc == 0:
            assert out[i] == ref, i


# --------------------------------------------------------------------------
# device-resident API

def _arena(pkts, slot_extra=160):
    import torch
    offs, pos = [], 0
    for p in pkts:
        offs.append(pos)
        pos += (len(p) + slot_extra + 15) & ~15
    buf = bytearray(pos + 16)
    for o, p in zip(offs, pkts):
        buf[o:o + len(p)] = p
    dev = torch.frombuffer(buf, dtype=torch.uint8).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    return dev, off, ln, offs


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16",
                                  "icm256_hmac32"])
def test_device_api_vs_oracle(name):
    _gpu()
    import torch
    rng = random.Random(name + "dev")
    pol = policy(name)
    lib_s, orc_s = L.Session([pol]), O.Session([pol])
    pkts = random_stream(rng, 500, 0xcafebabe, seq0=0xfff0)
    arena, off, ln, offs = _arena(pkts)
    out = torch.zeros_like(arena)
    cap = (ln + 144).clone()
    status = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    assert lib_s.protect_device(arena, off, ln, out, off, cap, status) == 0
    st = status.cpu().tolist()
    olen = cap.cpu().tolist()
    host = out.cpu().numpy().tobytes()
    srtp = []
    for i, p in enumerate(pkts):
        rc, ref = orc_s.protect(p, len(p) + 144)
        assert st[i] == rc, (i, st[i], rc)
        if rc == 0:
            assert host[offs[i]:offs[i] + olen[i]] == ref, i
            srtp.append(ref)
    # unprotect in place on the device
    arena2, off2, ln2, offs2 = _arena(srtp)
    cap2 = ln2.clone()
    status2 = torch.full((len(srtp),), -1, dtype=torch.int32).cuda()
    lib_r, orc_r = L.Session([pol]), O.Session([pol])
    assert lib_r.unprotect_device(arena2, off2, ln2, arena2, off2, cap2,
                                  status2) == 0
    st2, olen2 = status2.cpu().tolist(), cap2.cpu().tolist()
    host2 = arena2.cpu().numpy().tobytes()
    for i, p in enumerate(srtp):
        rc, ref = orc_r.unprotect(p, len(p))
        assert st2[i] == rc
        if rc == 0:
            assert host2[offs2[i]:offs2[i] + olen2[i]] == ref, i


def oracle_chunks(pol, orig, prot, rtp_len, trailer, seq0, chunk=65536):
    """Compare every packet of a one-stream batch (rows of orig / prot, the
    stream's packets in order from sequence number seq0, ROC 0) with the C
    oracle: chunks of 2^16 packets run on host threads, each on an oracle
    session whose stream is seated at the chunk's ROC by
    srtp_stream_set_roc (the sender's pending ROC, srtp.c:2069-2071) -- a
    chunk starting at sequence number seq0 with ROC >= 1.  Returns the
    mismatching packet numbers."""
    import concurrent.futures as cf
    import numpy as np
    n, slot = orig.shape
    assert chunk % 65536 == 0 and n % chunk == 0
    out_len = rtp_len + trailer
    sessions = []
    for c in range(n // chunk):
        o = O.Session([pol])
        roc = (seq0 + c * chunk) >> 16
        if roc:
            assert o.set_roc(pol["ssrc"], roc) == 0
        sessions.append(o)

    def one(c):
        lo = c * chunk
        part = np.ascontiguousarray(orig[lo:lo + chunk])
        offs = np.arange(chunk, dtype=np.uint64) * np.uint64(slot)
        lens = np.full(chunk, rtp_len, dtype=np.uint32)
        nbad, exp, olen = sessions[c].protect_many(part.reshape(-1), offs,
                                                   lens, slot)
        assert nbad == 0 and (olen == out_len).all()
        diff = (exp[:, :out_len] != prot[lo:lo + chunk, :out_len]).any(axis=1)
        return [lo + int(i) for i in np.nonzero(diff)[0]]

    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        return sum(ex.map(one, range(len(sessions))), [])


@pytest.mark.parametrize("name,n,trailer", [
    ("icm128_hmac80", 65536, 10),
    ("icm128_hmac80", 1 << 20, 10),   # configs[1] at its own size
    ("gcm256_16", 65536, 16),         # configs[2]'s cipher, uniform key
    ("gcm256_16", 1 << 20, 16),       # configs[2] at its own size
])
def test_large_uniform_batch_roundtrip(name, n, trailer):
    """n x 1400 B through the device API (the bench shape): every protected
    packet is compared byte-for-byte with the C oracle (at 2^20 packets ROC
    0 .. 16 across every CU's waves), and protect -> unprotect must restore
    every packet."""
    _gpu()
    import torch
    payload = 1400
    pol = policy(name)
    g = torch.Generator().manual_seed(5)
    body = torch.randint(0, 256, (n, payload), dtype=torch.uint8, generator=g)
    slot = (12 + payload + 160 + 15) & ~15
    hdr = torch.zeros((n, 12), dtype=torch.uint8)
    seq = (torch.arange(n) + 0x1234) & 0xffff
    hdr[:, 0] = 0x80
    hdr[:, 1] = 96
    hdr[:, 2] = (seq >> 8).to(torch.uint8)
    hdr[:, 3] = (seq & 0xff).to(torch.uint8)
    hdr[:, 8:12] = torch.tensor([0xca, 0xfe, 0xba, 0xbe], dtype=torch.uint8)
    arena = torch.zeros((n, slot), dtype=torch.uint8)
    arena[:, :12] = hdr
    arena[:, 12:12 + payload] = body
    del body
    orig = arena
    d = arena.reshape(-1).cuda()
    off = (torch.arange(n, dtype=torch.int64) * slot).cuda()
    ln = torch.full((n,), 12 + payload, dtype=torch.int32).cuda()
    cap = torch.full((n,), slot, dtype=torch.int32).cuda()
    st = torch.zeros(n, dtype=torch.int32).cuda()
    s = L.Session([pol])
    assert s.protect_device(d, off, ln, d, off, cap, st) == 0
    assert int(st.abs().sum()) == 0
    assert bool((cap == 12 + payload + trailer).all())
    prot = d.cpu().reshape(n, slot)
    # every packet against the oracle (ROC 0 .. 16 at n = 2^20)
    bad = oracle_chunks(pol, orig.numpy(), prot.numpy(), 12 + payload,
                        trailer, 0x1234)
    assert bad == [], bad[:5]
    # ciphertext differs from the plaintext everywhere but the header
    assert not torch.equal(prot[:, 12:12 + payload], orig[:, 12:12 + payload])
    del prot
    r = L.Session([pol])
    ln2 = cap.clone()
    cap2 = ln2.clone()
    st2 = torch.zeros(n, dtype=torch.int32).cuda()
    assert r.unprotect_device(d, off, ln2, d, off, cap2, st2) == 0
    assert int(st2.abs().sum()) == 0
    assert bool((cap2 == 12 + payload).all())
    back = d.cpu().reshape(n, slot)
    assert torch.equal(back[:, :12 + payload], orig[:, :12 + payload])
