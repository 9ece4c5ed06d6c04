"""GPU parity for SRTCP (srtp_protect_rtcp / srtp_unprotect_rtcp through the
C ABI, crypto in k_rtcp; AES-ICM/null and AES-GCM): the reference's own
outputs (tests/golden/ref_rtcp*.json, oracle/gen_golden_rtcp.c) and the CPU
restatement (oracle/srtcp_oracle.py) on seeded random traffic.  Bit-exact.
"""
import random

import pytest

import libsrtp_amd as L
from oracle.srtcp_oracle import SrtcpSession
from tests.golden_util import load
from tests.test_oracle_golden import replay_rtcp

pytestmark = pytest.mark.gpu
CASES = load("ref_rtcp.json")["cases"] + load("ref_rtcp_gcm.json")["cases"]


def _gpu():
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_srtcp(case):
    _gpu()
    replay_rtcp(case, L.Session([case["snd"]]), L.Session([case["rcv"]]))


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_random_srtcp_vs_oracle(case):
    """Same policies, fresh random RTCP packets of every length class
    (header only, partial and multiple AES blocks, > 4 KiB compound
    packets), sent out of order with replays; GPU and oracle must agree."""
    _gpu()
    rng = random.Random(sum(case["name"].encode()))
    g_snd, g_rcv = L.Session([case["snd"]]), L.Session([case["rcv"]])
    o_snd, o_rcv = SrtcpSession([case["snd"]]), SrtcpSession([case["rcv"]])
    nk = len(case["snd"]["keys"]) if case["snd"]["use_mki"] else 1
    ssrc = case["snd"]["ssrc"]
    sent = []
    for i in range(40):
        n = rng.choice([8, 9, 15, 16, 23, 24, 40, 100, 1000, 4200])
        pkt = bytearray(rng.randrange(256) for _ in range(n))
        pkt[0:2] = b"\x80\xc8"
        pkt[4:8] = ssrc.to_bytes(4, "big")
        mi = i % nk
        g = g_snd.protect_rtcp(bytes(pkt), n + 148, mi)
        o = o_snd.protect_rtcp(bytes(pkt), n + 148, mi)
        assert g == o, (i, n)
        if g[0] == 0:
            sent.append(g[1])
    order = list(range(len(sent))) + [rng.randrange(len(sent))
                                      for _ in range(5)]
    rng.shuffle(order)
    for j in order:
        p = sent[j]
        if rng.random() < 0.2:
            q = bytearray(p)
            q[rng.randrange(len(q))] ^= 1 << rng.randrange(8)
            p = bytes(q)
        g = g_rcv.unprotect_rtcp(p, len(p))
        o = o_rcv.unprotect_rtcp(p, len(p))
        assert g == o, (j, len(p))


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_srtcp_batched(case):
    """Runs of consecutive ops of one session/direction go through ONE
    srtp_{protect,unprotect}_rtcp_batch call: in-batch replays, late
    arrivals, template promotion and tamper-then-genuine must come out as
    the reference's sequential calls did."""
    _gpu()
    sess = {"snd": L.Session([case["snd"]]), "rcv": L.Session([case["rcv"]])}
    ops = case["ops"]
    i = 0
    while i < len(ops):
        j = i
        while j < len(ops) and ops[j]["sess"] == ops[i]["sess"] and \
                ops[j]["op"] == ops[i]["op"]:
            j += 1
        run = ops[i:j]
        s = sess[ops[i]["sess"]]
        pkts = [bytes.fromhex(o["in"]) for o in run]
        caps = [o["cap"] for o in run]
        if ops[i]["op"] == "protect_rtcp":
            st, out = s.protect_rtcp_batch(pkts, caps,
                                           [o["mki_index"] for o in run])
        else:
            st, out = s.unprotect_rtcp_batch(pkts, caps)
        for k, o in enumerate(run):
            assert st[k] == o["status"], (i + k, o["op"], st[k], o["status"])
            if o["status"] == 0:
                assert out[k].hex() == o["out"], (i + k, o["op"])
        i = j


def test_srtcp_batch_vs_oracle_large():
    """2000 compound packets over 8 SSRCs of a template session in one
    protect batch, then shuffled (with duplicates and tampering) through one
    unprotect batch; GPU and oracle must agree packet by packet."""
    _gpu()
    case = next(c for c in CASES if c["name"] == "rtcp_template")
    rng = random.Random(7)
    g_snd, g_rcv = L.Session([case["snd"]]), L.Session([case["rcv"]])
    o_snd, o_rcv = SrtcpSession([case["snd"]]), SrtcpSession([case["rcv"]])
    pkts = []
    for i in range(2000):
        n = rng.choice([8, 28, 52, 100, 300, 1200])
        p = bytearray(rng.randrange(256) for _ in range(n))
        p[0:2] = b"\x80\xc8"
        p[4:8] = (0x7000 + i % 8).to_bytes(4, "big")
        pkts.append(bytes(p))
    st, out = g_snd.protect_rtcp_batch(pkts)
    for i, p in enumerate(pkts):
        assert (st[i], out[i]) == o_snd.protect_rtcp(p, len(p) + 148), i
    rx = [out[i] for i in range(len(pkts))] + \
        [out[rng.randrange(len(pkts))] for _ in range(100)]
    rng.shuffle(rx)
    for k in range(0, len(rx), 17):
        q = bytearray(rx[k])
        q[rng.randrange(len(q))] ^= 4
        rx[k] = bytes(q)
    st, back = g_rcv.unprotect_rtcp_batch(rx)
    for k, p in enumerate(rx):
        assert (st[k], back[k]) == o_rcv.unprotect_rtcp(p, len(p)), k


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_rtcp_trailer_length_matches_reference_output(case):
    """srtp_get_protect_rtcp_trailer_length (srtp.c:4972-5000 with the
    rtcp_auth tag) equals the growth the reference's own srtp_protect_rtcp
    produced for the same session and MKI index."""
    _gpu()
    s = L.Session([case["snd"]])
    for op in case["ops"]:
        if op["op"] == "protect_rtcp" and op["status"] == 0:
            st, n = s.rtcp_trailer_length(op["mki_index"])
            assert st == 0
            assert n == (len(op["out"]) - len(op["in"])) // 2, op["mki_index"]
