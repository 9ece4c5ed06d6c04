"""srtp_protect_device_async (include/srtp_mi355x.h): batches submitted back
to back on one stream without waiting for their protect kernels, then
checked against the CPU oracle called once per packet in the same order.

A batch the device pre-pass declines (a replayed sequence number) must run
to completion through the host path in the middle of the queue, and the
batches after it must continue from the state it left.
"""
import random

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.test_gpu_parity import _gpu, policy, rtp_packet
from tests.test_gpu_prepass import _chains

pytestmark = pytest.mark.gpu


def _stage(pkts, caps):
    import torch
    offs, pos = [], 0
    for p, c in zip(pkts, caps):
        offs.append(pos)
        pos += (max(len(p), c) + 15) & ~15
    buf = bytearray(pos + 16)
    for o, p in zip(offs, pkts):
        buf[o:o + len(p)] = p
    t = dict(arena=torch.frombuffer(buf, dtype=torch.uint8).cuda(),
             off=torch.tensor(offs, dtype=torch.int64).cuda(),
             ln=torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda(),
             cap=torch.tensor(caps, dtype=torch.int32).cuda(),
             st=torch.full((len(pkts),), -1, dtype=torch.int32).cuda())
    t["offs"] = offs
    return t


def _run_async(sess, batches):
    """every batch submitted with srtp_protect_device_async on the current
    stream, one synchronize at the end"""
    import torch
    stream = torch.cuda.current_stream().cuda_stream
    staged = [_stage(p, c) for p, c in batches]
    for t in staged:
        t["desc"] = sess.prepare_device(t["arena"], t["off"], t["ln"],
                                        t["arena"], t["off"], t["cap"],
                                        t["st"], stream=stream)
        assert sess.protect_prepared_async(t["desc"]) == 0
    torch.cuda.synchronize()
    res = []
    for t in staged:
        st, cap = t["st"].cpu().tolist(), t["cap"].cpu().tolist()
        host = t["arena"].cpu().numpy().tobytes()
        res.append((st, [host[o:o + c] if s == 0 else None
                         for o, c, s in zip(t["offs"], cap, st)], cap))
    return res


@pytest.mark.parametrize("pname", ["icm128_hmac80", "gcm256_16"])
def test_async_batches_match_oracle(pname):
    _gpu()
    rng = random.Random(71)
    ssrcs = [0x4100 + k for k in range(5)]
    pols = [policy(pname, ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    lib, orc = L.Session(pols), O.Session(pols)
    batches, seq0 = [], [0xffe0, 7, 0x8000, 300, 0x7ff0]
    for k in range(6):
        pk, nxt = _chains(rng, ssrcs, 500, seq0, big=0)
        if k == 3:
            pk.insert(100, pk[40])   # replay: this batch takes the host path
        batches.append((pk, [len(p) + 32 for p in pk]))
        seq0 = [nxt[s] for s in ssrcs]
    res = _run_async(lib, batches)
    for (pk, caps), (st, outs, olen) in zip(batches, res):
        for i, p in enumerate(pk):
            rc, ref = orc.protect(p, caps[i])
            assert st[i] == rc, (i, st[i], rc)
            if rc == 0:
                assert outs[i] == ref, i
            else:
                assert olen[i] == caps[i], i
    assert lib.prepass_stats() == (5, 1)
    for s in ssrcs:
        assert lib.get_roc(s)[1] == orc.get_roc(s)[1], hex(s)


def test_async_single_stream_large_then_sync_call():
    """2^16-packet single-stream batches (the chain form) queued async, then
    a synchronous call continues from their state"""
    _gpu()
    rng = random.Random(3)
    pol = policy("icm128_hmac80", ssrc=0x99)
    lib, orc = L.Session([pol]), O.Session([pol])
    batches, seq = [], 0xfe00
    for _ in range(3):
        pk = [rtp_packet(rng, 0x99, (seq + j) & 0xffff, 160)
              for j in range(1 << 16)]
        seq += 1 << 16
        batches.append((pk, [len(p) + 16 for p in pk]))
    res = _run_async(lib, batches)
    assert lib.prepass_stats() == (3, 0)
    orc2 = orc
    for (pk, caps), (st, outs, _) in zip(batches, res):
        assert all(s == 0 for s in st)
        for i, p in enumerate(pk):
            rc, ref = orc2.protect(p, caps[i])
            assert rc == 0 and outs[i] == ref, i
    tail = [rtp_packet(rng, 0x99, (seq + j) & 0xffff, 100) for j in range(50)]
    st, out = lib.protect_batch(tail, [len(p) + 16 for p in tail])
    for i, p in enumerate(tail):
        rc, ref = orc2.protect(p, len(p) + 16)
        assert st[i] == rc and (rc or out[i] == ref), i


def test_async_then_host_calls_without_synchronize():
    """host-buffer batches, get_roc and a synchronous call on another stream
    right after queued async batches: the library finishes the queued work
    before it touches the stream table from elsewhere"""
    _gpu()
    import torch
    rng = random.Random(12)
    pol = policy("icm128_hmac80", ssrc=0x5150)
    lib, orc = L.Session([pol]), O.Session([pol])
    stream = torch.cuda.current_stream().cuda_stream
    seq, staged, batches = 0xff00, [], []
    for _ in range(3):
        pk = [rtp_packet(rng, 0x5150, (seq + j) & 0xffff, 1200)
              for j in range(20000)]
        seq += 20000
        caps = [len(p) + 16 for p in pk]
        t = _stage(pk, caps)
        t["desc"] = lib.prepare_device(t["arena"], t["off"], t["ln"],
                                       t["arena"], t["off"], t["cap"],
                                       t["st"], stream=stream)
        assert lib.protect_prepared_async(t["desc"]) == 0
        staged.append(t)
        batches.append((pk, caps))
    # no synchronize: a host-buffer batch on the library's own stream
    tail = [rtp_packet(rng, 0x5150, (seq + j) & 0xffff, 80)
            for j in range(300)]
    st_tail, out_tail = lib.protect_batch(tail, [len(p) + 16 for p in tail])
    roc = lib.get_roc(0x5150)[1]
    torch.cuda.synchronize()
    for (pk, caps), t in zip(batches, staged):
        st = t["st"].cpu().tolist()
        host = t["arena"].cpu().numpy().tobytes()
        for i, p in enumerate(pk):
            rc, ref = orc.protect(p, caps[i])
            assert rc == 0 and st[i] == 0, i
            o = t["offs"][i]
            assert host[o:o + len(ref)] == ref, i
    for i, p in enumerate(tail):
        rc, ref = orc.protect(p, len(p) + 16)
        assert st_tail[i] == rc and (rc or out_tail[i] == ref), i
    assert roc == orc.get_roc(0x5150)[1]


def test_async_failure_is_reported_not_spun_on():
    """a stream in an error state must end the wait for the
    pre-pass verdict with srtp_err_status_fail (not spin), and a queued
    batch whose drain fails must poison the session: every later packet
    call returns srtp_err_status_fail, no stream state is taken from the
    device table it left (srtp_mi355x_debug_inject_failure)."""
    import torch
    _gpu()
    rng = random.Random(5)
    ssrcs = [0x5100]
    pols = [policy("icm128_hmac80", ssrc=s) for s in ssrcs]
    lib = L.Session(pols)
    fail = lib.L.srtp_mi355x_debug_inject_failure
    stream = torch.cuda.current_stream().cuda_stream
    pk, nxt = _chains(rng, ssrcs, 300, [10], big=0)
    t = _stage(pk, [len(p) + 32 for p in pk])
    d = lib.prepare_device(t["arena"], t["off"], t["ln"], t["arena"],
                           t["off"], t["cap"], t["st"], stream=stream)
    fail(1, 1)                                # verdict wait sees an error
    assert lib.protect_prepared_async(d) == 1    # srtp_err_status_fail
    fail(1, 0)
    # a good async batch, then its drain fails
    pk, _ = _chains(rng, ssrcs, 300, [nxt[ssrcs[0]] + 1000], big=0)
    t = _stage(pk, [len(p) + 32 for p in pk])
    d = lib.prepare_device(t["arena"], t["off"], t["ln"], t["arena"],
                           t["off"], t["cap"], t["st"], stream=stream)
    assert lib.protect_prepared_async(d) == 0
    fail(2, 1)
    with pytest.raises(RuntimeError, match="fail"):
        lib.protect_batch([rtp_packet(rng, 0x5100, 5, 100)])
    fail(2, 0)
    # sticky: the session refuses packets and stream-state queries
    with pytest.raises(RuntimeError, match="fail"):
        lib.protect_batch([rtp_packet(rng, 0x5100, 6, 100)])
    st, _ = lib.get_roc(0x5100)
    assert int(st) == 1              # srtp_err_status_fail
    assert lib.protect_prepared_async(d) == 1
    torch.cuda.synchronize()
    lib.close()
