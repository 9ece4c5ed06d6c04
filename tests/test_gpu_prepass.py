"""Device pre-pass of srtp_protect_device (libsrtp_amd/csrc/srtp_prepass.hip)
against the CPU oracle.

The GPU pre-pass replaces the host's in-order walk (stream lookup, index
estimate, replay window, key usage) for batches of known streams whose
sequence numbers advance; everything else must fall back to the exact host
path.  Each test asserts WHICH path ran (prepass_stats) and that the bytes,
statuses, lengths and the stream state left behind (seen through later
host-path packets and get_roc) equal the sequential reference's.
"""
import random

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.test_gpu_parity import POLICIES, _gpu, policy, rtp_packet

pytestmark = pytest.mark.gpu


def _device_protect(sess, pkts, caps):
    """one srtp_protect_device call over pkts -> (status, out bytes list)"""
    import torch
    offs, pos = [], 0
    for p, c in zip(pkts, caps):
        offs.append(pos)
        pos += (max(len(p), c) + 15) & ~15
    buf = bytearray(pos + 16)
    for o, p in zip(offs, pkts):
        buf[o:o + len(p)] = p
    arena = torch.frombuffer(buf, dtype=torch.uint8).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    cap = torch.tensor(caps, dtype=torch.int32).cuda()
    st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    assert sess.protect_device(arena, off, ln, arena, off, cap, st) == 0
    st, cap = st.cpu().tolist(), cap.cpu().tolist()
    host = arena.cpu().numpy().tobytes()
    outs = [host[o:o + c] if s == 0 else None
            for o, c, s in zip(offs, cap, st)]
    return st, outs, cap


def _check(sess, orc, pkts, caps):
    st, outs, olen = _device_protect(sess, pkts, caps)
    for i, p in enumerate(pkts):
        rc, ref = orc.protect(p, caps[i])
        assert st[i] == rc, (i, st[i], rc)
        if rc == 0:
            assert outs[i] == ref, i
        else:
            assert olen[i] == caps[i], i   # error packets keep capacity


def _chains(rng, ssrcs, n, seq0, big=0.02):
    """interleaved per-SSRC packets whose sequence numbers advance by
    [1, 2^15): the fast path's domain (incl. ROC wraps and long gaps)"""
    seq = dict(zip(ssrcs, seq0))
    pk = []
    for _ in range(n):
        s = rng.choice(ssrcs)
        pk.append(rtp_packet(rng, s, seq[s] & 0xffff,
                             rng.choice([0, 1, 17, 160, 1400]),
                             rng.choice([0, 0, 2]),
                             rng.choice([-1, -1, 1])))
        step = rng.randrange(2, 0x7fff) if rng.random() < big else \
            rng.choice([1, 1, 1, 2, 5])
        seq[s] += step
    return pk, seq


MIX = ["icm128_hmac80", "icm256_hmac32", "gcm128_16", "gcm256_8",
       "null_hmac80", "icm192_hmac80", "icm128_nullauth"]


def test_fast_multi_stream_chain():
    _gpu()
    rng = random.Random(101)
    ssrcs = [0x200 + k for k in range(len(MIX))]
    pols = [policy(n, ssrc=s, seed=k) for k, (n, s) in
            enumerate(zip(MIX, ssrcs))]
    lib, orc = L.Session(pols), O.Session(pols)
    seq0 = [0xfff0, 1, 0x7fff, 0x8001, 0xff00, 40000, 7]
    for _ in range(3):
        pk, nxt = _chains(rng, ssrcs, 700, seq0)
        _check(lib, orc, pk, [len(p) + 64 for p in pk])
        seq0 = [nxt[s] for s in ssrcs]
    assert lib.prepass_stats() == (3, 0)
    for s in ssrcs:
        assert lib.get_roc(s)[1] == orc.get_roc(s)[1], hex(s)
    # the host path continues from the device-advanced state
    pk, _ = _chains(rng, ssrcs, 200, seq0)
    st, out = lib.protect_batch(pk, [len(p) + 64 for p in pk])
    for i, p in enumerate(pk):
        rc, ref = orc.protect(p, len(p) + 64)
        assert st[i] == rc and (rc or out[i] == ref), i


def test_fast_error_packets_do_not_break_the_chain():
    _gpu()
    rng = random.Random(5)
    pol = policy("icm128_hmac80", ssrc=0x77)
    lib, orc = L.Session([pol]), O.Session([pol])
    pk, caps, seq = [], [], 0x100
    for i in range(400):
        r = rng.random()
        if r < 0.05:
            pk.append(bytes([0x80, 96, 0, 1, 0, 0]))            # bad_param
            caps.append(64)
            continue
        p = rtp_packet(rng, 0x77, seq & 0xffff, rng.choice([0, 300]))
        pk.append(p)
        # buffer_small: the key is charged, the index does not move
        caps.append(len(p) + (5 if r < 0.10 else 20))
        if r >= 0.10:
            seq += rng.choice([1, 3])
    _check(lib, orc, pk, caps)
    assert lib.prepass_stats() == (1, 0)


def test_replay_in_batch_falls_back_to_host_path():
    _gpu()
    rng = random.Random(9)
    pol = policy("gcm256_16", ssrc=0x99)
    lib, orc = L.Session([pol]), O.Session([pol])
    pk, _ = _chains(rng, [0x99], 300, [500], big=0)
    _check(lib, orc, pk, [len(p) + 32 for p in pk])
    more, _ = _chains(rng, [0x99], 50, [1000], big=0)
    more.insert(20, more[10])                   # duplicate -> replay_fail
    more.insert(30, pk[-5])                     # old, in window
    _check(lib, orc, more, [len(p) + 32 for p in more])
    assert lib.prepass_stats() == (1, 1)
    # and the device path resumes on the next clean batch
    nxt, _ = _chains(rng, [0x99], 100, [2000], big=0)
    _check(lib, orc, nxt, [len(p) + 32 for p in nxt])
    assert lib.prepass_stats() == (2, 1)


def test_window_state_left_by_device_path():
    """Bits the device set (and the ones it did not) are seen by a later
    host-path replay check: seq 150 was skipped -> accepted, 160 was sent
    -> replay_fail, 40 is outside the 128-packet window -> replay_old."""
    _gpu()
    rng = random.Random(3)
    pol = policy("icm128_hmac80", ssrc=0x5, window=128)
    lib, orc = L.Session([pol]), O.Session([pol])
    seqs = [s for s in range(30, 201) if s != 150]
    pk = [rtp_packet(rng, 0x5, s, 40) for s in seqs]
    _check(lib, orc, pk, [len(p) + 16 for p in pk])
    assert lib.prepass_stats() == (1, 0)
    for s in (150, 160, 40, 201):
        p = rtp_packet(rng, 0x5, s, 40)
        st, out = lib.protect(p, len(p) + 16)
        rc, ref = orc.protect(p, len(p) + 16)
        assert st == rc, (s, st, rc)
        assert rc or out == ref


def test_template_clone_then_device_path():
    _gpu()
    rng = random.Random(21)
    pol = policy("icm128_hmac80", ssrc_type=3, seed=2)
    lib, orc = L.Session([pol]), O.Session([pol])
    ssrcs = [0x3000 + k for k in range(37)]
    pk, nxt = _chains(rng, ssrcs, 500, [rng.randrange(1, 60000)
                                        for _ in ssrcs], big=0)
    _check(lib, orc, pk, [len(p) + 16 for p in pk])   # clones on the device
    pk, _ = _chains(rng, ssrcs, 2000, [nxt[s] for s in ssrcs])
    _check(lib, orc, pk, [len(p) + 16 for p in pk])   # all known: device
    assert lib.prepass_stats() == (2, 0), lib.prepass_last_abort()
    for s in ssrcs[::5]:
        assert lib.get_roc(s) == orc.get_roc(s)


@pytest.mark.parametrize("fixed_stream", [True, False])
@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16", "gcm128_16"])
def test_template_clones_on_device_both_directions(name, fixed_stream):
    """Template sessions (ssrc_any_outbound sender, ssrc_any_inbound
    receiver; srtp_stream_clone srtp.c:762-863 at 2540 / 3141): the first
    batch of 300 unseen SSRCs creates every stream on the device, the
    receiver only for SSRCs whose packet authenticates (a forged first
    packet leaves none: the next genuine one creates it, 3117-3155); a
    stream known on the host (specific policy) beside them; three batches,
    every status and byte against the oracle called per packet, no batch on
    the host path, and the created streams' state visible through the host
    API (srtp_stream_get_roc) afterwards.  Without the fixed stream every
    stream has the template's key (one key for the batch: the order-free
    kernels' per-lane forms with one key in every lane)"""
    _gpu()
    rng = random.Random(808 + len(name) + fixed_stream)
    tx = policy(name, ssrc_type=3, seed=31)
    rx = dict(tx, ssrc_type=2)
    fixed = [policy(name, ssrc=0x0f0f0f0f, seed=32)] if fixed_stream else []
    snd, osnd = L.Session([tx] + fixed), O.Session([tx] + fixed)
    rcv, orcv = L.Session([rx] + fixed), O.Session([rx] + fixed)
    ssrcs = [0x31000000 + 11 * k for k in range(300)] + \
        ([0x0f0f0f0f] if fixed_stream else [])
    seq0 = {s: rng.randrange(1, 0xf000) for s in ssrcs}
    for b in range(3):
        pk = _interleaved(rng, ssrcs, seq0, 4, payloads=(0, 20, 160))
        st, out = _device_run(snd, pk, [len(p) + 32 for p in pk], "protect")
        srtp = []
        for i, p in enumerate(pk):
            rc, ref = osnd.protect(p, len(p) + 32)
            assert st[i] == rc, (b, i, st[i], rc)
            assert rc or out[i] == ref, (b, i)
            srtp.append(ref)
        if b == 0:
            # forge the first packet of every 7th SSRC
            seen = set()
            for i, p in enumerate(srtp):
                ss = int.from_bytes(p[8:12], "big")
                if ss not in seen:
                    seen.add(ss)
                    if ss % 7 == 0:
                        bad = bytearray(p)
                        bad[-1] ^= 0x33
                        srtp[i] = bytes(bad)
        _receive_check(rcv, orcv, srtp)
    assert snd.prepass_stats() == (3, 0), snd.prepass_last_abort()
    assert rcv.prepass_stats() == (3, 0), rcv.prepass_last_abort()
    for s in ssrcs[::13]:
        assert snd.get_roc(s) == osnd.get_roc(s), hex(s)
        assert rcv.get_roc(s) == orcv.get_roc(s), hex(s)


@pytest.mark.parametrize("name,tag", [("icm128_hmac80", 10),
                                      ("gcm256_16", 16)])
def test_configs3_template_bench_shape(name, tag):
    """BASELINE configs[3]'s template variant: 65,536 SSRCs
    under ONE ssrc_any_outbound key, 128 packets x 160 B each (8M packets,
    round-robin).  The first batch creates all 65,536 streams on the device
    (srtp_gpu_pp_clone) and runs there, as does the second; every packet of
    978 sampled SSRCs (all 64 lane positions) against the C oracle's
    template session, and every packet back through a receiver template
    session (its streams created on the device as its packets
    authenticate).  Under AES-256-GCM too (bench.py --config g711gcm)"""
    _gpu()
    import numpy as np
    import torch
    ns, per, payload = 65536, 128, 160
    rtp_len = 12 + payload
    slot = (rtp_len + tag + 15) & ~15
    n = ns * per
    base = 0x10000000
    tx = policy(name, ssrc_type=3, seed=77)
    rx = dict(tx, ssrc_type=2)
    snd, rcv = L.Session([tx]), L.Session([rx])
    sample = list(range(0, ns, 67))
    orc = O.Session([tx])
    rows = torch.tensor([k * ns + s for s in sample for k in range(per)],
                        dtype=torch.int64, device="cuda")
    gen = torch.Generator(device="cuda").manual_seed(505)
    off = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    seq0 = 0x4000
    for batch in range(2):
        a = _rr_arena(ns, per, payload, seq0, base, gen, slot)
        orig = a.clone()
        d = a.view(-1)
        ln = torch.full((n,), rtp_len, dtype=torch.int32, device="cuda")
        cap = torch.full((n,), slot, dtype=torch.int32, device="cuda")
        st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        assert snd.protect_device(d, off, ln, d, off, cap, st) == 0
        assert int((st != 0).sum()) == 0
        pin = orig[rows, :rtp_len].cpu().numpy().reshape(-1)
        m = len(sample) * per
        offs = np.arange(m, dtype=np.uint64) * rtp_len
        bad, ref, rlen = orc.protect_many(pin, offs, np.full(m, rtp_len),
                                          rtp_len + tag)
        assert bad == 0 and (rlen == rtp_len + tag).all()
        got = a[rows, :rtp_len + tag].cpu().numpy()
        diff = np.nonzero((got != ref).any(axis=1))[0]
        assert len(diff) == 0, ("oracle mismatch", batch, diff[:8])
        cap2 = torch.full((n,), slot, dtype=torch.int32, device="cuda")
        st2 = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        assert rcv.unprotect_device(d, off, cap, d, off, cap2, st2) == 0
        assert int((st2 != 0).sum()) == 0
        assert torch.equal(a[:, :rtp_len], orig[:, :rtp_len])
        del a, orig, d
        seq0 += per
    assert snd.prepass_stats() == (2, 0), snd.prepass_last_abort()
    assert rcv.prepass_stats() == (2, 0), rcv.prepass_last_abort()
    for s in sample[::97]:
        assert snd.get_roc(base + s) == orc.get_roc(base + s)


def test_receiver_stream_collision_falls_back():
    """A stream created for inbound traffic that the application protects
    on: the reference fires ssrc_collision per packet -> host path."""
    _gpu()
    rng = random.Random(4)
    pol = policy("icm128_hmac80", ssrc_type=2, seed=8)   # any inbound
    snd = policy("icm128_hmac80", ssrc_type=3, seed=8)
    tx, rx_l, rx_o = O.Session([snd]), L.Session([pol]), O.Session([pol])
    p0 = rtp_packet(rng, 0x42, 10, 30)
    _, s0 = tx.protect(p0, 100)
    assert rx_l.unprotect(s0, len(s0))[0] == 0 and \
        rx_o.unprotect(s0, len(s0))[0] == 0
    pk = [rtp_packet(rng, 0x42, 11 + k, 30) for k in range(5)]
    _check(rx_l, rx_o, pk, [len(p) + 16 for p in pk])
    assert rx_l.prepass_stats()[0] == 0


def test_many_streams_round_robin_stay_on_device():
    """The G.711 bench shape scaled down: 2048 streams with distinct keys,
    packets round-robin, three consecutive batches -- all on the device
    pre-pass, bytes equal to the oracle's."""
    _gpu()
    rng = random.Random(77)
    ns, per = 2048, 6
    ssrcs = [0x10000000 + k for k in range(ns)]
    pols = [policy("icm128_hmac80", ssrc=s, seed=k) for k, s in
            enumerate(ssrcs)]
    lib, orc = L.Session(pols), O.Session(pols)
    seq0 = 0x1234
    for b in range(3):
        pk = [rtp_packet(rng, ssrcs[i % ns], (seq0 + i // ns) & 0xffff, 160)
              for i in range(ns * per)]
        _check(lib, orc, pk, [len(p) + 16 for p in pk])
        assert lib.prepass_last_abort() == 0, (b, lib.prepass_last_abort())
        seq0 += per
    assert lib.prepass_stats() == (3, 0)


def test_device_api_orders_after_torch_default_stream():
    """stream=NULL is the HIP null stream (PyTorch's default stream handle
    is 0): headers and capacities written by torch kernels right before the
    call must be what the pre-pass reads.  Regression: NULL once meant the
    session's own non-blocking stream and raced with those writes."""
    _gpu()
    import torch
    n, payload, ns = 1 << 21, 20, 4096
    pol = [policy("icm128_hmac80", ssrc=0x10000000 + k, seed=k)
           for k in range(ns)]
    lib = L.Session(pol)
    slot = (12 + payload + 10 + 15) & ~15
    dev = torch.device("cuda", 0)
    idx = torch.arange(n, dtype=torch.int64, device=dev)
    for b in range(3):
        arena = torch.randint(0, 256, (n, slot), dtype=torch.uint8, device=dev)
        arena[:, 0], arena[:, 1] = 0x80, 96
        ss = 0x10000000 + idx % ns
        for k in range(4):
            arena[:, 8 + k] = ((ss >> (24 - 8 * k)) & 0xff).to(torch.uint8)
        seq = (0x1234 + b * (n // ns) + idx // ns) & 0xffff
        arena[:, 2] = (seq >> 8).to(torch.uint8)
        arena[:, 3] = (seq & 0xff).to(torch.uint8)
        off = idx * slot
        ln = torch.full((n,), 12 + payload, dtype=torch.int32, device=dev)
        cap = torch.full((n,), slot, dtype=torch.int32, device=dev)
        st = torch.full((n,), -1, dtype=torch.int32, device=dev)
        flat = arena.view(-1)
        assert lib.protect_device(flat, off, ln, flat, off, cap, st) == 0
        assert int((st != 0).sum()) == 0, b
        assert bool((cap == 12 + payload + 10).all()), b
    assert lib.prepass_stats() == (3, 0), lib.prepass_last_abort()


# --------------------------------------------------------------------------
# the order-free form of the many-stream pre-pass (no sort): packets of a
# stream may arrive in any order inside one replay window

def _interleaved(rng, ssrcs, seq0, per, shuffle_within=0, steps=(1, 1, 1, 2),
                 payloads=(0, 33, 160)):
    """per packets per stream, streams interleaved at random; each stream's
    sequence numbers advance by `steps`; with shuffle_within > 0 neighbouring
    packets of one stream may be swapped (reordering inside the window)"""
    chains = {}
    for s in ssrcs:
        q, seqs = seq0[s], []
        for _ in range(per):
            seqs.append(q & 0xffff)
            q += rng.choice(steps)
        if shuffle_within:
            for k in range(len(seqs) - 1):
                if rng.random() < shuffle_within:
                    seqs[k], seqs[k + 1] = seqs[k + 1], seqs[k]
        chains[s] = seqs
        seq0[s] = q
    order = [s for s in ssrcs for _ in range(per)]
    rng.shuffle(order)
    pos = {s: 0 for s in ssrcs}
    pk = []
    for s in order:
        pk.append(rtp_packet(rng, s, chains[s][pos[s]], rng.choice(payloads)))
        pos[s] += 1
    return pk


def _stream_set(n, name="icm128_hmac80"):
    ssrcs = [0x20000000 + 7 * k for k in range(n)]
    pols = [policy(name, ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    return ssrcs, L.Session(pols), O.Session(pols)


def test_order_free_reordered_streams_stay_on_device():
    _gpu()
    rng = random.Random(501)
    ssrcs, lib, orc = _stream_set(300)
    seq0 = {s: rng.randrange(1, 0x10000) for s in ssrcs}
    for b in range(3):
        # <= 50 packets, advances of 1..2: every batch spans < 128 indices
        pk = _interleaved(rng, ssrcs, seq0, 50, shuffle_within=0.2)
        _check(lib, orc, pk, [len(p) + 16 for p in pk])
    assert lib.prepass_stats() == (3, 0), lib.prepass_last_abort()
    assert lib.prepass_sorted_batches() == 0
    for s in ssrcs[::37]:
        assert lib.get_roc(s)[1] == orc.get_roc(s)[1]


def test_order_free_long_chain_takes_sorted_path():
    """a stream with more packets than its 128-packet window in one batch"""
    _gpu()
    rng = random.Random(502)
    ssrcs, lib, orc = _stream_set(5, "gcm128_16")
    seq0 = {s: 0xff00 + 3 * k for k, s in enumerate(ssrcs)}
    pk = _interleaved(rng, ssrcs, seq0, 200)
    _check(lib, orc, pk, [len(p) + 32 for p in pk])
    assert lib.prepass_stats() == (1, 0)
    assert lib.prepass_sorted_batches() == 1


def test_order_free_duplicate_goes_to_host():
    _gpu()
    rng = random.Random(503)
    ssrcs, lib, orc = _stream_set(50)
    seq0 = {s: 100 for s in ssrcs}
    pk = _interleaved(rng, ssrcs, seq0, 20)
    pk.insert(500, pk[17])                      # replay inside the batch
    _check(lib, orc, pk, [len(p) + 16 for p in pk])
    assert lib.prepass_stats() == (0, 1)
    # and the next clean batch is back on the device
    pk = _interleaved(rng, ssrcs, seq0, 20)
    _check(lib, orc, pk, [len(p) + 16 for p in pk])
    assert lib.prepass_stats() == (1, 1)


def test_configs3_shape_64k_distinct_key_streams():
    """BASELINE configs[3] at its own stream count: 65,536 streams with
    distinct master keys x 160-byte payloads, packets round-robin, two
    batches (2 and 3 packets per stream); every byte against the oracle."""
    _gpu()
    rng = random.Random(504)
    ns = 65536
    ssrcs = [0x10000000 + k for k in range(ns)]
    pols = [policy("icm128_hmac80", ssrc=s, seed=k) for k, s in
            enumerate(ssrcs)]
    lib, orc = L.Session(pols), O.Session(pols)
    seq0 = 0x7ff0
    for per in (2, 3):
        pk = [rtp_packet(rng, ssrcs[i % ns], (seq0 + i // ns) & 0xffff, 160)
              for i in range(ns * per)]
        _check(lib, orc, pk, [len(p) + 16 for p in pk])
        seq0 += per
    assert lib.prepass_stats() == (2, 0), lib.prepass_last_abort()
    assert lib.prepass_sorted_batches() == 0


@pytest.mark.parametrize("buckets", [0, 1])
@pytest.mark.parametrize("op", ["protect", "unprotect"])
def test_configs3_shape_64k_gcm256_streams_fused(op, buckets):
    """65,536 AES-256-GCM streams with distinct keys, packets round-robin,
    in place: the order-free form classified inside k_gcm (srtp_fused.h,
    per-lane keys), or with key buckets on the pre-pass form whose streams
    of 2-3 packets take k_gcm's per-lane record walk; two batches; every
    status and byte against the oracle called once per packet (protect, or
    the receive side of what the oracle's sender protected)"""
    _gpu()
    L.lib().srtp_mi355x_set_key_buckets(buckets)
    rng = random.Random(909)
    ns = 65536
    ssrcs = [0x11000000 + k for k in range(ns)]
    pols = [policy("gcm256_16", ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    lib, orc = L.Session(pols), O.Session(pols)
    snd = O.Session(pols)
    seq0 = 0x9000
    for per in (2, 3):
        pk = [rtp_packet(rng, ssrcs[i % ns], (seq0 + i // ns) & 0xffff,
                         rng.choice([0, 20, 160]))
              for i in range(ns * per)]
        _pending_run(lib, orc, snd, op, pk)
        seq0 += per
    L.lib().srtp_mi355x_set_key_buckets(-1)
    assert lib.prepass_stats() == (2, 0), lib.prepass_last_abort()
    assert lib.prepass_sorted_batches() == 0


@pytest.mark.parametrize("buckets", [1, -1])
@pytest.mark.parametrize("op", ["protect", "unprotect"])
@pytest.mark.parametrize("ciphers", ["mixed", "gcm", "gcm128_8"])
def test_key_buckets_both_regions_and_mixed_ciphers(ciphers, op, buckets):
    """key buckets with both regions in one batch -- streams of 90-120
    packets (wave buckets: k_gcm_bk / KM_WAVE) beside streams of 1-3 (the
    per-lane record walks) -- over AES-256-GCM and AES-128-ICM streams mixed
    (each cipher's launch skips the other's groups and records) or GCM
    only (AES-256-GCM-16, or AES-128-GCM and AES-256-GCM-8 alternating:
    the AES-128 kernel and the 8-byte tag), three batches; every status and
    byte against the oracle.  With
    buckets on (1) and in the default mode (-1: the GCM-only batches, with
    over 32 packets a stream on average, take them; the mixed ones run the
    fused forms)"""
    _gpu()
    L.lib().srtp_mi355x_set_key_buckets(buckets)
    try:
        rng = random.Random(911 + buckets)
        nb, nsm = (40, 900) if ciphers == "mixed" else (100, 150)
        big = [0x12000000 + k for k in range(nb)]
        small = [0x12100000 + k for k in range(nsm)]
        def pname(k):
            if ciphers == "gcm128_8":
                return "gcm128_16" if k % 2 else "gcm256_8"
            return "gcm256_16" if k % 2 or ciphers == "gcm" else \
                "icm128_hmac80"
        pols = [policy(pname(k), ssrc=s, seed=k)
                for k, s in enumerate(big + small)]
        lib, orc, snd = L.Session(pols), O.Session(pols), O.Session(pols)
        seq0 = {s: rng.randrange(1, 0xff00) for s in big + small}
        d0, h0 = lib.prepass_stats()
        k0 = lib.bucket_batches()
        for b in range(3):
            # (one step per packet in the big streams: a batch's span stays
            # inside the 128-bit window, so the order-free form holds)
            pk = _interleaved(rng, big, seq0, rng.randrange(90, 120),
                              steps=(1,), payloads=(0, 20, 160, 1000))
            pk += _interleaved(rng, small, seq0, rng.randrange(1, 4),
                               payloads=(0, 20, 160))
            _pending_run(lib, orc, snd, op, pk)
        assert lib.prepass_stats() == (d0 + 3, h0), lib.prepass_last_abort()
        bucketed = buckets == 1 or ciphers != "mixed"
        assert lib.bucket_batches() == k0 + (3 if bucketed else 0)
    finally:
        L.lib().srtp_mi355x_set_key_buckets(-1)


def _rr_arena(ns, per, payload, seq0, base_ssrc, gen, slot):
    """configs[3]-shaped arena on the GPU: ns streams round-robin, per
    packets each (packet i: stream i % ns, its packet i // ns)"""
    import torch
    n = ns * per
    a = torch.randint(0, 256, (n, slot), dtype=torch.uint8, device="cuda",
                      generator=gen)
    idx = torch.arange(n, dtype=torch.int64, device="cuda")
    a[:, 0] = 0x80
    a[:, 1] = 96
    seq = (idx // ns + seq0) & 0xffff
    a[:, 2] = (seq >> 8).to(torch.uint8)
    a[:, 3] = (seq & 0xff).to(torch.uint8)
    a[:, 4:8] = 0
    ssrc = base_ssrc + idx % ns
    for k in range(4):
        a[:, 8 + k] = ((ssrc >> (24 - 8 * k)) & 0xff).to(torch.uint8)
    return a


@pytest.mark.parametrize("buckets", [0, 1])
@pytest.mark.parametrize("name,tag", [("icm128_hmac80", 10),
                                      ("gcm256_16", 16)])
def test_configs3_bench_shape_128_per_stream(name, tag, buckets):
    """BASELINE configs[3] at the bench's own shape: 65,536 streams with
    distinct master keys x 128 packets x 160 B (8M packets, round-robin), so
    every stream's batch spans hi - est = 127 against its 128-bit window --
    the order-free form's acceptance boundary -- and the crypto runs from
    the key buckets (one key per wave).  Two consecutive batches.  Every
    packet of 978 sampled streams covering all 64 lane positions (125,184
    per batch) is compared byte for byte with the C oracle in stream order; every packet of the batch
    must come back bit-identical through srtp_unprotect_device.  Under
    AES-256-GCM too: per-lane keys read each key's 4-bit GHASH table, the
    buckets give a wave one key (k_gcm_bk, the key's table in LDS)."""
    _gpu()
    import numpy as np
    import torch
    ns, per, payload = 65536, 128, 160
    rtp_len = 12 + payload
    slot = (rtp_len + tag + 15) & ~15
    n = ns * per
    base = 0x10000000
    pols = [policy(name, ssrc=base + k, seed=k) for k in range(ns)]
    snd, rcv = L.Session(pols), L.Session(pols)
    snd.L.srtp_mi355x_set_key_buckets(buckets)
    # packet i runs on lane i mod 64 of its wave and i = k * ns + s, so
    # stream s always runs on lane s mod 64: a step of 67 samples every lane
    # position (978 streams), each lane's cached stream record and round
    # keys reused across its 64 packets of one stream at this shape
    sample = list(range(0, ns, 67))
    assert len({s % 64 for s in sample}) == 64
    orc = O.Session([pols[s] for s in sample])
    # sampled packets in stream order: stream s, its packets k = 0..per-1
    rows = torch.tensor([k * ns + s for s in sample for k in range(per)],
                        dtype=torch.int64, device="cuda")
    gen = torch.Generator(device="cuda").manual_seed(303)
    off = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    seq0 = 0xff00    # batch 2 runs 0xff80 .. 0x007f: across a ROC boundary
    for batch in range(2):
        a = _rr_arena(ns, per, payload, seq0, base, gen, slot)
        orig = a.clone()
        d = a.view(-1)
        ln = torch.full((n,), rtp_len, dtype=torch.int32, device="cuda")
        cap = torch.full((n,), slot, dtype=torch.int32, device="cuda")
        st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        assert snd.protect_device(d, off, ln, d, off, cap, st) == 0
        assert int((st != 0).sum()) == 0
        assert bool((cap == rtp_len + tag).all())
        # the oracle on the sampled streams
        pin = orig[rows, :rtp_len].cpu().numpy().reshape(-1)
        m = len(sample) * per
        offs = np.arange(m, dtype=np.uint64) * rtp_len
        bad, ref, rlen = orc.protect_many(pin, offs, np.full(m, rtp_len),
                                          rtp_len + tag)
        assert bad == 0 and (rlen == rtp_len + tag).all()
        got = a[rows, :rtp_len + tag].cpu().numpy()
        diff = np.nonzero((got != ref).any(axis=1))[0]
        assert len(diff) == 0, ("oracle mismatch", diff[:8])
        # every packet back through the receiver
        cap2 = cap.clone()
        st2 = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        assert rcv.unprotect_device(d, off, cap, d, off, cap2, st2) == 0
        assert int((st2 != 0).sum()) == 0
        assert bool((cap2 == rtp_len).all())
        assert torch.equal(a[:, :rtp_len], orig[:, :rtp_len])
        del a, orig, d
        seq0 = (seq0 + per) & 0xffff
    assert snd.prepass_stats() == (2, 0), snd.prepass_last_abort()
    assert rcv.prepass_stats() == (2, 0), rcv.prepass_last_abort()
    assert snd.prepass_sorted_batches() == 0
    assert snd.bucket_batches() == (2 if buckets else 0)
    assert rcv.bucket_batches() == (2 if buckets else 0)
    snd.L.srtp_mi355x_set_key_buckets(-1)


def _rtp_headers(a, lens, rng):
    """CSRCs and RFC 8285 extensions in the configs[3]-shaped arena `a`
    (uint8 (n, slot) on the GPU; SSRC and sequence numbers kept): 0, 1 or
    3 CSRCs, and for a third of the packets a 0xBEDE extension of 0..2
    words; returns the lengths raised to hold each header"""
    import numpy as np
    import torch
    n = a.shape[0]
    cc = rng.choice(np.array([0, 0, 1, 3]), n)
    x = rng.random(n) < 0.3
    xw = rng.integers(0, 3, n)
    hl = 12 + 4 * cc + np.where(x, 4 + 4 * xw, 0)
    host = a.cpu().numpy()
    host[:, 0] = 0x80 | cc | (x.astype(np.int64) << 4)
    idx = np.nonzero(x)[0]
    e = 12 + 4 * cc[idx]
    host[idx, e] = 0xbe
    host[idx, e + 1] = 0xde
    host[idx, e + 2] = 0
    host[idx, e + 3] = xw[idx]
    a.copy_(torch.from_numpy(host).cuda())
    return np.maximum(lens, hl)


@pytest.mark.parametrize("lengths,slot", [("uniform160", 192), ("mixed", 192),
                                          ("mixed", 320)])
def test_fused_midsize_every_packet_lane_reuse(lengths, slot):
    """The fused order-free path at a size where the persistent grid's
    stride (256 CUs x 512 lanes = 2^17) is below the batch: 2^18 packets
    over 2,048 distinct-key streams, round-robin, so every lane runs two
    packets of ONE stream -- the second takes fz_lookup's cached stream
    record and LaneKey::reload's kept round keys.  192-byte slots take the
    LDS-staged kernel (k_icm_stg: every wave group's slots tile one span),
    320-byte slots the per-lane form.  "mixed": lengths 12..166 with CSRCs
    and header extensions.  EVERY packet is compared with the C oracle,
    protect and then unprotect, both in place; two consecutive batches (the
    second across a ROC boundary)."""
    _gpu()
    import numpy as np
    import torch
    ns, per, tag = 2048, 128, 10
    n = ns * per
    base = 0x20000000
    pols = [policy("icm128_hmac80", ssrc=base + k, seed=7000 + k)
            for k in range(ns)]
    snd, rcv = L.Session(pols), L.Session(pols)
    osnd, orcv = O.Session(pols), O.Session(pols)
    gen = torch.Generator(device="cuda").manual_seed(404)
    off = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    rng = np.random.default_rng(405)
    # batch 1: 0xff40..0xffbf; batch 2 wraps (0xffc0..0x003f) from a stored
    # index above 2^15 (a fresh stream's first batch must not wrap: from
    # index 0 the reference takes seq as the index, srtp.c:2038-2071, and
    # the packets after the wrap then go through the sorted chain form)
    seq0 = 0xff40
    for batch in range(2):
        a = _rr_arena(ns, per, 0, seq0, base, gen, slot)
        if lengths == "uniform160":
            lens = np.full(n, 12 + 160, dtype=np.int64)
        else:
            lens = _rtp_headers(a, rng.integers(12, 192 - tag - 16, n), rng)
        orig = a.clone()
        d = a.view(-1)
        ln = torch.from_numpy(lens.astype(np.int32)).cuda()
        cap = torch.full((n,), slot, dtype=torch.int32, device="cuda")
        st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        assert snd.protect_device(d, off, ln, d, off, cap, st) == 0
        assert int((st != 0).sum()) == 0
        assert torch.equal(cap, ln + tag)
        host_in = orig.cpu().numpy().reshape(-1)
        offs = np.arange(n, dtype=np.uint64) * slot
        bad, ref, rlen = osnd.protect_many(host_in, offs, lens, slot)
        assert bad == 0 and (rlen == lens + tag).all()
        got = a.cpu().numpy()
        for i in range(0, n, 1 << 15):      # every packet, in slices
            g = got[i:i + (1 << 15)]
            r = ref[i:i + (1 << 15)]
            ln_i = lens[i:i + (1 << 15)] + tag
            mask = np.arange(slot)[None, :] < ln_i[:, None]
            diff = np.nonzero(((g != r) & mask).any(axis=1))[0]
            assert len(diff) == 0, ("protect mismatch", batch, i + diff[:8])
        # receive side, in place, against the oracle's receiver
        cap2 = torch.full((n,), slot, dtype=torch.int32, device="cuda")
        st2 = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        assert rcv.unprotect_device(d, off, cap.clone(), d, off, cap2, st2) == 0
        ost, oref, olen = orcv.unprotect_many(got.reshape(-1), offs,
                                              lens + tag, slot)
        assert (ost == 0).all() and (olen == lens).all()
        assert int((st2 != 0).sum()) == 0 and torch.equal(cap2, ln)
        back = a.cpu().numpy()
        mask = np.arange(slot)[None, :] < lens[:, None]
        diff = np.nonzero(((back != oref) & mask).any(axis=1))[0]
        assert len(diff) == 0, ("unprotect mismatch", batch, diff[:8])
        assert not ((back != orig.cpu().numpy()) & mask).any()
        del a, orig, d
        seq0 = (seq0 + per) & 0xffff
    assert snd.prepass_stats() == (2, 0), snd.prepass_last_abort()
    assert rcv.prepass_stats() == (2, 0), rcv.prepass_last_abort()
    assert snd.prepass_sorted_batches() == 0
    for s in (base, base + 1, base + 63, base + ns - 1):
        assert snd.get_roc(s)[1] == osnd.get_roc(s)[1]


@pytest.mark.parametrize("case", ["duplicate", "unknown_ssrc", "long_chain"])
def test_staged_declined_batch_is_restored(case):
    """A batch of the LDS-staged kernel's shape (192-byte slots, capacity =
    slot) that the order-free form declines: the staged kernel has written
    every slot back (protected packets, tags, the rest of each slot as it
    was); the decline restores it, then the host path (duplicate, unknown
    SSRC) or the sorted chain form (a stream with more packets than its
    window) runs.  Every status and byte equal to the oracle's, and every
    slot byte past each protected packet exactly as it was."""
    _gpu()
    import numpy as np
    import torch
    rng = np.random.default_rng(900 + len(case))
    ns, per, slot, tag = 256, 64, 192, 10
    base = 0x30000000
    pols = [policy("icm128_hmac80", ssrc=base + k, seed=9000 + k)
            for k in range(ns)]
    lib, orc = L.Session(pols), O.Session(pols)
    gen = torch.Generator(device="cuda").manual_seed(901)
    a = _rr_arena(ns, per, 0, 0x1000, base, gen, slot)
    n = ns * per
    lens = rng.integers(12, slot - tag, n)
    if case == "duplicate":
        a[5000] = a[300]
        lens[5000] = lens[300]
    elif case == "unknown_ssrc":
        a[777, 8:12] = torch.tensor([0x0b, 0xad, 0x0b, 0xad], dtype=torch.uint8)
    else:
        # stream 3's packets advance past its 128-packet window
        k = np.arange(3, n, ns)
        seqs = 0x1000 + 3 * np.arange(len(k))
        h = a[torch.from_numpy(k).cuda(), :4].cpu().numpy()
        h[:, 2] = (seqs >> 8) & 0xff
        h[:, 3] = seqs & 0xff
        a[torch.from_numpy(k).cuda(), :4] = torch.from_numpy(h).cuda()
    orig = a.cpu().numpy().copy()
    d = a.view(-1)
    off = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    ln = torch.from_numpy(lens.astype(np.int32)).cuda()
    cap = torch.full((n,), slot, dtype=torch.int32, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    assert lib.protect_device(d, off, ln, d, off, cap, st) == 0
    st, cap, got = st.cpu().numpy(), cap.cpu().numpy(), a.cpu().numpy()
    for i in range(n):
        rc, ref = orc.protect(bytes(orig[i, :lens[i]]), slot)
        assert st[i] == rc, (i, st[i], rc)
        if rc == 0:
            assert bytes(got[i, :cap[i]]) == ref, i
            assert (got[i, cap[i]:] == orig[i, cap[i]:]).all(), i
        else:
            assert cap[i] == slot and (got[i] == orig[i]).all(), i
    want = {"duplicate": (0, 1), "unknown_ssrc": (0, 1), "long_chain": (1, 0)}
    assert lib.prepass_stats() == want[case], lib.prepass_last_abort()


# --------------------------------------------------------------------------
# the order-free form classified inside the AES-ICM kernel (in place, one
# ICM variant, per-lane keys: srtp_prepass.hip pp_protect_fused): a batch it
# declines must come back untouched before the sorted / host path runs

def _device_protect_raw(sess, pkts, caps, fill=0xa5):
    """in place; the capacity region past each packet pre-filled with
    `fill`; returns (status, arena bytes, offsets, out lengths)"""
    import torch
    offs, pos = [], 0
    for p, c in zip(pkts, caps):
        offs.append(pos)
        pos += (max(len(p), c) + 15) & ~15
    buf = bytearray([fill]) * (pos + 16)
    for o, p in zip(offs, pkts):
        buf[o:o + len(p)] = p
    orig = bytes(buf)
    arena = torch.frombuffer(buf, dtype=torch.uint8).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    cap = torch.tensor(caps, dtype=torch.int32).cuda()
    st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    assert sess.protect_device(arena, off, ln, arena, off, cap, st) == 0
    return st.cpu().tolist(), arena.cpu().numpy().tobytes(), orig, offs, \
        cap.cpu().tolist()


@pytest.mark.parametrize("name", ["icm128_hmac80", "icm128_nullauth",
                                  "icm256_hmac32", "gcm256_16", "gcm256_8"])
@pytest.mark.parametrize("caps_mode", ["roomy", "tight"])
@pytest.mark.parametrize("case", ["duplicate", "unknown_ssrc", "long_chain"])
def test_fused_order_free_declined_batch_is_restored(case, caps_mode, name):
    """duplicate -> host path, unknown SSRC -> host path, a stream with more
    packets than its window -> the sorted chain form: statuses and bytes
    equal to the oracle's, and every rejected packet's bytes up to its
    capacity (its trailer space included) exactly as they were; "tight":
    capacities of the tag's length (+0..2), the trailer save reading around
    the tag space at every byte alignment; tags of 10, 0 and 4 bytes"""
    _gpu()
    rng = random.Random(600 + len(case))
    ssrcs, lib, orc = _stream_set(40, name)
    seq0 = {s: 0xfff0 - 3 * k for k, s in enumerate(ssrcs)}
    pk = _interleaved(rng, ssrcs, seq0, 150 if case == "long_chain" else 20,
                      payloads=(0, 1, 2, 3, 4, 5, 6, 7, 33, 160))
    if case == "duplicate":
        pk.insert(300, pk[17])
    elif case == "unknown_ssrc":
        pk.insert(100, rtp_packet(rng, 0x0bad0bad, 5, 40))
    if caps_mode == "roomy":
        caps = [len(p) + 16 for p in pk]
    else:
        tag = {"icm128_hmac80": 10, "icm128_nullauth": 0,
               "icm256_hmac32": 4, "gcm256_16": 16, "gcm256_8": 8}[name]
        caps = [len(p) + tag + rng.randrange(0, 3) for p in pk]
    st, got, orig, offs, olen = _device_protect_raw(lib, pk, caps)
    for i, p in enumerate(pk):
        rc, ref = orc.protect(p, caps[i])
        assert st[i] == rc, (i, st[i], rc)
        o = offs[i]
        if rc == 0:
            assert got[o:o + olen[i]] == ref, i
        else:
            assert got[o:o + caps[i]] == orig[o:o + caps[i]], i
    if case == "long_chain":
        assert lib.prepass_stats() == (1, 0)
        assert lib.prepass_sorted_batches() == 1
    else:
        assert lib.prepass_stats() == (0, 1)


def test_fused_order_free_trailer_space_untouched_on_success():
    """accepted packets: bytes past packet + tag up to the capacity are not
    written (the saved-trailer logic reads exactly the tag's bytes)"""
    _gpu()
    rng = random.Random(611)
    ssrcs, lib, orc = _stream_set(64)
    seq0 = {s: 7 for s in ssrcs}
    pk = _interleaved(rng, ssrcs, seq0, 8, payloads=(0, 1, 2, 3, 4, 5, 6, 7, 160))
    caps = [len(p) + 10 + rng.randrange(0, 40) for p in pk]
    st, got, orig, offs, olen = _device_protect_raw(lib, pk, caps)
    assert lib.prepass_stats() == (1, 0)
    for i, p in enumerate(pk):
        rc, ref = orc.protect(p, caps[i])
        assert st[i] == rc == 0
        o = offs[i]
        assert got[o:o + olen[i]] == ref
        assert got[o + olen[i]:o + caps[i]] == orig[o + olen[i]:o + caps[i]]


def test_fused_window_sizes_jumps_and_state():
    """the fused order-free form's replay windows (srtp_prepass.hip
    k_fz_stream: a bitmap of the batch's indices mod the window size rounded
    up to a power of two, merged into the shifted stored window) at window
    sizes 64, 96, 160 and 1024, with streams that jump past their whole
    window inside the batch; the windows left behind are probed packet by
    packet through the host path (skipped indices accepted, sent ones
    replay_fail, ones past the window replay_old) against the oracle"""
    _gpu()
    rng = random.Random(612)
    wins = [64, 96, 160, 1024]
    ssrcs = [0x21000000 + 5 * k for k in range(48)]
    pols = [policy("icm128_hmac80", ssrc=s, seed=k, window=wins[k % 4])
            for k, s in enumerate(ssrcs)]
    lib, orc = L.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(100, 0xf000) for s in ssrcs}
    sent = {s: [] for s in ssrcs}
    for b in range(3):
        if b == 1:   # every third stream jumps ahead by 70 .. 3000
            for s in ssrcs[::3]:
                seq0[s] += rng.randrange(70, 3000)
        pk = _interleaved(rng, ssrcs, seq0, 24, shuffle_within=0.3,
                          payloads=(0, 5, 160))
        for p in pk:
            sent[int.from_bytes(p[8:12], "big")].append(
                int.from_bytes(p[2:4], "big"))
        _check(lib, orc, pk, [len(p) + 16 for p in pk])
        assert lib.prepass_last_abort() == 0, (b, lib.prepass_last_abort())
    assert lib.prepass_stats() == (3, 0)
    assert lib.prepass_sorted_batches() == 0
    for k, s in enumerate(ssrcs):
        assert lib.get_roc(s)[1] == orc.get_roc(s)[1]
        top = (seq0[s] - 1) & 0xffff
        probes = {top - d for d in (1, 2, 3, 7, 40, 63, 64, 65, 95, 96, 97,
                                    159, 160, 161, 700, 1023, 1024, 1100)}
        probes |= set(rng.sample(sent[s], 3))
        for q in sorted(probes):
            if not 0 < q < 0x10000:
                continue
            p = rtp_packet(rng, s, q & 0xffff, 20)
            st, out = lib.protect(p, len(p) + 16)
            rc, ref = orc.protect(p, len(p) + 16)
            assert st == rc, (k, wins[k % 4], top - q, st, rc)
            assert rc or out == ref


def _device_run(sess, pkts, caps, op, mki=None):
    """one srtp_{un}protect_device call in place -> (status, outputs)"""
    import torch
    offs, pos = [], 0
    for p, c in zip(pkts, caps):
        offs.append(pos)
        pos += (max(len(p), c) + 15) & ~15
    buf = bytearray(pos + 16)
    for o, p in zip(offs, pkts):
        buf[o:o + len(p)] = p
    arena = torch.frombuffer(buf, dtype=torch.uint8).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    cap = torch.tensor(caps, dtype=torch.int32).cuda()
    st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    fn = sess.protect_device if op == "protect" else sess.unprotect_device
    kw = {"mki": mki} if mki is not None else {}
    assert fn(arena, off, ln, arena, off, cap, st, **kw) == 0
    st, cap = st.cpu().tolist(), cap.cpu().tolist()
    host = arena.cpu().numpy().tobytes()
    return st, [host[o:o + c] if s == 0 else None
                for o, c, s in zip(offs, cap, st)]


def _key_left_equal(lib, orc, ssrcs, nkeys):
    for s in ssrcs:
        for j in range(nkeys):
            rc, got = lib.debug_key_left(s, j)
            orc_rc, want = orc.key_left(s, j)
            assert rc == 0 and orc_rc == 0, (s, j, rc, orc_rc)
            assert got == want, (hex(s), j, got, want)


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_mki_streams_on_device_prepass(name):
    """MKI streams (srtp.c:1961-2036, 2536-2545) on the device pre-pass:
    protect batches run every packet on the master key its mki_index
    selects -- one index for the batch or a different one per packet -- and
    charge the use to that key (key.c:74-90); a batch with an index past a
    stream's keys (bad_mki) takes the host path.  Receive batches run on the
    device whatever keys their MKIs select (srtp.c:1961-2016 per packet).
    Every status and byte against the oracle, one packet at a time, and
    every key's remaining uses."""
    _gpu()
    rng = random.Random(613)
    ssrcs = [0x22000000 + 3 * k for k in range(24)]
    pols = [policy(name, ssrc=s, seed=k, mki=4, nkeys=3)
            for k, s in enumerate(ssrcs)]
    snd, orc = L.Session(pols), O.Session(pols)
    rcv, orc_r = L.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(1, 0xff00) for s in ssrcs}
    plan = [("uniform", 0, 1), ("uniform", 2, 1), ("uniform", 2, 1),
            ("mixed", None, 1), ("mixed", None, 1), ("bad", None, 0),
            ("uniform", 1, 1), ("uniform", 1, 1), ("mixed", None, 1)]
    d0, h0 = 0, 0
    for kind, j, dev in plan:
        pk = _interleaved(rng, ssrcs, seq0, 12, payloads=(0, 7, 160))
        mki = [j] * len(pk) if kind == "uniform" else \
            [rng.randrange(3) for _ in pk]
        if kind == "bad":
            mki[rng.randrange(len(pk))] = 3   # srtp_err_status_bad_mki
        caps = [len(p) + 32 for p in pk]
        for i in rng.sample(range(len(pk)), 5):
            caps[i] = len(pk[i]) + 2           # buffer_small: charged too
        st, out = _device_run(snd, pk, caps, "protect", mki)
        sent = []
        for i, p in enumerate(pk):
            rc, ref = orc.protect(p, caps[i], mki[i])
            assert st[i] == rc, (kind, i, st[i], rc)
            assert rc or out[i] == ref, (kind, i)
            if rc == 0:
                sent.append(ref)
        d, h = snd.prepass_stats()
        assert (d - d0, h - h0) == ((1, 0) if dev else (0, 1)), (kind, j)
        d0, h0 = d, h
        _key_left_equal(snd, orc, ssrcs[::4], 3)
        # the receiver: first batch of a new key on the host, then device
        st, out = _device_run(rcv, sent, [len(p) for p in sent], "unprotect")
        for i, p in enumerate(sent):
            rc, ref = orc_r.unprotect(p, len(p))
            assert st[i] == rc, ("rx", kind, i, st[i], rc)
            assert rc or out[i] == ref, ("rx", kind, i)
    rd, rh = rcv.prepass_stats()
    # keys 0, 2, 2, mixed, mixed, mixed, 1, 1, mixed: every receive batch on
    # the device, each packet on the key its MKI selects (k_pu_classify)
    assert (rd, rh) == (len(plan), 0), (rd, rh)
    _key_left_equal(rcv, orc_r, ssrcs[::4], 3)
    for s in ssrcs[::5]:
        assert snd.get_roc(s)[1] == orc.get_roc(s)[1]
        assert rcv.get_roc(s)[1] == orc_r.get_roc(s)[1]


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_mki_one_stream_mixed_keys_on_device(name):
    """one MKI stream (the one-stream chain form, k_pp_chain1): 4k-packet
    protect batches whose packets pick master keys 0-3 at random run on the
    device, every packet on its key, bytes / statuses / per-key uses equal
    to the oracle; a second session with a template (ssrc_any_outbound, 4
    keys) does the same through device-created streams"""
    _gpu()
    rng = random.Random(615)
    ssrc = 0x22400000
    pols = [policy(name, ssrc=ssrc, seed=3, mki=4, nkeys=4)]
    for variant in ("stream", "template"):
        if variant == "template":
            pols = [dict(policy(name, ssrc=0, seed=5, mki=4, nkeys=4),
                         ssrc_type=3)]
            ssrcs = [0x22500000 + k for k in range(37)]
        else:
            ssrcs = [ssrc]
        lib, orc = L.Session(pols), O.Session(pols)
        seq0 = {s: rng.randrange(1, 0xff00) for s in ssrcs}
        d0, h0 = lib.prepass_stats()
        for b in range(3):
            pk = _interleaved(rng, ssrcs, seq0, 4096 // len(ssrcs),
                              payloads=(0, 20, 172))
            mki = [rng.randrange(4) for _ in pk]
            caps = [len(p) + 32 for p in pk]
            st, out = _device_run(lib, pk, caps, "protect", mki)
            for i, p in enumerate(pk):
                rc, ref = orc.protect(p, caps[i], mki[i])
                assert st[i] == rc, (variant, b, i, st[i], rc)
                assert rc or out[i] == ref, (variant, b, i)
        d, h = lib.prepass_stats()
        assert (d - d0, h - h0) == (3, 0), (variant, d - d0, h - h0)
        _key_left_equal(lib, orc, ssrcs[:5], 4)


# --------------------------------------------------------------------------
# the receive side's order-free form classified inside the AES-ICM kernel
# (srtp_prepass.hip pp_unprotect_fused): several streams, in place

def _send_batches(snd, ssrcs, seq0, per, nb, rng, payloads=(0, 7, 160)):
    out = []
    for _ in range(nb):
        pk = _interleaved(rng, ssrcs, seq0, per, payloads=payloads)
        sent = []
        for p in pk:
            rc, ref = snd.protect(p, len(p) + 32)
            assert rc == 0
            sent.append(ref)
        out.append(sent)
    return out


def _receive_check(lib, orc, pkts):
    st, out = _device_run(lib, pkts, [len(p) for p in pkts], "unprotect")
    for i, p in enumerate(pkts):
        rc, ref = orc.unprotect(p, len(p))
        assert st[i] == rc, (i, st[i], rc)
        assert rc or out[i] == ref, i
    return st


@pytest.mark.parametrize("name", ["icm128_hmac80", "icm256_hmac32",
                                  "icm128_nullauth", "gcm256_16", "gcm256_8"])
def test_fused_unprotect_clean_forged_and_declined(name):
    """clean batches, reordered inside the window, with forgeries (auth_fail,
    undone in place), then a duplicate (-> host), an unknown SSRC (-> host),
    a stream past its window (-> sorted form): statuses, bytes and the
    stream state against the oracle's srtp_unprotect per packet"""
    _gpu()
    rng = random.Random(614)
    ssrcs = [0x23000000 + 7 * k for k in range(40)]
    pols = [policy(name, ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    lib, orc, snd = L.Session(pols), O.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(1, 0xff00) for s in ssrcs}
    batches = _send_batches(snd, ssrcs, seq0, 20, 3, rng)
    forge = name != "icm128_nullauth"
    d0, h0 = lib.prepass_stats()
    for b, sent in enumerate(batches):
        rx = list(sent)
        rng.shuffle(rx)     # every stream's 20 packets span < 64 indices
        if forge and b == 1:
            for k in rng.sample(range(len(rx)), 25):
                x = bytearray(rx[k])
                x[-1] ^= 0x20
                rx[k] = bytes(x)
        st = _receive_check(lib, orc, rx)
        if forge and b == 1:
            assert st.count(7) == 25
    d, h = lib.prepass_stats()
    assert (d - d0, h - h0) == (3, 0), lib.prepass_last_abort()
    # declined batches: duplicate -> host, unknown SSRC -> host
    sent = _send_batches(snd, ssrcs, seq0, 10, 1, rng)[0]
    dup = sent[:50] + [sent[20]] + sent[50:]
    _receive_check(lib, orc, dup)
    unk_pol = policy(name, ssrc=0x0bad0bad, seed=99)
    unk = O.Session([unk_pol]).protect(rtp_packet(rng, 0x0bad0bad, 5, 20), 64)[1]
    sent = _send_batches(snd, ssrcs, seq0, 10, 1, rng)[0]
    _receive_check(lib, orc, sent[:30] + [unk] + sent[30:])
    d2, h2 = lib.prepass_stats()
    assert h2 - h == 2, (d2 - d, h2 - h)
    # long chains: the sorted chain form takes the batch after the restore
    sent = _send_batches(snd, ssrcs[:4], seq0, 150, 1, rng)[0]
    _receive_check(lib, orc, sent)
    assert lib.prepass_stats()[1] == h2
    for s in ssrcs[::3]:
        assert lib.get_roc(s)[1] == orc.get_roc(s)[1]


def test_fused_unprotect_windows_and_state():
    """window sizes 64 / 96 / 160 / 1024, streams jumping past their window
    between batches; afterwards old, replayed and skipped indices probed
    one by one through the host path against the oracle"""
    _gpu()
    rng = random.Random(615)
    wins = [64, 96, 160, 1024]
    ssrcs = [0x24000000 + 5 * k for k in range(32)]
    pols = [policy("icm128_hmac80", ssrc=s, seed=k, window=wins[k % 4])
            for k, s in enumerate(ssrcs)]
    lib, orc = L.Session(pols), O.Session(pols)
    snd = O.Session(pols)
    seq0 = {s: rng.randrange(100, 0xf000) for s in ssrcs}
    kept = {s: [] for s in ssrcs}
    for b in range(3):
        if b == 1:
            for s in ssrcs[::3]:
                seq0[s] += rng.randrange(70, 3000)
        pk = _interleaved(rng, ssrcs, seq0, 16, shuffle_within=0.3,
                          payloads=(0, 5, 160))
        rx = []
        for p in pk:
            rc, ref = snd.protect(p, len(p) + 32)
            assert rc == 0
            rx.append(ref)
            kept[int.from_bytes(p[8:12], "big")].append(ref)
        _receive_check(lib, orc, rx)
        assert lib.prepass_last_abort() == 0, (b, lib.prepass_last_abort())
    assert lib.prepass_stats() == (3, 0)
    for k, s in enumerate(ssrcs):
        assert lib.get_roc(s)[1] == orc.get_roc(s)[1]
        for p in rng.sample(kept[s], 4):   # replays: host path, one by one
            st, out = lib.unprotect(p, len(p))
            rc, ref = orc.unprotect(p, len(p))
            assert st == rc, (k, st, rc)


@pytest.mark.parametrize("step", ["max", "mixed"])
def test_one_stream_chain_over_many_tiles_with_large_advances(step):
    """one stream, 300,000 packets (73 look-back tiles of 4096) whose
    sequence numbers advance by up to 2^15 - 1 each: the index sum crosses
    2^32 inside the batch (the look-back's advance sum must not
    wrap).  Protect on the device chain form and unprotect on the device
    receive chain, every packet against the C oracle."""
    _gpu()
    import numpy as np
    import torch
    n, slot = 300000, 48
    rng = np.random.default_rng(77 if step == "max" else 78)
    if step == "max":
        adv = np.full(n, 32767, dtype=np.int64)
    else:
        adv = np.where(rng.random(n) < 0.5, 32767, rng.integers(1, 32768, n))
    adv[0] = 0
    idx = 5 + np.cumsum(adv)
    assert idx[-1] > 1 << 32
    pol = policy("icm128_hmac80", ssrc=0x31415926, seed=9)
    a = rng.integers(0, 256, (n, slot), dtype=np.uint8)
    plen = rng.integers(0, 17, n)
    seq = idx & 0xffff
    a[:, 0], a[:, 1] = 0x80, 96
    a[:, 2], a[:, 3] = seq >> 8, seq & 0xff
    a[:, 8:12] = np.frombuffer((0x31415926).to_bytes(4, "big"), dtype=np.uint8)
    ln = (12 + plen).astype(np.uint32)
    orc = O.Session([pol])
    bad, ref, rlen = orc.protect_many(a.reshape(-1),
                                      np.arange(n, dtype=np.uint64) * slot,
                                      ln, slot)
    assert bad == 0
    lib = L.Session([pol])
    d = torch.from_numpy(a.copy()).cuda().view(-1)
    off = (torch.arange(n, dtype=torch.int64) * slot).cuda()
    tl = torch.from_numpy(ln.astype(np.int32)).cuda()
    cap = torch.full((n,), slot, dtype=torch.int32).cuda()
    st = torch.full((n,), -1, dtype=torch.int32).cuda()
    assert lib.protect_device(d, off, tl, d, off, cap, st) == 0
    assert lib.prepass_stats() == (1, 0), lib.prepass_last_abort()
    assert int((st != 0).sum()) == 0
    got = d.cpu().numpy().reshape(n, slot)
    cap = cap.cpu().numpy()
    assert (cap == rlen).all()
    used = np.arange(slot)[None, :] < rlen[:, None]   # each packet's bytes
    diff = np.nonzero(((got != ref) & used).any(axis=1))[0]
    assert len(diff) == 0, diff[:8]
    assert lib.get_roc(0x31415926)[1] == orc.get_roc(0x31415926)[1]
    # the receiver, same batch, device chain
    rcv = L.Session([pol])
    cap2 = torch.full((n,), slot, dtype=torch.int32).cuda()
    st2 = torch.full((n,), -1, dtype=torch.int32).cuda()
    srl = torch.from_numpy(rlen.astype(np.int32)).cuda()
    assert rcv.unprotect_device(d, off, srl, d, off, cap2, st2) == 0
    assert rcv.prepass_stats() == (1, 0), rcv.prepass_last_abort()
    assert int((st2 != 0).sum()) == 0
    back = d.cpu().numpy().reshape(n, slot)
    used = np.arange(slot)[None, :] < ln[:, None].astype(np.int64)
    assert not ((back != a) & used).any()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fused_paths_random_traffic(seed):
    """randomised batches through the device pre-passes (order-free forms in
    the AES-ICM kernel, sorted chain form, host fallbacks), protect and
    unprotect, in place: streams with windows 64..1024, payloads 0..300 B,
    reordering inside and beyond the window, duplicates, unknown SSRCs,
    forged packets, jumps.  Every status and byte of both sides against the
    oracle, and the stream state at the end."""
    _gpu()
    rng = random.Random(700 + seed)
    ns = rng.choice([3, 17, 64])
    ssrcs = [0x25000000 + 11 * k + seed for k in range(ns)]
    pols = [policy(rng.choice(["icm128_hmac80", "icm128_hmac80",
                               "icm256_hmac32"]) if seed == 3 else
                   "icm128_hmac80", ssrc=s, seed=k,
                   window=rng.choice([64, 128, 128, 256, 1024]))
            for k, s in enumerate(ssrcs)]
    slib, sorc = L.Session(pols), O.Session(pols)
    rlib, rorc = L.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(1, 0xffff) for s in ssrcs}
    for b in range(8):
        per = rng.choice([1, 5, 20, 40])
        pk = _interleaved(rng, ssrcs, seq0, per,
                          shuffle_within=rng.choice([0, 0.1, 0.5]),
                          payloads=(0, 1, 13, 160, 300))
        event = rng.choice(["none", "none", "dup", "unknown", "jump"])
        if event == "dup" and len(pk) > 10:
            pk.insert(rng.randrange(5, len(pk)), pk[rng.randrange(0, 5)])
        elif event == "unknown":
            pk.insert(rng.randrange(0, len(pk)),
                      rtp_packet(rng, 0x0badf00d, 7, 30))
        elif event == "jump":
            s = rng.choice(ssrcs)
            seq0[s] += rng.randrange(100, 20000)
        caps = [len(p) + rng.choice([10, 16, 40]) for p in pk]
        st, out = _device_run(slib, pk, caps, "protect")
        sent = []
        for i, p in enumerate(pk):
            rc, ref = sorc.protect(p, caps[i])
            assert st[i] == rc, (b, event, i, st[i], rc)
            assert rc or out[i] == ref, (b, event, i)
            if rc == 0:
                sent.append(ref)
        # the receiver: the sent packets shuffled, some forged / repeated
        rx = list(sent)
        if rng.random() < 0.5:
            rng.shuffle(rx)
        for k in rng.sample(range(len(rx)), min(len(rx), rng.choice([0, 3]))):
            x = bytearray(rx[k])
            x[-1] ^= 0x11
            rx[k] = bytes(x)
        if rx and rng.random() < 0.3:
            rx.append(rx[rng.randrange(len(rx))])
        if not rx:
            continue
        st, out = _device_run(rlib, rx, [len(p) for p in rx], "unprotect")
        for i, p in enumerate(rx):
            rc, ref = rorc.unprotect(p, len(p))
            assert st[i] == rc, ("rx", b, i, st[i], rc)
            assert rc or out[i] == ref, ("rx", b, i)
    for s in ssrcs:
        assert slib.get_roc(s)[1] == sorc.get_roc(s)[1]
        assert rlib.get_roc(s)[1] == rorc.get_roc(s)[1]


def test_fused_paths_ineligible_stream_of_another_variant():
    """a stream the device pre-pass cannot take (pending ROC after
    srtp_stream_set_roc) whose cipher is not the batch's AES-ICM kernel
    variant (AES-GCM): its packets must not be counted as processed by the
    fused kernel, so the declined batch's undo leaves them alone and the
    host path produces the reference's bytes (protect and unprotect)"""
    _gpu()
    rng = random.Random(616)
    ssrcs = [0x26000000 + 3 * k for k in range(24)]
    g_ssrc = 0x26ffff01
    pols = [policy("icm128_hmac80", ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    pols.append(policy("gcm256_16", ssrc=g_ssrc, seed=77))
    for op in ("protect", "unprotect"):
        lib, orc = L.Session(pols), O.Session(pols)
        snd = O.Session(pols)
        seq0 = {s: rng.randrange(1, 0xf000) for s in ssrcs + [g_ssrc]}
        # a clean batch first (device), then set_roc on the GCM stream
        for b in range(2):
            pk = _interleaved(rng, ssrcs + [g_ssrc], seq0, 6,
                              payloads=(0, 20, 160))
            if b == 1:
                assert lib.set_roc(g_ssrc, 3) == 0
                assert orc.set_roc(g_ssrc, 3) == 0
            if op == "protect":
                caps = [len(p) + 32 for p in pk]
                st, out = _device_run(lib, pk, caps, "protect")
                for i, p in enumerate(pk):
                    rc, ref = orc.protect(p, caps[i])
                    assert st[i] == rc, (b, i, st[i], rc)
                    assert rc or out[i] == ref, (b, i)
            else:
                if b == 1:
                    assert snd.set_roc(g_ssrc, 3) == 0
                rx = [snd.protect(p, len(p) + 32)[1] for p in pk]
                _receive_check(lib, orc, rx)
        d, h = lib.prepass_stats()
        # the pending ROC is resolved on the device (srtp_host.c
        # pend_resolve): the set_roc batch stays there too
        assert (d, h) == (2, 0), (op, d, h, lib.prepass_last_abort())


def _pending_run(lib, orc, snd, op, pk, caps=None):
    """one device batch in place against the oracle (protect: caps; receive:
    the sender session `snd` protects pk first) -> statuses"""
    if op == "protect":
        caps = caps or [len(p) + 32 for p in pk]
        st, out = _device_run(lib, pk, caps, "protect")
        for i, p in enumerate(pk):
            rc, ref = orc.protect(p, caps[i])
            assert st[i] == rc, (i, st[i], rc)
            assert rc or out[i] == ref, i
        return st
    rx = [snd.protect(p, len(p) + 32)[1] for p in pk]
    return _receive_check(lib, orc, rx)


@pytest.mark.parametrize("op", ["protect", "unprotect"])
@pytest.mark.parametrize("shape", ["fused_many", "one_stream", "gcm_many"])
def test_pending_roc_on_device(op, shape):
    """srtp_stream_set_roc on running streams (srtp.c:5137-5167; the
    estimate 2038-2081): a set ROC ahead of the stream's (its first packet
    then resets index and window, 2674-2678 / 3161-3167) and a set ROC equal
    to the current one (it stays pending: every estimate is pending_roc ||
    seq), on the device pre-pass -- the AES-ICM kernel's fused order-free
    form among 600 streams, the one-stream chain form, and the separate
    order-free form (AES-GCM) -- bit-exact against the oracle's per-packet
    srtp_protect / srtp_unprotect, no batch on the host path; a ROC set
    below the stream's (the first packet 2^15 behind: pkt_idx_old) goes to
    the host path, whose result the next device batch continues from"""
    _gpu()
    rng = random.Random(700 + len(shape) + len(op))
    name = "gcm256_16" if shape == "gcm_many" else "icm128_hmac80"
    ns = 1 if shape == "one_stream" else 600
    ssrcs = [0x28000000 + 5 * k for k in range(ns)]
    pols = [policy(name, ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    lib, orc, snd = L.Session(pols), O.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(0x9000, 0xf000) for s in ssrcs}
    per = 200 if ns == 1 else 6
    ahead, same = ssrcs[0], ssrcs[-1]
    for b in range(4):
        pk = _interleaved(rng, ssrcs, seq0, per, payloads=(0, 20, 160))
        if b == 1:
            # ahead: ROC 5 set on a stream at ROC 0: its first packet resets
            for sess in (lib, orc, snd):
                assert sess.set_roc(ahead, 5) == 0
        if b == 0 and ns > 1:
            # a fresh stream (index 0) given ROC 3 before its first packet
            for sess in (lib, orc, snd):
                assert sess.set_roc(same, 3) == 0
        if b == 2 and ns > 1:
            # the same ROC again, while its packets stay within 2^15: it
            # stays pending for the whole batch
            for sess in (lib, orc, snd):
                assert sess.set_roc(same, orc.get_roc(same)[1]) == 0
        _pending_run(lib, orc, snd, op, pk)
    d, h = lib.prepass_stats()
    assert (d, h) == (4, 0), (d, h, lib.prepass_last_abort())
    for s in (ahead, same):
        assert lib.get_roc(s) == orc.get_roc(s), hex(s)
    # a ROC below the stream's (the receiver's or the sender's own):
    # pkt_idx_old from the host path (the sender keeps ROC 5)
    for sess in (lib, orc):
        assert sess.set_roc(ahead, 2) == 0
    pk = _interleaved(rng, ssrcs, seq0, per, payloads=(0, 20))
    st = _pending_run(lib, orc, snd, op, pk)
    assert lib.prepass_stats()[1] == 1
    pk = _interleaved(rng, ssrcs, seq0, per, payloads=(0, 20))
    _pending_run(lib, orc, snd, op, pk)
    assert lib.get_roc(ahead) == orc.get_roc(ahead)


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
@pytest.mark.parametrize("ns", [1, 50])
def test_mki_mixed_keys_with_pending_roc(name, ns):
    """MKI streams with per-packet keys (k_mki_keys) meeting a pending ROC
    (k_pend_apply) in the same batch -- the one-stream chain form and the
    order-free form: every status and byte, every key's remaining uses and
    the ROCs against the oracle, no batch on the host path"""
    _gpu()
    rng = random.Random(720 + ns)
    ssrcs = [0x28800000 + 9 * k for k in range(ns)]
    pols = [policy(name, ssrc=s, seed=k, mki=4, nkeys=3)
            for k, s in enumerate(ssrcs)]
    lib, orc = L.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(0x9000, 0xf000) for s in ssrcs}
    per = 300 if ns == 1 else 8
    for b in range(3):
        if b == 1:
            for sess in (lib, orc):
                assert sess.set_roc(ssrcs[0], 4) == 0
        pk = _interleaved(rng, ssrcs, seq0, per, payloads=(0, 20, 160))
        mki = [rng.randrange(3) for _ in pk]
        caps = [len(p) + 32 for p in pk]
        st, out = _device_run(lib, pk, caps, "protect", mki)
        for i, p in enumerate(pk):
            rc, ref = orc.protect(p, caps[i], mki[i])
            assert st[i] == rc, (b, i, st[i], rc)
            assert rc or out[i] == ref, (b, i)
    d, h = lib.prepass_stats()
    assert (d, h) == (3, 0), (d, h, lib.prepass_last_abort())
    _key_left_equal(lib, orc, ssrcs[:4], 3)
    assert lib.get_roc(ssrcs[0]) == orc.get_roc(ssrcs[0])


@pytest.mark.parametrize("shape", ["fused_many", "one_stream"])
def test_pending_roc_forged_first_packet(shape):
    """receive side: the first packet of a stream with a pending ROC does not
    authenticate -- the reference keeps the ROC pending (the reset happens
    only after the tag, srtp.c:3157-3167), so the device batch is declined
    (AB_PENDING) and the host path decides: statuses and bytes equal to the
    oracle's"""
    _gpu()
    rng = random.Random(720 + len(shape))
    ns = 1 if shape == "one_stream" else 300
    ssrcs = [0x29000000 + 3 * k for k in range(ns)]
    pols = [policy("icm128_hmac80", ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    lib, orc, snd = L.Session(pols), O.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(0x100, 0xf000) for s in ssrcs}
    per = 100 if ns == 1 else 5
    pk = _interleaved(rng, ssrcs, seq0, per, payloads=(0, 40))
    _pending_run(lib, orc, snd, "unprotect", pk)
    tgt = ssrcs[ns // 2]
    for sess in (lib, orc, snd):
        assert sess.set_roc(tgt, 9) == 0
    pk = _interleaved(rng, ssrcs, seq0, per, payloads=(0, 40))
    rx = [snd.protect(p, len(p) + 32)[1] for p in pk]
    first = next(i for i, p in enumerate(pk) if p[8:12] == tgt.to_bytes(4, "big"))
    bad = bytearray(rx[first])
    bad[-1] ^= 0x5a
    rx[first] = bytes(bad)
    d0, h0 = lib.prepass_stats()
    st = _receive_check(lib, orc, rx)
    assert st[first] == 7
    assert lib.prepass_stats()[1] == h0 + 1, lib.prepass_last_abort()
    assert lib.get_roc(tgt) == orc.get_roc(tgt)


@pytest.mark.parametrize("declined", [False, True], ids=["clean", "declined"])
def test_large_host_batch_pipelined_chunks(declined):
    """srtp_protect_batch / srtp_unprotect_batch over 2^18 host packets run
    as 8 consecutive device batches with the copies overlapped
    (srtp_host.c batch_device_pipelined); "declined": a duplicate inside
    the fifth chunk sends that chunk and the rest to the host path.  Every
    status and byte against the oracle, both directions."""
    _gpu()
    rng = random.Random(617 + declined)
    ssrcs = [0x27000000 + k for k in range(4)]
    pols = [policy("icm128_hmac80", ssrc=s, seed=k) for k, s in enumerate(ssrcs)]
    seq0 = {s: rng.randrange(1, 0xff00) for s in ssrcs}
    n = 1 << 18
    pk = []
    for i in range(n):
        s = ssrcs[i % 4]
        pk.append(rtp_packet(rng, s, seq0[s] & 0xffff, rng.randrange(0, 40)))
        seq0[s] += 1
    if declined:
        j = 5 * n // 8 - 100
        pk[j + 40] = pk[j]          # a replay inside chunk 4
    lib, orc = L.Session(pols), O.Session(pols)
    caps = [len(p) + 16 for p in pk]
    st, out = lib.protect_batch(pk, caps)
    sent = []
    for i, p in enumerate(pk):
        rc, ref = orc.protect(p, caps[i])
        assert st[i] == rc, (i, st[i], rc)
        assert rc or out[i] == ref, i
        if rc == 0:
            sent.append(ref)
    # device batches: every chunk, or the four before the declined one
    # (host-buffer batches that fall back are not counted as host batches)
    assert lib.prepass_stats() == ((4 if declined else 8), 0)
    rlib, rorc = L.Session(pols), O.Session(pols)
    st, out = rlib.unprotect_batch(sent)
    for i, p in enumerate(sent):
        rc, ref = rorc.unprotect(p, len(p))
        assert st[i] == rc, ("rx", i, st[i], rc)
        assert rc or out[i] == ref, ("rx", i)
    assert rlib.prepass_stats() == (8, 0)


# --------------------------------------------------------------------------
# one stream in order: the indices computed inside the AES-ICM kernel
# (srtp_prepass.hip pp_protect_inorder, srtp_icm.hip inorder_meta)

def _arena_run(sess, pkts, caps, slot_extra, rng):
    """srtp_protect_device in place over an arena whose bytes around the
    packets are random -> (statuses, the arena before, the arena after,
    offsets)"""
    import torch
    offs, pos = [], 0
    for p, c in zip(pkts, caps):
        offs.append(pos)
        pos += (max(len(p), c) + slot_extra + 15) & ~15
    before = bytearray(rng.randbytes(pos + 16))
    for o, p in zip(offs, pkts):
        before[o:o + len(p)] = p
    arena = torch.frombuffer(bytearray(before), dtype=torch.uint8).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    cap = torch.tensor(caps, dtype=torch.int32).cuda()
    st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    assert sess.protect_device(arena, off, ln, arena, off, cap, st) == 0
    return st.cpu().tolist(), bytes(before), arena.cpu().numpy().tobytes(), offs


def _check_arena(orc, pkts, caps, st, before, after, offs):
    """every status and every arena byte against the oracle's per-packet
    srtp_protect: a protected packet's bytes, the rest untouched"""
    expect = bytearray(before)
    for i, p in enumerate(pkts):
        rc, ref = orc.protect(p, caps[i])
        assert st[i] == rc, (i, st[i], rc)
        if rc == 0:
            expect[offs[i]:offs[i] + len(ref)] = ref
    if bytes(expect) != after:
        bad = next(k for k in range(len(after)) if after[k] != expect[k])
        raise AssertionError("arena byte %d differs" % bad)


@pytest.mark.parametrize("name", ["icm128_hmac80", "icm192_hmac80",
                                  "icm256_hmac32", "icm128_nullauth",
                                  "icm128_authonly", "gcm128_16",
                                  "gcm256_16", "gcm256_8"])
def test_one_stream_in_order_form(name):
    """a sender's batches of consecutive sequence numbers (across a ROC
    wrap, headers with CSRCs and extensions) take the in-order form; a
    duplicate, a gap, a too-small buffer or a replayed packet in the batch
    declines it -- the input comes back exactly and the chain form runs;
    every status and every arena byte (the slot bytes after each packet
    included) against the oracle, then the stream's window through a
    replayed packet"""
    _gpu()
    rng = random.Random(731)
    ssrc = 0x29000000
    pols = [policy(name, ssrc=ssrc, seed=2)]
    lib, orc = L.Session(pols), O.Session(pols)
    seq = 0xffff - 1500

    def batch(n, tweak=None):
        nonlocal seq
        seqs = [(seq + k) & 0xffff for k in range(n)]
        seq += n
        pk = []
        for k, q in enumerate(seqs):
            cc = rng.choice((0, 0, 0, 2))
            xw = rng.choice((-1, -1, 1, 3))
            pk.append(rtp_packet(rng, ssrc, q, rng.choice((0, 7, 160, 1000)),
                                 cc=cc, xwords=xw))
        caps = [len(p) + 32 for p in pk]
        if tweak:
            tweak(pk, caps)
        return pk, caps

    def dup(pk, caps):
        pk[700] = pk[699]

    def gap(pk, caps):
        nonlocal seq
        seq += 1                        # the next batch continues after it
        for k in range(900, len(pk)):   # one advance of 2 from packet 900 on
            p = bytearray(pk[k])
            q = ((p[2] << 8) | p[3]) + 1
            p[2], p[3] = (q >> 8) & 0xff, q & 0xff
            pk[k] = bytes(p)

    def small(pk, caps):
        caps[1234] = len(pk[1234]) + 3

    # a fresh stream's first packet 1500 below the sequence wrap: the
    # reference's first estimate (rdbx.c:112-145 from index 0) is the host
    # path's; the batches after it run on the device
    pk, caps = batch(16)
    st, before, after, offs = _arena_run(lib, pk, caps, 24, rng)
    _check_arena(orc, pk, caps, st, before, after, offs)
    plan = [(3000, None), (2000, dup), (2000, gap), (2000, small), (3000, None)]
    d0, h0 = lib.prepass_stats()
    sent, where = [], []
    for n, tw in plan:
        pk, caps = batch(n, tw)
        hb = lib.prepass_stats()[1]
        st, before, after, offs = _arena_run(lib, pk, caps, 24, rng)
        where.append((lib.prepass_stats()[1] - hb, lib.prepass_last_abort()))
        _check_arena(orc, pk, caps, st, before, after, offs)
        sent.append(pk)
    d, h = lib.prepass_stats()
    # the duplicate sends its batch to the host (the chain form takes
    # advances in [1, 2^15) only); the gap and the small buffer stay on the
    # device through the chain form
    assert (d - d0, h - h0) == (len(plan) - 1, 1), (d - d0, h - h0, where)
    assert lib.get_roc(ssrc) == orc.get_roc(ssrc)
    _key_left_equal(lib, orc, [ssrc], 1)   # key uses (key.c:74-90)
    # the window the batches left: the last packets again (replay_fail /
    # replay_old on the sender's side) next to a new one
    pk = sent[-1][-40:] + sent[0][:3]
    pk.append(rtp_packet(rng, ssrc, seq & 0xffff, 50))
    caps = [len(p) + 32 for p in pk]
    st, before, after, offs = _arena_run(lib, pk, caps, 24, rng)
    _check_arena(orc, pk, caps, st, before, after, offs)


def _arena_run_rx(sess, pkts, caps, slot_extra, rng):
    """srtp_unprotect_device in place over an arena with random bytes
    around the packets"""
    import torch
    offs, pos = [], 0
    for p, c in zip(pkts, caps):
        offs.append(pos)
        pos += (max(len(p), c) + slot_extra + 15) & ~15
    before = bytearray(rng.randbytes(pos + 16))
    for o, p in zip(offs, pkts):
        before[o:o + len(p)] = p
    arena = torch.frombuffer(bytearray(before), dtype=torch.uint8).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    cap = torch.tensor(caps, dtype=torch.int32).cuda()
    st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    assert sess.unprotect_device(arena, off, ln, arena, off, cap, st) == 0
    return st.cpu().tolist(), bytes(before), arena.cpu().numpy().tobytes(), offs


@pytest.mark.parametrize("name", ["icm128_hmac80", "icm192_hmac80",
                                  "icm256_hmac32", "icm128_nullauth",
                                  "icm128_authonly", "gcm128_16",
                                  "gcm256_16", "gcm256_8"])
def test_one_stream_in_order_receive(name):
    """the receive side of the in-order form: runs of consecutive packets
    (across a ROC wrap) with forged tags among them -- rejected, their
    decryption undone, the others accepted at the same indices -- and runs
    with a swapped pair, a repeated packet or a too-short packet (declined,
    restored, the chain form decides), a one-packet run, a run with every
    tag forged (the stream does not move) and one whose last 1,100 tags are
    forged; every status and every arena byte against the oracle's
    srtp_unprotect per packet, the key uses, then the window through
    replayed packets"""
    _gpu()
    rng = random.Random(733)
    ssrc = 0x29100000
    pols = [policy(name, ssrc=ssrc, seed=3)]
    snd = O.Session(pols)
    lib, orc = L.Session(pols), O.Session(pols)
    tag = POLICIES[name][4]
    seq = 0xffff - 2500
    sent_all = []

    def run(n):
        nonlocal seq
        out = []
        for k in range(n):
            p = rtp_packet(rng, ssrc, seq & 0xffff,
                           rng.choice((0, 7, 160, 1000)),
                           cc=rng.choice((0, 0, 2)),
                           xwords=rng.choice((-1, -1, 2)))
            seq += 1
            rc, ref = snd.protect(p, len(p) + 64)
            assert rc == 0
            out.append(ref)
        sent_all.extend(out)
        return out

    def forge(pk):
        if tag == 0:
            return
        for k in rng.sample(range(len(pk)), 25) + [len(pk) - 1]:
            b = bytearray(pk[k])
            b[-1] ^= 0x40
            pk[k] = bytes(b)

    def swap(pk):
        pk[500], pk[501] = pk[501], pk[500]

    def repeat(pk):
        pk[800] = pk[799]

    def short(pk):
        pk[321] = pk[321][:8]

    def forge_all(pk):   # nothing accepted: the stream does not move
        if tag == 0:
            return
        for k in range(len(pk)):
            b = bytearray(pk[k])
            b[-1] ^= 0x01
            pk[k] = bytes(b)

    def forge_tail(pk):  # the last accepted packet 1,100 from the end
        if tag == 0:
            return
        for k in range(len(pk) - 1100, len(pk)):
            b = bytearray(pk[k])
            b[-2] ^= 0x10
            pk[k] = bytes(b)

    warm = run(8)   # the stream's first packets (host path: fresh index)
    st, before, after, offs = _arena_run_rx(lib, warm, [len(p) for p in warm],
                                            24, rng)
    _check_rx_arena(orc, warm, st, before, after, offs)
    plan = [(2000, None), (2000, forge), (2000, swap), (2000, repeat),
            (2000, short), (2000, forge), (2000, None), (1, None),
            (300, forge_all), (2000, forge_tail), (2000, None)]
    for b, (n, tw) in enumerate(plan):
        pk = run(n)
        if tw:
            tw(pk)
        caps = [len(p) for p in pk]
        st, before, after, offs = _arena_run_rx(lib, pk, caps, 24, rng)
        _check_rx_arena(orc, pk, st, before, after, offs,
                        "batch %d %s" % (b, tw.__name__ if tw else "clean"))
    assert lib.get_roc(ssrc) == orc.get_roc(ssrc)
    _key_left_equal(lib, orc, [ssrc], 1)   # key uses (key.c:74-90)
    # the window: recent packets again (replay_fail) and older ones
    # (replay_old), then a new one
    pk = sent_all[-30:] + sent_all[-3000:-2990]
    pk += run(1)
    st, before, after, offs = _arena_run_rx(lib, pk, [len(p) for p in pk], 24,
                                            rng)
    _check_rx_arena(orc, pk, st, before, after, offs)
    _key_left_equal(lib, orc, [ssrc], 1)


def _check_rx_arena(orc, pkts, st, before, after, offs, what=""):
    expect = bytearray(before)
    for i, p in enumerate(pkts):
        rc, ref = orc.unprotect(p, len(p))
        assert st[i] == rc, (what, i, st[i], rc)
        if rc == 0:
            expect[offs[i]:offs[i] + len(ref)] = ref
    if bytes(expect) != after:
        bad = next(k for k in range(len(after)) if after[k] != expect[k])
        i = max(k for k in range(len(offs)) if offs[k] <= bad)
        raise AssertionError("%s: arena byte %d differs: packet %d (len %d, "
                             "status %d) byte %d" % (what, bad, i, len(pkts[i]),
                                                     st[i], bad - offs[i]))


def _rx_stream(name, ssrc, seed):
    pols = [policy(name, ssrc=ssrc, seed=seed)]
    return O.Session(pols), L.Session(pols), O.Session(pols)


def _sender_run(snd, rng, ssrc, seq, n, payloads=(0, 7, 40)):
    out = []
    for k in range(n):
        p = rtp_packet(rng, ssrc, (seq + k) & 0xffff, rng.choice(payloads))
        rc, ref = snd.protect(p, len(p) + 64)
        assert rc == 0
        out.append(ref)
    return out


def _forge(pk, ks, bit=0x10):
    for k in ks:
        b = bytearray(pk[k])
        b[-1] ^= bit
        pk[k] = bytes(b)


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_in_order_receive_long_forged_tail(name):
    """a run whose last 4,500 of 5,000 tags are forged: the last accepted
    packet lies 4,500 from the end (k_io_rx_commit finds it from the block
    records, no LDS flag loop), the in-order form commits it (no decline),
    and every status, arena byte, key use and the window through replays
    equal the oracle's (srtp.c:3157-3167: replay add after the tag;
    rdbx.c:253-270)"""
    _gpu()
    rng = random.Random(741)
    ssrc = 0x29200000
    snd, lib, orc = _rx_stream(name, ssrc, 4)
    seq = 0xffff - 700          # across a ROC wrap
    warm = _sender_run(snd, rng, ssrc, seq, 4)
    seq += 4
    st, before, after, offs = _arena_run_rx(lib, warm, [len(p) for p in warm],
                                            24, rng)
    _check_rx_arena(orc, warm, st, before, after, offs, "warm")
    sent = []
    for b, forged in enumerate([range(500, 5000), range(0, 4990),
                                range(100, 5000)]):
        pk = _sender_run(snd, rng, ssrc, seq, 5000)
        seq += 5000
        _forge(pk, forged)
        r0, d0 = lib.inorder_stats()
        st, before, after, offs = _arena_run_rx(lib, pk, [len(p) for p in pk],
                                                24, rng)
        _check_rx_arena(orc, pk, st, before, after, offs, "batch %d" % b)
        assert lib.inorder_stats() == (r0 + 1, d0), ("in-order form", b)
        sent += pk
    assert lib.get_roc(ssrc) == orc.get_roc(ssrc)
    _key_left_equal(lib, orc, [ssrc], 1)
    # the window: accepted and forged packets again, then a new one
    pk = sent[-5000 + 95:-5000 + 130] + sent[-20:]
    pk += _sender_run(snd, rng, ssrc, seq, 1)
    st, before, after, offs = _arena_run_rx(lib, pk, [len(p) for p in pk], 24,
                                            rng)
    _check_rx_arena(orc, pk, st, before, after, offs, "window")


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
@pytest.mark.parametrize("case", ["long_reject", "gap_then_reject",
                                  "just_below"])
def test_in_order_receive_reject_run_past_2_15(name, case):
    """rejected runs that carry a packet 2^15 or more past the last accepted
    index (or the stored one): the reference's estimate from that top
    (rdbx.c:112-145) is then another ROC -- replay_old, or a decryption at
    another index -- so the in-order form must decline the batch (AB_GAP)
    and the chain form / host decide; a run just below 2^15 stays in the
    in-order form.  Every status and arena byte against the oracle"""
    _gpu()
    rng = random.Random(743)
    ssrc = 0x29300000
    snd, lib, orc = _rx_stream(name, ssrc, 5)
    # a stored index above 2^15 (below it index_guess keeps ROC 0 and the
    # estimates would not diverge inside one ROC)
    seq = 40000
    warm = _sender_run(snd, rng, ssrc, seq, 4)
    seq += 4
    st, before, after, offs = _arena_run_rx(lib, warm, [len(p) for p in warm],
                                            24, rng)
    _check_rx_arena(orc, warm, st, before, after, offs, "warm")
    if case == "long_reject":          # 33,000 forged, then authentic ones
        n, skip, forged, declined = 34000, 0, range(0, 33000), True
    elif case == "gap_then_reject":    # 20,000 skipped, then 13,000 forged
        n, skip, forged, declined = 14000, 20000, range(0, 13000), True
    else:                              # a reject run of 32,000: in the form
        n, skip, forged, declined = 33000, 0, range(500, 32500), False
    seq += skip
    pk = _sender_run(snd, rng, ssrc, seq, n, payloads=(0, 12))
    seq += n
    _forge(pk, forged)
    r0, d0 = lib.inorder_stats()
    st, before, after, offs = _arena_run_rx(lib, pk, [len(p) for p in pk], 24,
                                            rng)
    _check_rx_arena(orc, pk, st, before, after, offs, case)
    assert lib.inorder_stats() == ((r0, d0 + 1) if declined else (r0 + 1, d0))
    assert lib.get_roc(ssrc) == orc.get_roc(ssrc)
    _key_left_equal(lib, orc, [ssrc], 1)
    pk = _sender_run(snd, rng, ssrc, seq, 50)
    st, before, after, offs = _arena_run_rx(lib, pk, [len(p) for p in pk], 24,
                                            rng)
    _check_rx_arena(orc, pk, st, before, after, offs, "after")


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_mki_mixed_keys_with_key_buckets(name):
    """key buckets on (srtp_mi355x_set_key_buckets(1)): a many-stream MKI
    protect batch whose packets pick different master keys must not take
    the bucketed kernel, which runs one key per 64-record group -- every
    packet on the key its mki_index selects (srtp.c:2536-2545), every byte,
    status and per-key use against the oracle"""
    _gpu()
    rng = random.Random(751)
    ssrcs = [0x22600000 + 5 * k for k in range(12)]
    pols = [policy(name, ssrc=s, seed=40 + k, mki=4, nkeys=3)
            for k, s in enumerate(ssrcs)]
    lib, orc = L.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(1, 0xff00) for s in ssrcs}
    L.lib().srtp_mi355x_set_key_buckets(1)
    try:
        d0, h0 = lib.prepass_stats()
        for b in range(2):
            pk = _interleaved(rng, ssrcs, seq0, 96, payloads=(0, 20, 172))
            mki = [rng.randrange(3) for _ in pk]
            caps = [len(p) + 32 for p in pk]
            st, out = _device_run(lib, pk, caps, "protect", mki)
            for i, p in enumerate(pk):
                rc, ref = orc.protect(p, caps[i], mki[i])
                assert st[i] == rc, (b, i, st[i], rc)
                assert rc or out[i] == ref, (b, i, mki[i])
        assert lib.prepass_stats() == (d0 + 2, h0)
        _key_left_equal(lib, orc, ssrcs, 3)
    finally:
        L.lib().srtp_mi355x_set_key_buckets(-1)


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_mki_pending_roc_stream_with_fewer_keys_than_rx_hint(name):
    """a session receiving on an MKI stream with 3 keys (the host path
    matched key 2 last, so receive batches use master key 2) and sending on
    an MKI stream with ONE key whose ROC the application set: the sender is
    receive-ineligible (fewer keys than 2) but protect-eligible, and its
    packets must still be estimated as pending_roc || seq (srtp.c:2069-2076)
    -- every byte, status and the ROC afterwards against the oracle"""
    _gpu()
    rng = random.Random(753)
    ra, sb = 0x22700000, 0x22700001
    pols = [policy(name, ssrc=ra, seed=61, mki=4, nkeys=3),
            policy(name, ssrc=sb, seed=62, mki=4, nkeys=1)]
    peer = O.Session(pols)
    lib, orc = L.Session(pols), O.Session(pols)
    seq = 300
    for b in range(3):   # key 2 on the receive stream: host, then device
        pk = []
        for k in range(40):
            p = rtp_packet(rng, ra, seq, 40)
            seq += 1
            rc, ref = peer.protect(p, len(p) + 64, 2)
            assert rc == 0
            pk.append(ref)
        st, out = _device_run(lib, pk, [len(p) for p in pk], "unprotect")
        for i, p in enumerate(pk):
            rc, ref = orc.unprotect(p, len(p))
            assert st[i] == rc == 0 and out[i] == ref, (b, i)
    assert lib.set_roc(sb, 7) == 0 and orc.set_roc(sb, 7) == 0
    d0, h0 = lib.prepass_stats()
    for b, s0 in enumerate((0x1000, 0x1000 + 64)):
        pk = [rtp_packet(rng, sb, s0 + k, rng.choice((0, 30, 160)))
              for k in range(64)]
        caps = [len(p) + 32 for p in pk]
        st, out = _device_run(lib, pk, caps, "protect", [0] * len(pk))
        for i, p in enumerate(pk):
            rc, ref = orc.protect(p, caps[i], 0)
            assert st[i] == rc == 0, (b, i, st[i], rc)
            assert out[i] == ref, (b, i)
    d, h = lib.prepass_stats()
    assert d - d0 >= 1, (d - d0, h - h0)
    assert lib.get_roc(sb)[1] == orc.get_roc(sb)[1] == 7


def _set_mki(pkt, name, mki_size, val):
    """the packet with its MKI bytes replaced (ICM: MKI || tag at the end;
    AES-GCM: the MKI alone at the end)"""
    tag = POLICIES[name][4]
    back = mki_size + (0 if name.startswith("gcm") else tag)
    b = bytearray(pkt)
    b[len(b) - back:len(b) - back + mki_size] = val
    return bytes(b)


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
@pytest.mark.parametrize("shape", ["one_stream", "many_streams"])
def test_mki_receive_bursts_of_several_keys_on_device(name, shape):
    """a receiver during a rekey overlap (srtp.c:1961-2016, called at 2908):
    bursts whose packets alternate between two master keys' MKIs, with
    packets carrying an MKI no key has (bad_mki 25 -- after the replay
    check, so a replayed one says replay_fail), forged tags under either
    key, and (one stream: the chain form's verdicts) replays; every batch
    on the device (host count 0), every
    status and byte equal to the oracle's srtp_unprotect per packet, and
    every master key's remaining uses equal (key.c:74-90: AES-ICM charges
    the accepted packets, AES-GCM every packet past the replay check,
    bad_mki none)"""
    _gpu()
    rng = random.Random(761)
    mki = 4
    ssrcs = [0x22800000] if shape == "one_stream" else \
        [0x22810000 + 7 * k for k in range(40)]
    pols = [policy(name, ssrc=s, seed=70 + k, mki=mki, nkeys=3)
            for k, s in enumerate(ssrcs)]
    snd = O.Session(pols)
    lib, orc = L.Session(pols), O.Session(pols)
    seq0 = {s: rng.randrange(1, 0xff00) for s in ssrcs}
    per = 600 if shape == "one_stream" else 24
    sent = []
    for b in range(4):
        pk = _interleaved(rng, ssrcs, seq0, per, payloads=(0, 20, 172))
        out = []
        for k, p in enumerate(pk):
            j = (k + b) % 2 if b < 3 else 2     # keys 0/1 alternate, then 2
            rc, ref = snd.protect(p, len(p) + 64, j)
            assert rc == 0
            out.append(ref)
        for k in rng.sample(range(len(out)), 9):        # unknown MKI
            out[k] = _set_mki(out[k], name, mki, b"\xee" * mki)
        for k in rng.sample(range(len(out)), 5):        # forged tag
            x = bytearray(out[k])
            x[-1 if name.startswith("icm") else -mki - 1] ^= 0x20
            out[k] = bytes(x)
        if sent and shape == "one_stream":   # replays (k_pu_verdict1), one bad
            old = rng.sample(sent[-1], 4)
            old[0] = _set_mki(old[0], name, mki, b"\xee" * mki)
            out[len(out) // 2:len(out) // 2] = old
        d0, h0 = lib.prepass_stats()
        st, res = _device_run(lib, out, [len(p) for p in out], "unprotect")
        codes = set()
        for i, p in enumerate(out):
            rc, ref = orc.unprotect(p, len(p))
            codes.add(rc)
            assert st[i] == rc, (b, i, st[i], rc)
            assert rc or res[i] == ref, (b, i)
        assert lib.prepass_stats() == (d0 + 1, h0), b
        assert {0, 7, 25} <= codes, codes
        _key_left_equal(lib, orc, ssrcs[:6], 3)
        sent.append(out)
    for s in ssrcs[:6]:
        assert lib.get_roc(s)[1] == orc.get_roc(s)[1]


def _arena_run_oop(sess, pkts, caps, slot_extra, rng, op="protect"):
    """srtp_{un}protect_device out of place: input and output arenas with
    random bytes around the packets -> (statuses, input before, input after,
    output before, output after, offsets)"""
    import torch
    offs, pos = [], 0
    for p, c in zip(pkts, caps):
        offs.append(pos)
        pos += (max(len(p), c) + slot_extra + 15) & ~15
    bin_ = bytearray(rng.randbytes(pos + 16))
    for o, p in zip(offs, pkts):
        bin_[o:o + len(p)] = p
    bout = rng.randbytes(pos + 16)
    ain = torch.frombuffer(bytearray(bin_), dtype=torch.uint8).cuda()
    aout = torch.frombuffer(bytearray(bout), dtype=torch.uint8).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    cap = torch.tensor(caps, dtype=torch.int32).cuda()
    st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    fn = sess.protect_device if op == "protect" else sess.unprotect_device
    assert fn(ain, off, ln, aout, off, cap, st) == 0
    return (st.cpu().tolist(), bytes(bin_), ain.cpu().numpy().tobytes(), bout,
            aout.cpu().numpy().tobytes(), offs)


def _arena_run_async(sess, pkts, caps, slot_extra, rng):
    """srtp_protect_device_async in place, then the stream drained"""
    import torch
    offs, pos = [], 0
    for p, c in zip(pkts, caps):
        offs.append(pos)
        pos += (max(len(p), c) + slot_extra + 15) & ~15
    before = bytearray(rng.randbytes(pos + 16))
    for o, p in zip(offs, pkts):
        before[o:o + len(p)] = p
    arena = torch.frombuffer(bytearray(before), dtype=torch.uint8).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
    cap = torch.tensor(caps, dtype=torch.int32).cuda()
    st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
    torch.cuda.synchronize()
    b = sess.prepare_device(arena, off, ln, arena, off, cap, st)
    assert sess.protect_prepared_async(b) == 0
    torch.cuda.synchronize()
    return st.cpu().tolist(), bytes(before), arena.cpu().numpy().tobytes(), offs


@pytest.mark.parametrize("name", ["icm128_hmac80", "icm256_hmac32",
                                  "gcm256_16"])
@pytest.mark.parametrize("mode", ["out_of_place", "async"])
def test_one_stream_in_order_form_out_of_place_and_async(name, mode):
    """the in-order form for the reference's other callers: out of place
    (test/srtp_driver.c:262-264's not-in-place wrapper) and asynchronous
    (srtp_protect_device_async) -- k_io_check verifies the batch before the
    crypto kernel, so a declined batch (a duplicate, a gap, a too-small
    buffer) has written nothing and the chain form runs it.  Every status,
    every output byte (out of place: the output arena's bytes around and
    after the packets untouched, the input arena unchanged) against the
    oracle; clean batches commit in the in-order form, the others decline"""
    _gpu()
    rng = random.Random(771)
    ssrc = 0x29400000
    pols = [policy(name, ssrc=ssrc, seed=6)]
    lib, orc = L.Session(pols), O.Session(pols)
    seq = 0xffff - 1200

    def batch(n, tweak=None):
        nonlocal seq
        seqs = [(seq + k) & 0xffff for k in range(n)]
        seq += n
        pk = [rtp_packet(rng, ssrc, q, rng.choice((0, 7, 160, 1000)),
                         cc=rng.choice((0, 0, 2)), xwords=rng.choice((-1, 1)))
              for q in seqs]
        caps = [len(p) + 32 for p in pk]
        if tweak:
            tweak(pk, caps)
        return pk, caps

    def dup(pk, caps):
        pk[700] = pk[699]

    def gap(pk, caps):
        nonlocal seq
        seq += 1
        for k in range(900, len(pk)):
            p = bytearray(pk[k])
            q = ((p[2] << 8) | p[3]) + 1
            p[2], p[3] = (q >> 8) & 0xff, q & 0xff
            pk[k] = bytes(p)

    def small(pk, caps):
        caps[1234] = len(pk[1234]) + 3

    def run(pk, caps):
        if mode == "async":
            st, before, after, offs = _arena_run_async(lib, pk, caps, 24, rng)
            _check_arena(orc, pk, caps, st, before, after, offs)
            return
        st, bin_, ain, bout, aout, offs = _arena_run_oop(lib, pk, caps, 24, rng)
        assert ain == bin_, "input arena changed"
        expect = bytearray(bout)
        for i, p in enumerate(pk):
            rc, ref = orc.protect(p, caps[i])
            assert st[i] == rc, (i, st[i], rc)
            if rc == 0:
                expect[offs[i]:offs[i] + len(ref)] = ref
        if bytes(expect) != aout:
            bad = next(k for k in range(len(aout)) if aout[k] != expect[k])
            i = max(k for k in range(len(offs)) if offs[k] <= bad)
            raise AssertionError("output byte %d differs: packet %d status %d"
                                 % (bad, i, st[i]))

    run(*batch(16))   # the fresh stream's first packets
    r0, d0 = lib.inorder_stats()
    for n, tw in [(3000, None), (2000, dup), (2000, gap), (2000, small),
                  (3000, None)]:
        run(*batch(n, tw))
    assert lib.inorder_stats() == (r0 + 2, d0 + 3)
    assert lib.get_roc(ssrc) == orc.get_roc(ssrc)
    _key_left_equal(lib, orc, [ssrc], 1)


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_async_in_order_batches_back_to_back(name):
    """srtp_protect_device_async batches submitted one after another with no
    synchronize between them (a pipelined sender): a long clean batch, one
    the in-order check declines (a duplicate: the chain form runs it), then
    clean ones again -- each call's verdict is its own batch's, never a
    verdict an earlier batch's kernels publish after the call began.  Every
    status and byte against the oracle run in submission order"""
    _gpu()
    import torch
    rng = random.Random(779)
    ssrc = 0x29600000
    pols = [policy(name, ssrc=ssrc, seed=8)]
    lib, orc = L.Session(pols), O.Session(pols)
    seq = 0xffff - 30000
    plan = [(16, None), (24000, None), (2000, "dup"), (3000, None),
            (2000, "dup"), (20000, None), (1000, None)]
    subs = []
    for n, tw in plan:
        pk = [rtp_packet(rng, ssrc, (seq + k) & 0xffff,
                         rng.choice((160, 1000, 1400)) if n > 5000 else
                         rng.choice((0, 7, 160)))
              for k in range(n)]
        seq += n
        if tw == "dup":
            pk[n // 3] = pk[n // 3 - 1]
        caps = [len(p) + 32 for p in pk]
        offs, pos = [], 0
        for p, c in zip(pk, caps):
            offs.append(pos)
            pos += (max(len(p), c) + 24 + 15) & ~15
        before = bytearray(rng.randbytes(pos + 16))
        for o, p in zip(offs, pk):
            before[o:o + len(p)] = p
        arena = torch.frombuffer(bytearray(before), dtype=torch.uint8).cuda()
        t = dict(pk=pk, caps=caps, offs=offs, before=bytes(before),
                 arena=arena,
                 off=torch.tensor(offs, dtype=torch.int64).cuda(),
                 ln=torch.tensor([len(p) for p in pk],
                                 dtype=torch.int32).cuda(),
                 cap=torch.tensor(caps, dtype=torch.int32).cuda(),
                 st=torch.full((n,), -1, dtype=torch.int32).cuda())
        t["b"] = lib.prepare_device(t["arena"], t["off"], t["ln"],
                                    t["arena"], t["off"], t["cap"], t["st"])
        subs.append(t)
    torch.cuda.synchronize()
    assert lib.protect_prepared_async(subs[0]["b"]) == 0   # the first packets
    torch.cuda.synchronize()
    r0, d0 = lib.inorder_stats()
    for t in subs[1:]:
        assert lib.protect_prepared_async(t["b"]) == 0
    torch.cuda.synchronize()
    for t in subs:
        _check_arena(orc, t["pk"], t["caps"], t["st"].cpu().tolist(),
                     t["before"], t["arena"].cpu().numpy().tobytes(),
                     t["offs"])
    assert lib.inorder_stats() == (r0 + 4, d0 + 2)
    assert lib.get_roc(ssrc) == orc.get_roc(ssrc)
    _key_left_equal(lib, orc, [ssrc], 1)


@pytest.mark.parametrize("name", ["icm128_hmac80", "gcm256_16"])
def test_one_stream_in_order_receive_out_of_place(name):
    """the receive side's in-order form out of place: forged tags rejected
    (their output never holds plaintext), the rest decrypted at e_0 + i,
    a reordered batch declined to the chain form; statuses, accepted
    plaintexts and the unchanged input against the oracle"""
    _gpu()
    rng = random.Random(773)
    ssrc = 0x29500000
    pols = [policy(name, ssrc=ssrc, seed=7)]
    snd, lib, orc = O.Session(pols), L.Session(pols), O.Session(pols)
    tag = POLICIES[name][4]
    seq = 0xffff - 900
    r0 = d0 = None
    for b, n in enumerate((8, 2000, 2000, 2000)):
        pk = []
        for k in range(n):
            p = rtp_packet(rng, ssrc, (seq + k) & 0xffff,
                           rng.choice((0, 7, 160, 1000)))
            rc, ref = snd.protect(p, len(p) + 64)
            assert rc == 0
            pk.append(ref)
        seq += n
        if b >= 1:
            for k in rng.sample(range(n), 30):
                x = bytearray(pk[k])
                x[-1] ^= 0x08
                pk[k] = bytes(x)
        if b == 3:
            pk[400], pk[401] = pk[401], pk[400]
        if b == 1:
            r0, d0 = lib.inorder_stats()
        st, bin_, ain, bout, aout, offs = _arena_run_oop(
            lib, pk, [len(p) for p in pk], 24, rng, op="unprotect")
        assert ain == bin_, "input arena changed"
        for i, p in enumerate(pk):
            rc, ref = orc.unprotect(p, len(p))
            assert st[i] == rc, (b, i, st[i], rc)
            o, m = offs[i], len(p) - tag
            if rc == 0:
                assert aout[o:o + len(ref)] == ref, (b, i)
            else:
                assert aout[o:o + m] in (bout[o:o + m], p[:m]), (b, i)
    assert lib.inorder_stats() == (r0 + 2, d0 + 1)
    assert lib.get_roc(ssrc) == orc.get_roc(ssrc)
    _key_left_equal(lib, orc, [ssrc], 1)
