"""Randomised device-path stress against the oracle (GPU box).

Each seed builds a session of 1..600 streams over random policies (AES-ICM
and AES-GCM, HMAC tags, replay windows, MKI with several keys, or one
ssrc_any template for all of them), then runs batches through every
device form the library chooses among -- one stream in order (in place, out
of place, asynchronous back to back), the order-free and sorted forms, key
buckets forced on / off / by default -- with reordering, duplicates, jumps
and unknown SSRCs and application-set ROCs on the sender side and shuffles,
forgeries and replays on the receiver side.  Every status and byte of both sides is compared with
the oracle called once per packet, and the streams' ROCs at the end.

  python tests/stress_random.py [seconds] [first_seed]

(test infrastructure, kept under tests/ with the oracle's other callers;
not collected by pytest: a run takes minutes)

Prints one line per seed and a summary; exits 1 on the first mismatch
(with the seed, so that tests can pin it).
"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import libsrtp_amd as L                                       # noqa: E402
from oracle import pyoracle as O                              # noqa: E402
from tests.test_gpu_parity import policy, rtp_packet          # noqa: E402
from tests.test_gpu_prepass import (_arena_run_oop, _device_run,  # noqa: E402
                                    _interleaved)

POLS = ["icm128_hmac80", "icm128_hmac32", "icm256_hmac80", "gcm128_16",
        "gcm256_16", "gcm256_8"]


def _async_many(lib, batches, rng):
    """several protect batches submitted asynchronously one after another,
    the stream drained once at the end -> [(st, before, after, offs)]"""
    import torch
    subs = []
    for pk, caps in batches:
        offs, pos = [], 0
        for p, c in zip(pk, caps):
            offs.append(pos)
            pos += (max(len(p), c) + 24 + 15) & ~15
        before = bytearray(rng.randbytes(pos + 16))
        for o, p in zip(offs, pk):
            before[o:o + len(p)] = p
        t = dict(before=bytes(before), offs=offs,
                 arena=torch.frombuffer(bytearray(before),
                                        dtype=torch.uint8).cuda(),
                 off=torch.tensor(offs, dtype=torch.int64).cuda(),
                 ln=torch.tensor([len(p) for p in pk],
                                 dtype=torch.int32).cuda(),
                 cap=torch.tensor(caps, dtype=torch.int32).cuda(),
                 st=torch.full((len(pk),), -1, dtype=torch.int32).cuda())
        t["b"] = lib.prepare_device(t["arena"], t["off"], t["ln"], t["arena"],
                                    t["off"], t["cap"], t["st"])
        subs.append(t)
    torch.cuda.synchronize()
    for t in subs:
        assert lib.protect_prepared_async(t["b"]) == 0
    torch.cuda.synchronize()
    return [(t["st"].cpu().tolist(), t["before"],
             t["arena"].cpu().numpy().tobytes(), t["offs"]) for t in subs]


def run_seed(seed):
    rng = random.Random(seed)
    ns = rng.choice([1, 1, 2, 17, 64, 600])
    one_cipher = rng.random() < 0.5
    c0 = rng.choice(POLS)
    ssrcs = [0x2a000000 + 7 * k + seed for k in range(ns)]
    # MKI sessions: every stream with 2-3 master keys, a random key per
    # protected packet (srtp.c:2536-2545), the receiver picking by MKI
    nkeys = rng.choice([2, 3]) if rng.random() < 0.25 else 0
    mkw = dict(mki=4, nkeys=nkeys) if nkeys else {}
    pols = [policy(c0 if one_cipher else rng.choice(POLS), ssrc=s, seed=k,
                   window=rng.choice([64, 128, 128, 1024]), **mkw)
            for k, s in enumerate(ssrcs)]
    spols = rpols = pols
    templ = not nkeys and ns > 1 and rng.random() < 0.2
    if templ:
        # one ssrc_any_outbound / _inbound template for every stream: the
        # streams are created on the device (srtp_stream_clone)
        tp = policy(c0, ssrc_type=3, seed=5)
        spols, rpols = [tp], [dict(tp, ssrc_type=2)]
    slib, sorc = L.Session(spols), O.Session(spols)
    rlib, rorc = L.Session(rpols), O.Session(rpols)
    seq0 = {s: rng.randrange(1, 0xffff) for s in ssrcs}
    what = []
    for b in range(6):
        L.lib().srtp_mi355x_set_key_buckets(rng.choice([-1, -1, 0, 1]))
        if b and not templ and rng.random() < 0.25:
            # an application-set ROC (srtp_stream_set_roc, srtp.c:5137-5167)
            # on a sender stream: ahead, or the current one (pending)
            s = rng.choice(ssrcs)
            roc = sorc.get_roc(s)[1] + rng.choice([0, 1])
            assert slib.set_roc(s, roc) == 0 and sorc.set_roc(s, roc) == 0
            what.append("roc")
        per = rng.choice([1, 5, 40, 150]) if ns > 1 else \
            rng.choice([20, 700, 3000])
        clean = ns == 1 and rng.random() < 0.6
        pk = _interleaved(rng, ssrcs, seq0, per,
                          shuffle_within=0 if clean else
                          rng.choice([0, 0, 0.1]),
                          steps=(1,) if clean else (1, 1, 1, 2),
                          payloads=(0, 1, 13, 160, 300, 1000))
        if rng.random() < 0.3:
            # headers with CSRCs and extensions (the payload's offset and the
            # keystream phase vary per packet); sequence numbers kept
            pk = [rtp_packet(rng, int.from_bytes(p[8:12], "big"),
                             (p[2] << 8) | p[3], len(p) - 12,
                             cc=rng.choice([0, 0, 1, 3]),
                             xwords=rng.choice([-1, -1, 0, 2]))
                  for p in pk]
        event = "none" if clean else rng.choice(["none", "none", "dup",
                                                 "unknown", "jump"])
        if event == "dup" and len(pk) > 10:
            pk.insert(rng.randrange(5, len(pk)), pk[rng.randrange(0, 5)])
        elif event == "unknown":
            pk.insert(rng.randrange(0, len(pk)),
                      rtp_packet(rng, 0x0badf00d, 7, 30))
        elif event == "jump":
            s = rng.choice(ssrcs)
            seq0[s] += rng.randrange(100, 20000)
        caps = [len(p) + rng.choice([16, 16, 40]) for p in pk]
        mode = rng.choice(["inplace", "inplace", "oop", "async", "host",
                           "single"])
        if mode == "single" and len(pk) > 400:
            mode = "host"
        if nkeys and mode not in ("host", "single"):
            mode = "mki"
        what.append("%s/%d/%s/%s" % (mode, len(pk), event,
                                     "clean" if clean else "mixed"))
        sent = []
        if mode == "async":
            # this batch and a second one of the next indices, back to back
            pk2 = _interleaved(rng, ssrcs, seq0, max(1, per // 2),
                               steps=(1,) if clean else (1, 2),
                               payloads=(0, 160))
            caps2 = [len(p) + 16 for p in pk2]
            res = _async_many(slib, [(pk, caps), (pk2, caps2)], rng)
            for (q, cq), (st, before, after, offs) in zip(
                    [(pk, caps), (pk2, caps2)], res):
                expect = bytearray(before)
                for i, p in enumerate(q):
                    rc, ref = sorc.protect(p, cq[i])
                    assert st[i] == rc, ("async", b, i, st[i], rc)
                    if rc == 0:
                        expect[offs[i]:offs[i] + len(ref)] = ref
                        sent.append(ref)
                assert bytes(expect) == after, ("async arena", b)
        elif mode in ("host", "single"):
            # the host-buffer batch API (srtp_protect_batch: staged into HBM,
            # the device pre-pass) or one srtp_protect per packet (k_one)
            mk = [rng.randrange(nkeys) for _ in pk] if nkeys else [0] * len(pk)
            if mode == "host":
                st, out = slib.protect_batch(pk, caps, mki=mk,
                                             inplace=rng.random() < 0.5)
            else:
                st, out = [], []
                for i, p in enumerate(pk):
                    rc, o = slib.protect(p, caps[i], mk[i],
                                         inplace=rng.random() < 0.5)
                    st.append(rc)
                    out.append(o)
            for i, p in enumerate(pk):
                rc, ref = sorc.protect(p, caps[i], mk[i])
                assert st[i] == rc, (mode, b, event, i, st[i], rc)
                assert rc or out[i] == ref, (mode, b, event, i)
                if rc == 0:
                    sent.append(ref)
        elif mode == "mki":
            mk = [rng.randrange(nkeys) for _ in pk]
            st, out = _device_run(slib, pk, caps, "protect", mki=mk)
            for i, p in enumerate(pk):
                rc, ref = sorc.protect(p, caps[i], mk[i])
                assert st[i] == rc, ("mki", b, event, i, st[i], rc)
                assert rc or out[i] == ref, ("mki", b, event, i)
                if rc == 0:
                    sent.append(ref)
        elif mode == "oop":
            st, bin_, ain, bout, aout, offs = _arena_run_oop(
                slib, pk, caps, 24, rng)
            assert ain == bin_, "input arena changed"
            for i, p in enumerate(pk):
                rc, ref = sorc.protect(p, caps[i])
                assert st[i] == rc, (b, i, st[i], rc)
                if rc == 0:
                    assert aout[offs[i]:offs[i] + len(ref)] == ref, (b, i)
                    sent.append(ref)
        else:
            st, out = _device_run(slib, pk, caps, "protect")
            for i, p in enumerate(pk):
                rc, ref = sorc.protect(p, caps[i])
                assert st[i] == rc, (b, event, i, st[i], rc)
                assert rc or out[i] == ref, (b, event, i)
                if rc == 0:
                    sent.append(ref)
        rx = list(sent)
        if not clean and rng.random() < 0.5:
            rng.shuffle(rx)
        for k in rng.sample(range(len(rx)), min(len(rx), rng.choice([0, 3]))):
            x = bytearray(rx[k])
            x[-1] ^= 0x11
            rx[k] = bytes(x)
        if rx and rng.random() < 0.3:
            rx.append(rx[rng.randrange(len(rx))])
        if not rx:
            continue
        rmode = rng.random()
        if rmode < 0.15 or (rmode < 0.25 and len(rx) <= 400):
            # the host-buffer batch API, or one srtp_unprotect per packet
            if rmode < 0.15:
                st, out = rlib.unprotect_batch(rx, inplace=rng.random() < 0.5)
            else:
                st, out = zip(*[rlib.unprotect(p, inplace=rng.random() < 0.5)
                                for p in rx])
            for i, p in enumerate(rx):
                rc, ref = rorc.unprotect(p, len(p))
                assert st[i] == rc, ("rx host", b, i, st[i], rc)
                assert rc or out[i] == ref, ("rx host", b, i)
            continue
        if rng.random() < 0.3:   # out of place: the input arena untouched
            st, bin_, ain, bout, aout, offs = _arena_run_oop(
                rlib, rx, [len(p) for p in rx], 24, rng, op="unprotect")
            assert ain == bin_, "rx input arena changed"
            for i, p in enumerate(rx):
                rc, ref = rorc.unprotect(p, len(p))
                assert st[i] == rc, ("rx oop", b, i, st[i], rc)
                assert rc or aout[offs[i]:offs[i] + len(ref)] == ref, \
                    ("rx oop", b, i)
            continue
        st, out = _device_run(rlib, rx, [len(p) for p in rx], "unprotect")
        for i, p in enumerate(rx):
            rc, ref = rorc.unprotect(p, len(p))
            assert st[i] == rc, ("rx", b, i, st[i], rc)
            assert rc or out[i] == ref, ("rx", b, i)
    for s in ssrcs:
        assert slib.get_roc(s) == sorc.get_roc(s), hex(s)
        assert rlib.get_roc(s) == rorc.get_roc(s), hex(s)
    L.lib().srtp_mi355x_set_key_buckets(-1)
    return ns, what


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 240.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    t0 = time.time()
    n = 0
    while time.time() - t0 < secs:
        try:
            ns, what = run_seed(seed)
        except AssertionError as e:
            print("FAIL seed %d: %r" % (seed, e), flush=True)
            raise SystemExit(1)
        print("seed %d ok: %d streams, %s" % (seed, ns, " ".join(what)),
              flush=True)
        seed += 1
        n += 1
    print("stress: %d seeds ok in %.0f s" % (n, time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
