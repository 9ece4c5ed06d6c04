"""Session replication (srtp_mi355x_session_export / _import / _broadcast)
and BASELINE configs[4]'s N > 1 path with real kernels.

A replica must behave exactly as the session it was taken from: the next
packets of every stream (specific, MKI, AES-GCM, template clones) give the
same bytes and statuses on both, equal to the CPU oracle that saw every
packet in order; a receiver's replay window and index survive.  The N > 1
tests run two ranks on the one GPU of the box (SRTP_BENCH_DEVICE=0, gloo:
RCCL refuses two ranks on one device): bench.py's own multi-rank path, and a
two-rank job whose every output packet is compared with the C oracle.
"""
import json
import os
import random
import subprocess
import sys
import tempfile

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.test_gpu_parity import policy, rtp_packet

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpu():
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")


def _policies():
    tpl = policy("icm128_hmac80", ssrc_type=3, seed=7)   # ssrc_any_outbound
    return [policy("icm128_hmac80", ssrc=0x1111, seed=1),
            policy("gcm256_16", ssrc=0x2222, seed=2),
            policy("icm256_hmac80", ssrc=0x3333, seed=3, mki=4, nkeys=3),
            policy("icm128_hmac32", ssrc=0x4444, seed=4, window=1024), tpl]


def _batch(rng, seqs, ssrcs, sizes=(0, 17, 160, 1400)):
    return [rtp_packet(rng, ssrcs[i % len(ssrcs)], seqs[i % len(ssrcs)] + i //
                       len(ssrcs) & 0xffff, rng.choice(sizes), ts=i)
            for i in range(len(ssrcs) * 24)]


def _oracle_protect(orc, pkts, mki):
    res = []
    for p, m in zip(pkts, mki):
        rc, out = orc.protect(p, len(p) + 64, m)
        res.append((rc, out))
    return res


def test_export_import_sender_continues():
    """protect batch 1 on the session, replicate it, protect batch 2 on the
    session and on the replica: identical, and equal to the oracle."""
    _gpu()
    rng = random.Random(41)
    pols = _policies()
    ssrcs = [0x1111, 0x2222, 0x3333, 0x4444, 0x5555]   # 0x5555: a clone
    seqs = [0xfff0, 0x10, 0x7ff0, 0x100, 0xfffe]
    src, orc = L.Session(pols), O.Session(pols)
    b1 = _batch(rng, seqs, ssrcs)
    mki1 = [(i // 5) % 3 if ssrcs[i % 5] == 0x3333 else 0
            for i in range(len(b1))]
    st, out = src.protect_batch(b1, [len(p) + 64 for p in b1], mki1)
    for (rc, exp), s, o in zip(_oracle_protect(orc, b1, mki1), st, out):
        assert s == rc == 0 and o == exp
    blob = src.export_blob()
    rep = L.Session.from_blob(blob)
    assert rep.export_blob() == blob          # a replica exports the same
    b2 = _batch(rng, [s + 24 for s in seqs], ssrcs)
    mki2 = [2 if ssrcs[i % 5] == 0x3333 else 0 for i in range(len(b2))]
    caps = [len(p) + 64 for p in b2]
    st_a, out_a = src.protect_batch(b2, caps, mki2)
    st_b, out_b = rep.protect_batch(b2, caps, mki2)
    exp = _oracle_protect(orc, b2, mki2)
    for i in range(len(b2)):
        assert st_a[i] == st_b[i] == exp[i][0] == 0, i
        assert out_a[i] == out_b[i] == exp[i][1], i
    for s in ssrcs:
        assert src.get_roc(s) == rep.get_roc(s)


def test_export_import_receiver_state():
    """A receiver's indices and replay windows travel: after batch 1, the
    replica rejects batch 1's packets as replays and accepts batch 2,
    exactly as the original and the oracle do."""
    _gpu()
    rng = random.Random(42)
    pols = [dict(p, ssrc_type=1 if p["ssrc_type"] == 1 else 2)
            for p in _policies()]                    # template: any_inbound
    ssrcs = [0x1111, 0x2222, 0x3333, 0x4444, 0x5555]
    seqs = [0xffe0, 0x10, 0x7ff0, 0x100, 0x2000]
    snd = O.Session([dict(p, ssrc_type=3 if p["ssrc_type"] == 2 else 1)
                     for p in pols])
    b1 = _batch(rng, seqs, ssrcs)
    b2 = _batch(rng, [s + 24 for s in seqs], ssrcs)
    p1 = [snd.protect(p, len(p) + 64, 1 if ssrcs[i % 5] == 0x3333 else 0)[1]
          for i, p in enumerate(b1)]
    p2 = [snd.protect(p, len(p) + 64)[1] for p in b2]
    rcv, orc = L.Session(pols), O.Session(pols)
    st, out = rcv.unprotect_batch(p1)
    for i, p in enumerate(p1):
        rc, exp = orc.unprotect(p, len(p))
        assert st[i] == rc == 0 and out[i] == exp == b1[i], i
    rep = L.Session.from_blob(rcv.export_blob())
    # replays of batch 1 (every third packet), then batch 2
    pk = [p1[i] for i in range(0, len(p1), 3)] + p2
    st_a, out_a = rcv.unprotect_batch(pk)
    st_b, out_b = rep.unprotect_batch(pk)
    for i, p in enumerate(pk):
        rc, exp = orc.unprotect(p, len(p))
        assert st_a[i] == st_b[i] == rc, (i, st_a[i], st_b[i], rc)
        if rc == 0:
            assert out_a[i] == out_b[i] == exp, i
    assert any(s == 9 for s in st_b)           # replay_fail seen


def test_export_refuses_bad_blob():
    _gpu()
    src = L.Session([policy("icm128_hmac80")])
    blob = bytearray(src.export_blob())
    for bad in (bytes(blob[:-1]), b"X" + bytes(blob[1:]), bytes(blob) + b"\0"):
        with pytest.raises(RuntimeError):
            L.Session.from_blob(bad)


def test_replica_device_batch_bit_identical():
    """The replica's key records drive the device pre-pass and k_gcm /
    k_icm_hmac exactly as the original's: the same 64k-packet batch
    protected on both sessions is byte-identical."""
    _gpu()
    import torch
    for name, trailer in (("gcm256_16", 16), ("icm128_hmac80", 10)):
        src = L.Session([policy(name)])
        rep = L.Session.from_blob(src.export_blob())
        n, payload = 65536, 1400
        slot = (12 + payload + trailer + 15) & ~15
        g = torch.Generator(device="cuda").manual_seed(9)
        a = torch.randint(0, 256, (n, slot), dtype=torch.uint8, device="cuda",
                          generator=g)
        seq = (torch.arange(n, device="cuda") + 0x1234) & 0xffff
        a[:, 0], a[:, 1] = 0x80, 96
        a[:, 2], a[:, 3] = (seq >> 8).to(torch.uint8), (seq & 0xff).to(torch.uint8)
        a[:, 8:12] = torch.tensor([0xca, 0xfe, 0xba, 0xbe], dtype=torch.uint8,
                                  device="cuda")
        outs = []
        for s in (src, rep):
            d = a.clone().view(-1)
            off = torch.arange(n, dtype=torch.int64, device="cuda") * slot
            ln = torch.full((n,), 12 + payload, dtype=torch.int32, device="cuda")
            cap = torch.full((n,), slot, dtype=torch.int32, device="cuda")
            st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            assert s.protect_device(d, off, ln, d, off, cap, st) == 0
            assert int((st != 0).sum()) == 0
            assert s.prepass_stats() == (1, 0)   # the device pre-pass ran
            outs.append(d)
        assert torch.equal(outs[0], outs[1]), name


def _run(cmd, env, timeout):
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    return r


def _two_rank_env():
    env = dict(os.environ, SRTP_BENCH_DEVICE="0", SRTP_DIST_BACKEND="gloo",
               HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_two_ranks_real_kernels():
    """bench.py --config gcm256 --gpus 2 (BASELINE configs[4]'s code path,
    2^16 packets per rank): two ranks with real HIP sessions replicated
    from rank 0, one JSON line with n_gpus 2, no host-path batch, and the
    roofline of rank 0's kernel."""
    _gpu()
    r = _run([sys.executable, "bench.py", "--config", "gcm256", "--gpus", "2",
              "--packets", "65536", "--steps", "3", "--warmup", "1",
              "--no-cpu-baseline", "--traffic", "off"],
             _two_rank_env(), 300)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["packets_total"] == 2 * 65536
    assert rec["prepass"]["host_batches"] == 0
    assert rec["roofline"]["kernel"] == "k_gcm"
    assert rec["roofline"]["kernel_ms"] > 0
    assert "session_export" in rec["session_replication"]


def test_two_ranks_vs_oracle():
    """Two ranks (tests/replica_rank.py): rank 0 creates the AES-256-GCM
    session of both ranks' streams, the replica reaches rank 1 through
    bench.replicate_session; each rank protects 8192 packets of its own
    stream with srtp_protect_device.  Every packet of both ranks equals the
    C oracle's."""
    _gpu()
    import numpy as np
    out = tempfile.mkdtemp(prefix="srtp_rep_", dir="/tmp")
    port = str(29500 + os.getpid() % 1000)
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
          "--nproc-per-node=2", "--master-addr=127.0.0.1",
          "--master-port=" + port, "tests/replica_rank.py", out],
         _two_rank_env(), 300)
    for r in range(2):
        z = np.load(os.path.join(out, "rank%d.npz" % r))
        pol = json.loads(str(z["policy"]))
        orc = O.Session([pol])
        bad, exp, olen = orc.protect_many(z["arena"], z["off"], z["len"],
                                          int(z["slot"]))
        assert bad == 0
        n = len(z["len"])
        got = z["out"].reshape(n, -1)
        assert (z["status"] == 0).all()
        assert (z["olen"] == olen).all()
        for i in range(n):
            assert bytes(got[i, :olen[i]]) == bytes(exp[i, :olen[i]]), (r, i)
