"""Replay window and index estimation of the GPU library against the
reference's own ut_sim-driven runs (tests/golden/ref_replay.json, made by
oracle/gen_replay.c: windows 64/128/1024/32767; receiver reordering, large
index gaps across many ROC values, sender-side reordering).

Every entry point is checked: the single-packet API, host-buffer batches
(whole run in one call, and in 97-packet calls) and the device-arena API
(srtp_protect_device / srtp_unprotect_device: the device pre-pass, or its
exact host fallback)."""
import pytest

import libsrtp_amd as L
from tests import replay_util as RU
from tests.test_gpu_parity import _gpu

pytestmark = pytest.mark.gpu
RUNS = RU.runs()
IDS = [RU.run_id(r) for r in RUNS]


def _single(fn):
    def many(pkts):
        st, out = [], []
        for p in pkts:
            s, o = fn(p, len(p) + 64)
            st.append(s)
            out.append(o)
        return st, out
    return many


def _batched(fn, chunk=None):
    def many(pkts):
        st, out = [], []
        step = chunk or max(1, len(pkts))
        for i in range(0, len(pkts), step):
            part = pkts[i:i + step]
            s, o = fn(part, [len(p) + 64 for p in part])
            st += s
            out += o
        return st, out
    return many


def _device(sess, fname):
    def many(pkts):
        import torch
        caps = [len(p) + 64 for p in pkts]
        offs, pos = [], 0
        for c in caps:
            offs.append(pos)
            pos += (c + 15) & ~15
        buf = bytearray(pos + 16)
        for o, p in zip(offs, pkts):
            buf[o:o + len(p)] = p
        arena = torch.frombuffer(buf, dtype=torch.uint8).cuda()
        out = torch.zeros_like(arena)
        off = torch.tensor(offs, dtype=torch.int64).cuda()
        ln = torch.tensor([len(p) for p in pkts], dtype=torch.int32).cuda()
        cap = torch.tensor(caps, dtype=torch.int32).cuda()
        st = torch.full((len(pkts),), -1, dtype=torch.int32).cuda()
        assert getattr(sess, fname)(arena, off, ln, out, off, cap, st) == 0
        st, cap = st.cpu().tolist(), cap.cpu().tolist()
        host = out.cpu().numpy().tobytes()
        return st, [host[o:o + c] if s == 0 else None
                    for o, c, s in zip(offs, cap, st)]
    return many


def _sessions(run):
    return L.Session([RU.policy(run)]), L.Session([RU.policy(run)])


def _rocs(run, snd, rcv):
    assert snd.get_roc(0x5eed0001)[1] == run["roc_tx"]
    assert rcv.get_roc(0x5eed0001)[1] == run["roc_rx"]


@pytest.mark.parametrize("run", RUNS, ids=IDS)
def test_replay_single_packet_api(run):
    _gpu()
    snd, rcv = _sessions(run)
    RU.check_run(run, _single(snd.protect), _single(rcv.unprotect))
    _rocs(run, snd, rcv)


@pytest.mark.parametrize("run", RUNS, ids=IDS)
@pytest.mark.parametrize("chunk", [None, 97], ids=["whole", "chunk97"])
def test_replay_batch_api(run, chunk):
    _gpu()
    snd, rcv = _sessions(run)
    RU.check_run(run, _batched(snd.protect_batch, chunk),
                 _batched(rcv.unprotect_batch, chunk))
    _rocs(run, snd, rcv)


@pytest.mark.parametrize("run", RUNS, ids=IDS)
def test_replay_device_api(run):
    _gpu()
    snd, rcv = _sessions(run)
    RU.check_run(run, _device(snd, "protect_device"),
                 _device(rcv, "unprotect_device"))
    _rocs(run, snd, rcv)
