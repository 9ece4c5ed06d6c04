"""Host-side packet-index / replay-window logic (no GPU).

srtp_mi355x_debug_index drives the library's own rdbx restatement
(libsrtp_amd/csrc/srtp_host.c) through sequences of sequence numbers; the
CPU oracle (pinned to the reference by tests/test_oracle_golden.py) gives the
expected statuses and ROCs through a null-cipher/null-auth session."""
import ctypes as C
import random

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O


def lib_index(seqs, window=128, allow_repeat=0, pending_roc=0):
    f = L.lib().srtp_mi355x_debug_index
    f.argtypes = [C.c_size_t, C.c_int, C.c_uint32, C.c_size_t, C.c_void_p,
                  C.c_void_p, C.c_void_p]
    n = len(seqs)
    s = (C.c_uint16 * n)(*seqs)
    st = (C.c_int32 * n)()
    est = (C.c_uint64 * n)()
    assert f(window, allow_repeat, pending_roc, n, s, st, est) == 0
    return list(st), list(est)


def oracle_index(seqs, window=128, allow_repeat=0, pending_roc=0):
    pol = dict(ssrc_type=1, ssrc=0x1234, cipher_type=0, cipher_key_len=0,
               auth_type=0, auth_key_len=0, auth_tag_len=0, sec_serv=0,
               use_mki=0, mki_size=0, window_size=window,
               allow_repeat_tx=allow_repeat, keys=["00" * 46])
    s = O.Session([pol])
    if pending_roc:
        s.set_roc(0x1234, pending_roc)
    st, est = [], []
    for q in seqs:
        pkt = bytes([0x80, 96, q >> 8, q & 0xff, 0, 0, 0, 0, 0, 0, 0x12, 0x34])
        rc, out = s.protect(pkt, 64)
        st.append(rc)
        if rc == 0:
            _, roc = s.get_roc(0x1234)
        est.append(((roc << 16) | q) if rc == 0 else 0)
    return st, est


def _check(seqs, **kw):
    ls, le = lib_index(seqs, **kw)
    os_, oe = oracle_index(seqs, **kw)
    assert ls == os_
    # the oracle reports the stream ROC after the packet: compare only the
    # packets that advanced the index
    for i, (a, b) in enumerate(zip(le, oe)):
        if ls[i] == 0 and a >= max([0] + le[:i]):
            assert a == b, i


def test_in_order_with_wrap():
    _check([(0xfff0 + i) & 0xffff for i in range(64)])


def test_first_packet_zero_and_duplicates():
    _check([0, 0, 1, 1, 2, 5, 3, 3, 4])


@pytest.mark.parametrize("window", [64, 100, 128, 1024])
def test_random_reorder(window):
    rng = random.Random(window)
    base = [(30000 + i) & 0xffff for i in range(3000)]
    seqs = []
    for q in base:
        seqs.append(q)
        if rng.random() < 0.2:
            seqs.append((q - rng.randrange(0, 2 * window)) & 0xffff)
    _check(seqs, window=window)


def test_allow_repeat_tx():
    _check([10, 11, 11, 12, 12, 12, 9], allow_repeat=1)


def test_pending_roc_advance_and_old():
    _check([5, 6, 7], pending_roc=3)
    _check([100, 101], pending_roc=1)
