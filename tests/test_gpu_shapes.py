"""GPU parity of the uniform-key protect paths (k_icm_hmac's lane-quad
cooperative steady state, srtp_icm.hip; AES-GCM by k_gcm, srtp_gcm.hip)
over device
arenas of many packet shapes, against the CPU oracle (oracle/srtp_oracle.c,
pinned to the reference's fixtures).

Groups of 64 packets vary header size (CSRC count, extension), payload
length (0 .. 4500 bytes, across the 4 KiB counter-cache epoch), 16-byte
packet placement (every 64-byte misalignment of input and output), in place
and out of place, with mixed-shape groups.  Every output byte and length
must equal the oracle's, and no byte outside the packets' output ranges may
change (the cooperative path writes whole aligned 64-byte segments).
"""
import random

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O
from tests.test_gpu_parity import POLICIES, policy, rtp_packet

pytestmark = pytest.mark.gpu


def _gpu():
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")


SIZES = (0, 1, 3, 15, 16, 17, 51, 52, 53, 160, 1388, 1400, 1452, 4000, 4095,
         4096)


def _groups(rng, ngroups, mixed_every, ssrcs, seq):
    """packets (in batch order) with 64-packet groups of one shape"""
    pkts = []
    for g in range(ngroups):
        payload = rng.choice(SIZES + (4097, 4500) if g % 7 == 6 else SIZES)
        cc = rng.choice([0, 0, 1, 3, 15])
        xw = rng.choice([-1, -1, 0, 1, 2, 5])
        for k in range(64):
            ssrc = ssrcs[rng.randrange(len(ssrcs))]
            p, c, x = payload, cc, xw
            if mixed_every and g % mixed_every == 1 and k == 17:
                p = (payload + 5) % 1500   # one odd packet: group falls back
            pkts.append(rtp_packet(rng, ssrc, seq[ssrc], p, c, x,
                                   ts=rng.randrange(1 << 32)))
            seq[ssrc] = (seq[ssrc] + 1) & 0xffff
    return pkts


def _payload_len(p):
    cc = p[0] & 15
    h = 12 + 4 * cc
    if p[0] & 0x10:
        h += 4 + 4 * ((p[h + 2] << 8) | p[h + 3])
    return len(p) - h


def _layout(rng, pkts, trailer, base_skew):
    """16-byte aligned offsets with random gaps: every 64-byte phase"""
    off, cur = [], base_skew
    for p in pkts:
        off.append(cur)
        cur += (len(p) + trailer + 15) & ~15
        cur += 16 * rng.randrange(4)
    return off, cur + 64


def _run(seed, ngroups, inplace, mixed_every=0, nssrc=1, tail=0,
         pname="icm128_hmac80"):
    import torch
    _gpu()
    rng = random.Random(seed)
    ssrcs = [0xcafebabe + 7919 * k for k in range(nssrc)]
    if nssrc == 1:
        pol = policy(pname, ssrc=ssrcs[0], seed=seed)
    else:   # ssrc_any_outbound template: every stream clones one key
        pol = policy(pname, ssrc=0, ssrc_type=3, seed=seed)
    seq = {s: rng.randrange(0x10000) for s in ssrcs}
    pkts = _groups(rng, ngroups, mixed_every, ssrcs, seq)
    pkts += _groups(rng, 1, 0, ssrcs, seq)[:tail]
    n = len(pkts)
    trailer = POLICIES[pname][4]
    ioff, isize = _layout(rng, pkts, trailer, 16 * rng.randrange(4))
    if inplace:
        ooff, osize = ioff, isize
    else:
        ooff, osize = _layout(rng, pkts, trailer, 16 * rng.randrange(4))
    fill = 0xa5
    ain = torch.full((isize,), fill, dtype=torch.uint8)
    for p, o in zip(pkts, ioff):
        ain[o:o + len(p)] = torch.frombuffer(bytearray(p), dtype=torch.uint8)
    dev = torch.device("cuda", 0)
    d_in = ain.to(dev)
    d_out = d_in if inplace else torch.full((osize,), 0x5a, dtype=torch.uint8,
                                             device=dev)
    before = d_out.cpu().numpy().tobytes()
    t = lambda v, dt: torch.tensor(v, dtype=dt, device=dev)
    caps = [len(p) + trailer for p in pkts]
    olen = t(caps, torch.int32)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    s = L.Session([pol])
    assert s.protect_device(d_in, t(ioff, torch.int64),
                            t([len(p) for p in pkts], torch.int32), d_out,
                            t(ooff, torch.int64), olen, st) == 0
    import numpy as np
    out_np = d_out.cpu().numpy()
    out = out_np.tobytes()
    st, olen = st.cpu().tolist(), olen.cpu().tolist()
    orc = O.Session([pol])
    covered = np.zeros(len(out), dtype=bool)
    for i, p in enumerate(pkts):
        rc, ref = orc.protect(p, caps[i])
        assert st[i] == rc == 0, (i, st[i], rc)
        assert olen[i] == len(ref), (i, olen[i], len(ref))
        got = out[ooff[i]:ooff[i] + olen[i]]
        assert got == ref, (i, len(p), next(k for k in range(len(ref))
                                          if got[k] != ref[k]))
        covered[ooff[i]:ooff[i] + olen[i]] = True
    # nothing outside the packets' output ranges was written
    if not inplace:
        diff = (out_np != np.frombuffer(before, dtype=np.uint8)) & ~covered
        assert not diff.any(), ("stray writes", np.nonzero(diff)[0][:8])
    else:
        for i, p in enumerate(pkts):
            e = ooff[i] + olen[i]
            nxt = ooff[i + 1] if i + 1 < n else len(out)
            assert out[e:nxt] == before[e:nxt], ("stray write after", i)
    # unprotect the protected arena (every 5th packet tampered) into a fresh
    # arena: plaintext == the original packets, tampered ones auth_fail
    tam = torch.tensor([i for i in range(n) if i % 5 == 3], dtype=torch.int64)
    src = d_out.clone()
    flip = torch.tensor(ooff, dtype=torch.int64)[tam] + \
        torch.tensor(olen, dtype=torch.int64)[tam] - 1
    src[flip.to(dev)] ^= 1
    roff, rsize = _layout(rng, pkts, trailer, 16 * rng.randrange(4))
    dst = torch.full((rsize,), 0x3c, dtype=torch.uint8, device=dev)
    rlen = t(olen, torch.int32)
    rcap = t([len(p) for p in pkts], torch.int32)
    rst = torch.zeros(n, dtype=torch.int32, device=dev)
    r = L.Session([pol])
    assert r.unprotect_device(src, t(ooff, torch.int64), rlen, dst,
                              t(roff, torch.int64), rcap, rst) == 0
    back = dst.cpu().numpy().tobytes()
    rst, rcap = rst.cpu().tolist(), rcap.cpu().tolist()
    for i, p in enumerate(pkts):
        if i % 5 == 3:
            assert rst[i] == 7, (i, rst[i])   # srtp_err_status_auth_fail
            continue
        assert rst[i] == 0 and rcap[i] == len(p), (i, rst[i], rcap[i])
        assert back[roff[i]:roff[i] + len(p)] == p, i


def test_shapes_one_stream_out_of_place():
    _run(1, ngroups=48, inplace=False)


def test_shapes_one_stream_in_place():
    _run(2, ngroups=48, inplace=True)


def test_shapes_mixed_groups_fall_back():
    # every 3rd group has one odd packet: those waves take the per-lane path
    _run(3, ngroups=30, inplace=False, mixed_every=3, tail=37)


def test_shapes_template_many_ssrcs():
    # per-lane SSRC / ROC / sequence differ inside a wave
    _run(4, ngroups=24, inplace=True, nssrc=9, tail=5)


def test_shapes_roc_wrap():
    """sequence numbers crossing 0xffff inside groups: per-lane ROC"""
    import torch
    _gpu()
    rng = random.Random(11)
    pol = policy("icm128_hmac80", ssrc=0x1234abcd, seed=11)
    pkts = [rtp_packet(rng, 0x1234abcd, (0xff00 + k) & 0xffff, 1400, 0, -1,
                       ts=k) for k in range(64 * 8)]
    slot = 1424
    n = len(pkts)
    dev = torch.device("cuda", 0)
    arena = torch.zeros(n * slot, dtype=torch.uint8)
    for i, p in enumerate(pkts):
        arena[i * slot:i * slot + len(p)] = torch.frombuffer(bytearray(p),
                                                             dtype=torch.uint8)
    d = arena.to(dev)
    off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    ln = torch.full((n,), 1412, dtype=torch.int32, device=dev)
    cap = torch.full((n,), slot, dtype=torch.int32, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    s = L.Session([pol])
    assert s.protect_device(d, off, ln, d, off, cap, st) == 0
    out = d.cpu().numpy().tobytes()
    orc = O.Session([pol])
    for i, p in enumerate(pkts):
        rc, ref = orc.protect(p, slot)
        assert rc == 0 and out[i * slot:i * slot + len(ref)] == ref, i


# AES-GCM: k_gcm (uniform keys: four AES tables + 8-copy GHASH table)


@pytest.mark.parametrize("pname", ["gcm128_16", "gcm256_16", "gcm256_8"])
def test_shapes_gcm_out_of_place(pname):
    _run(21, ngroups=40, inplace=False, tail=9, pname=pname)


@pytest.mark.parametrize("pname", ["gcm128_16", "gcm256_16"])
def test_shapes_gcm_in_place_mixed(pname):
    _run(22, ngroups=30, inplace=True, mixed_every=3, pname=pname)


def test_shapes_gcm_template_many_ssrcs():
    _run(23, ngroups=20, inplace=False, nssrc=7, tail=3, pname="gcm256_16")
