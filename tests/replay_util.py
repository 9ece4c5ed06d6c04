"""Rebuilds the packets of tests/golden/ref_replay.json (oracle/gen_replay.c:
replay-window / index-estimation runs of the reference driven by its
test/ut_sim.c) and checks any protect/unprotect implementation against the
reference's statuses and output digests."""
from tests.golden_util import load

FNV0 = 0xcbf29ce484222325


def fnv(h, data):
    for b in data:
        h = ((h ^ b) * 0x100000001b3) & 0xffffffffffffffff
    return h


def runs():
    return load("ref_replay.json")["runs"]


def run_id(r):
    return "w%d-%s" % (r["window"], r["pattern"])


def policy(r):
    key = bytes.fromhex(r["key"]) + bytes(16)
    return dict(ssrc_type=1, ssrc=0x5eed0001, cipher_type=1, cipher_key_len=30,
                auth_type=3, auth_key_len=20, auth_tag_len=10, sec_serv=3,
                window_size=r["window"], allow_repeat_tx=0, keys=[key.hex()])


def packet(idx, j):
    seq = idx & 0xffff
    pay = (idx * 2654435761) & 0xffffffff
    return (bytes([0x80, 0x60, seq >> 8, seq & 0xff]) + j.to_bytes(4, "big")
            + bytes([0x5e, 0xed, 0x00, 0x01]) + pay.to_bytes(4, "big"))


def check_run(r, protect_many, unprotect_many):
    """protect_many(pkts) / unprotect_many(pkts) -> (statuses, outputs);
    each called once per direction with the run's whole packet list (an
    implementation may split it into calls of any size)."""
    pk = [packet(idx, j) for j, idx in enumerate(r["tx_idx"])]
    st, out = protect_many(pk)
    st = [int(s) for s in st]
    assert st == r["tx_status"], next(
        (j, st[j], r["tx_status"][j]) for j in range(len(st))
        if st[j] != r["tx_status"][j])
    h = FNV0
    for s, o in zip(st, out):
        if s == 0:
            h = fnv(h, o)
    assert "%016x" % h == r["tx_fnv"]
    deliver = [(k, src) for k, src in enumerate(r["rx_src"])
               if r["rx_status"][k] != -1]
    st, res = unprotect_many([out[src] for _, src in deliver])
    h = FNV0
    for (k, src), s, o in zip(deliver, st, res):
        assert int(s) == r["rx_status"][k], (k, src, int(s),
                                             r["rx_status"][k])
        if s == 0:
            assert o == pk[src], k
            h = fnv(h, o)
    assert "%016x" % h == r["rx_fnv"]
