"""Helpers to read the committed reference fixtures (tests/golden/*.json).

The fixtures were produced by oracle/gen_golden.c driving the reference
(cisco/libsrtp built from its sources, oracle/Makefile.ref); see
tests/golden/README.md.
"""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def all_cases():
    out = []
    for f in ("ref_int.json", "ref_ossl.json"):
        for c in load(f)["cases"]:
            out.append(c)
    return out


def case_ids():
    return [c["name"] for c in all_cases()]


def prefix_cases():
    """Keystream-prefix sessions (null auth with a tag, srtp.c:2729-2741)
    from oracle/gen_golden.c -DPREFIX_CASES; the oracle does not restate
    this legacy mode, so these rows pin the library to the reference
    directly."""
    return load("ref_prefix.json")["cases"]


def kat_cases():
    """The published packet KATs of test/srtp_driver.c (srtp_validate*,
    srtp_test_empty_payload*), reproduced by the reference build before
    oracle/gen_golden.c emits them."""
    out = []
    for f in ("ref_int.json", "ref_ossl.json"):
        out += load(f)["kats"]
    return out


def replay_ops(case, snd, rcv):
    """Runs a case's op rows on two session objects exposing protect /
    unprotect / protect_rtcp / unprotect_rtcp; asserts status and bytes."""
    H = bytes.fromhex
    for i, op in enumerate(case["ops"]):
        s = snd if op["sess"] == "snd" else rcv
        kind = op["op"]
        if kind == "protect":
            st, out = s.protect(H(op["in"]), op["cap"], op["mki_index"])
        elif kind == "protect_rtcp":
            st, out = s.protect_rtcp(H(op["in"]), op["cap"], op["mki_index"])
        elif kind == "unprotect":
            st, out = s.unprotect(H(op["in"]), op["cap"])
        else:
            st, out = s.unprotect_rtcp(H(op["in"]), op["cap"])
        assert st == op["status"], (case["name"], i, kind, st, op["status"])
        if st == 0:
            assert out.hex() == op["out"], (case["name"], i, kind)


def replay_ops_batched(case, snd, rcv):
    """Like replay_ops, but consecutive RTP ops of one session and direction
    go through ONE protect_batch / unprotect_batch call."""
    H = bytes.fromhex
    sess = {"snd": snd, "rcv": rcv}
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
            assert st[k] == o["status"], (case["name"], i + k, o["op"], st[k],
                                          o["status"])
            if st[k] == 0:
                assert out[k].hex() == o["out"], (case["name"], i + k, o["op"])
        i = j
