"""Key-usage limit and SSRC-collision events (srtp.c:1723-1773,
crypto/kernel/key.c:74-90) against the reference's own outputs
(tests/golden/ref_*.json "events", oracle/gen_golden.c): the key limit is
lowered through a test hook exactly where the reference fixture lowered it
(its srtp_key_limit_ctx_t), and every op must give the reference's status,
bytes and the events the reference raised (soft limit on every packet past
it, hard limit -> key_expired, AES-GCM counting a forged packet and the
HMAC path not, collision when a stream is used in both directions)."""
import pytest

import libsrtp_amd as L
from tests.golden_util import load

pytestmark = pytest.mark.gpu
H = bytes.fromhex
CASES = load("ref_int.json")["events"] + load("ref_ossl.json")["events"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_events_match_reference(case):
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")
    got = []
    L.install_event_handler(lambda ev, ssrc: got.append([ev, ssrc]))
    try:
        sess = {"snd": L.Session([case["snd"]]), "rcv": L.Session([case["rcv"]])}
        for i, op in enumerate(case["ops"]):
            s = sess[op["sess"]]
            got.clear()
            if op["op"] == "set_limit":
                assert s.debug_set_key_limit(op["ssrc"], op["num_left"]) == 0
                continue
            if op["op"] == "protect":
                st, out = s.protect(H(op["in"]), op["cap"])
            else:
                st, out = s.unprotect(H(op["in"]), op["cap"])
            assert st == op["status"], (i, op["op"], st, op["status"])
            if st == 0:
                assert out.hex() == op["out"], i
            assert got == op["events"], (i, op["op"], got, op["events"])
    finally:
        L.install_event_handler(None)
