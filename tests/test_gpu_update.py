"""srtp_update / srtp_stream_update against the reference's own outputs
(tests/golden/ref_update*.json, oracle/gen_update.c): what an update keeps
(srtp.c:3430-3617) -- the RTP extended sequence number and the SRTCP replay
database, for a specific-SSRC stream and for template clones -- with the same
key and with a new one, for AES-ICM + HMAC-SHA1 and AES-GCM.  Every op must
give the reference's status and bytes (the SRTCP index continues after an
update; old SRTCP packets are replays; old-key packets fail)."""
import pytest

import libsrtp_amd as L
from tests.golden_util import load

pytestmark = pytest.mark.gpu
H = bytes.fromhex
CASES = load("ref_update.json")["cases"] + load("ref_update_gcm.json")["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_update_matches_reference(case):
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")
    sess = {"snd": L.Session([case["snd"]]), "rcv": L.Session([case["rcv"]])}
    for i, op in enumerate(case["ops"]):
        s = sess[op["sess"]]
        if op["op"] == "update":
            assert s.update(op["policy"]) == op["status"], i
            continue
        st, out = getattr(s, op["op"])(H(op["in"]), op["cap"])
        assert st == op["status"], (i, op["op"], st, op["status"])
        if st == 0:
            assert out.hex() == op["out"], (i, op["op"])
