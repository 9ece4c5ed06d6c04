"""libsrtp's legacy keystream-prefix mode (null auth with a non-zero tag and
the auth service on: the tag is the packet's first tag_len keystream bytes,
srtp/srtp.c:2729-2741 protect, 3006-3020 unprotect; crypto/hash/
null_auth.c:80 prefix_len = out_len).  Such sessions run per packet through
the cipher / auth vtables (srtp_host.c run_routed); the fixtures come from
the reference itself (oracle/gen_golden.c -DPREFIX_CASES), through the
single-packet and batch APIs."""
import pytest

import libsrtp_amd as L
from tests.golden_util import prefix_cases, replay_ops, replay_ops_batched

pytestmark = pytest.mark.gpu
CASES = prefix_cases()


def _gpu():
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_prefix_single(case):
    _gpu()
    replay_ops(case, L.Session([case["snd"]]), L.Session([case["rcv"]]))


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_prefix_batched(case):
    _gpu()
    replay_ops_batched(case, L.Session([case["snd"]]),
                       L.Session([case["rcv"]]))
