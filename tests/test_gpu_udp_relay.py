"""The socket-side batching caller (tools/udp_relay.c):
RTP over 127.0.0.1 UDP -> recvmmsg into a batch -> srtp_protect_batch (GPU)
-> sendmmsg -> sink recvmmsg -> srtp_unprotect_batch; every packet must come
back bit-identical to what the source sent."""
import json
import os
import subprocess

import pytest

import libsrtp_amd as L

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "udp_relay")


@pytest.mark.parametrize("packets,payload,batch,chunk", [
    (20000, 1400, 8192, 64),   # 1400-byte payloads, partial last batch
    (40000, 160, 16384, 128),  # G.711 frames
    (3, 0, 2, 1),              # header-only packets, tiny batches
])
def test_udp_relay_roundtrip(packets, payload, batch, chunk):
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")
    assert os.path.exists(BIN), "tools/udp_relay not built (build())"
    r = subprocess.run([BIN, str(packets), str(payload), str(batch),
                        str(chunk)], capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["verified"] == packets and res["failed"] == 0
