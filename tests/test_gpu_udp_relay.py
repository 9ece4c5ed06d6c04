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


def test_rtcp_bench_roundtrip():
    """tools/rtcp_bench.c: 65536 SRTCP packets per batch through the C batch
    API, ICM-128 + HMAC-80 and GCM-256; the tool exits non-zero unless every
    packet unprotects back to its original bytes."""
    if not L.lib().srtp_mi355x_gpu_available():
        pytest.skip("no GPU")
    exe = os.path.join(ROOT, "tools", "rtcp_bench")
    assert os.path.exists(exe), "tools/rtcp_bench not built (build())"
    r = subprocess.run([exe, "65536", "100", "1"], capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [json.loads(x) for x in r.stdout.strip().splitlines()]
    assert [x["policy"] for x in lines] == ["icm128_sha1_80", "gcm256_16"]
    assert all(x["verified"] for x in lines)
