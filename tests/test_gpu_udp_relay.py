"""The socket-side batching caller (tools/udp_relay.c):
RTP over 127.0.0.1 UDP -> recvmmsg into a batch -> srtp_protect_batch (GPU)
-> sendmmsg -> sink recvmmsg -> srtp_unprotect_batch; every packet must come
back bit-identical to what the source sent, and the SRTP bytes that crossed
the socket must equal the CPU oracle's srtp_protect of the same RTP packets
in the same order (the relay dumps its key and every (RTP, SRTP) pair)."""
import json
import os
import struct
import subprocess
import tempfile

import pytest

import libsrtp_amd as L
from oracle import pyoracle as O

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
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "wire.bin")
        r = subprocess.run([BIN, str(packets), str(payload), str(batch),
                            str(chunk), path], capture_output=True, text=True,
                           timeout=100)
        assert r.returncode == 0, r.stdout + r.stderr
        res = json.loads(r.stdout.strip().splitlines()[-1])
        print(res)
        assert res["verified"] == packets and res["failed"] == 0
        blob = open(path, "rb").read()
    # the wire bytes against the oracle: a sender session with the relay's
    # key and policy (AES-128-ICM + HMAC-SHA1-80, ssrc_any_outbound)
    key, pos = blob[:30], 30
    pol = dict(ssrc_type=3, ssrc=0, cipher_type=1, cipher_key_len=30,
               auth_type=3, auth_key_len=20, auth_tag_len=10, sec_serv=3,
               window_size=1024, allow_repeat_tx=0,
               keys=[(key + bytes(16)).hex()])
    orc = O.Session([pol])
    n = 0
    while pos < len(blob):
        (a,) = struct.unpack_from("<H", blob, pos)
        rtp = blob[pos + 2:pos + 2 + a]
        pos += 2 + a
        (b,) = struct.unpack_from("<H", blob, pos)
        wire = blob[pos + 2:pos + 2 + b]
        pos += 2 + b
        rc, ref = orc.protect(rtp, len(rtp) + 64)
        assert rc == 0 and wire == ref, n
        n += 1
    assert n == packets


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
