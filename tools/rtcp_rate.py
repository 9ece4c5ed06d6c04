"""Host-buffer SRTCP rate through srtp_protect_rtcp_batch /
srtp_unprotect_rtcp_batch (PCIe-inclusive wall clock; k_rtcp is not a bench
line).  usage: python tools/rtcp_rate.py [packets] [bytes]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libsrtp_amd as L  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    key = bytes(range(46)).hex()
    for name, ct, ckl, at, akl, tl in (("icm128_sha1_80", 1, 30, 3, 20, 10),
                                       ("gcm256_16", 7, 44, 0, 0, 16)):
        pol = dict(ssrc_type=1, ssrc=0x1234, cipher_type=ct, cipher_key_len=ckl,
                   auth_type=at, auth_key_len=akl, auth_tag_len=tl, sec_serv=3,
                   window_size=128, allow_repeat_tx=0, keys=[key])
        snd, rcv = L.Session([pol]), L.Session([pol])
        pkt = bytes([0x80, 200, 0, size // 4 - 1, 0, 0, 0x12, 0x34]) + \
            bytes(size - 8)
        pkts = [pkt] * n
        snd.protect_rtcp_batch(pkts[:1000])   # warm up
        snd2 = L.Session([pol])
        t0 = time.perf_counter()
        st, out = snd2.protect_rtcp_batch(pkts)
        t1 = time.perf_counter()
        st2, back = rcv.unprotect_rtcp_batch(out)
        t2 = time.perf_counter()
        assert all(s == 0 for s in st) and all(s == 0 for s in st2)
        assert all(b == pkt for b in back)
        print('{"tool": "rtcp_rate", "policy": "%s", "packets": %d, '
              '"bytes": %d, "protect_pkt_per_s": %.0f, '
              '"unprotect_pkt_per_s": %.0f}'
              % (name, n, size, n / (t1 - t0), n / (t2 - t1)))
        snd.close(), snd2.close(), rcv.close()


if __name__ == "__main__":
    main()
