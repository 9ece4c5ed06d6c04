"""Mass (re)key timing: srtp_create with N streams of distinct master keys,
then one srtp_update of all N (a rekey), with the session keys derived on
the GPU (k_kdf, the default) and on the host (SRTP_MI355X_HOST_KDF=1).
Prints one JSON line per (cipher, KDF side).

    python3 tools/rekey_bench.py [--streams 65536]
"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

CIPHERS = {"icm128_hmac80": (1, 30, 3, 20, 10, 3),
           "gcm256_16": (7, 44, 0, 0, 16, 3)}


def run_one(name, n, host):
    import libsrtp_amd as L
    from bench import stream_keys
    c, ckl, a, akl, tag, sv = CIPHERS[name]
    keys = stream_keys(n)
    keys2 = stream_keys(n, seed=0x1234)

    def pols(ks):
        return [dict(ssrc_type=1, ssrc=0x10000 + i, cipher_type=c,
                     cipher_key_len=ckl, auth_type=a, auth_key_len=akl,
                     auth_tag_len=tag, sec_serv=sv, keys=[k])
                for i, k in enumerate(ks)]
    import ctypes as C
    from libsrtp_amd.srtp import _PolicyHolder

    def chain(ps):   # the srtp_policy_t list, built before the clock starts
        hs = [_PolicyHolder(p) for p in ps]
        for x, y in zip(hs, hs[1:]):
            x.policy.next = C.pointer(y.policy)
        return hs
    h1, h2 = chain(pols(keys)), chain(pols(keys2))
    lib = L.lib()
    L.Session([pols(keys[:1])[0]]).close()   # HIP and library initialisation
    sess = C.c_void_p()
    t0 = time.perf_counter()
    assert lib.srtp_create(C.byref(sess), C.byref(h1[0].policy)) == 0
    t1 = time.perf_counter()
    assert lib.srtp_update(sess, C.byref(h2[0].policy)) == 0
    t2 = time.perf_counter()
    lib.srtp_dealloc(sess)
    return {"cipher": name, "streams": n, "kdf": "host" if host else "gpu",
            "create_s": round(t1 - t0, 4), "update_s": round(t2 - t1, 4),
            "streams_per_s_create": round(n / (t1 - t0)),
            "streams_per_s_update": round(n / (t2 - t1))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=65536)
    ap.add_argument("--one", nargs=2)
    a = ap.parse_args()
    if a.one:
        print(json.dumps(run_one(a.one[0], a.streams, a.one[1] == "host")))
        return
    for name in CIPHERS:
        for side in ("gpu", "host"):
            env = dict(os.environ, SRTP_MI355X_HOST_KDF="1" if side == "host"
                       else "0")
            r = subprocess.run([sys.executable, __file__, "--streams",
                                str(a.streams), "--one", name, side],
                               env=env, capture_output=True, text=True,
                               timeout=600)
            sys.stdout.write(r.stdout)
            if r.returncode:
                sys.stderr.write(r.stderr[-2000:])
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
