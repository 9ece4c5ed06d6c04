"""One rank of tests/test_gpu_broadcast.py: srtp_mi355x_session_broadcast
between two processes on one GPU, with tests/c/rccl_shim.so standing in for
RCCL (loaded RTLD_GLOBAL, so the library's run-time symbol lookup finds it).
Usage: bcast_rank.py <rank> <socket path> <case> <out json>"""
import ctypes as C
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def policies():
    from tests.test_gpu_parity import policy
    pols = [policy("icm128_hmac80", ssrc=0x100 + k, seed=k) for k in range(3)]
    pols.append(policy("gcm256_16", ssrc=0x200, seed=9))
    pols.append(policy("icm256_hmac80", ssrc_type=3, seed=12))   # template
    return pols


def batch(seed, seq0):
    """the same packets on both ranks: the four streams and two SSRCs that
    the template clones"""
    from tests.test_gpu_parity import rtp_packet
    rng = random.Random(seed)
    ssrcs = [0x100, 0x101, 0x102, 0x200, 0x7000, 0x7001]
    return [rtp_packet(rng, ssrcs[i % 6], (seq0 + i // 6) & 0xffff,
                       rng.choice([0, 20, 160, 1400])) for i in range(240)]


def main(rank, path, case, out):
    import libsrtp_amd as L
    shim = C.CDLL(os.path.join(ROOT, "tests", "c", "rccl_shim.so"),
                  mode=C.RTLD_GLOBAL)
    shim.shim_comm_init.restype = C.c_void_p
    shim.shim_comm_init.argtypes = [C.c_int, C.c_int, C.c_char_p]
    comm = shim.shim_comm_init(rank, 2, path.encode())
    assert comm, "shim connect"
    res = {"rank": rank}
    sess = None
    if case in ("replica", "alloc_fail") and rank == 0:
        sess = L.Session(policies())
        st, _ = sess.protect_batch(batch(1, 0xfff0))   # advance the state
        assert all(s == 0 for s in st)
    if case == "alloc_fail" and rank == 1:
        L.lib().srtp_mi355x_debug_inject_failure(3, 1)
    try:
        rep = L.session_broadcast(sess, comm, 0, 0)
        res["bcast"] = "ok"
    except RuntimeError as e:
        res["bcast"] = str(e)
        rep = None
    if rep is not None:
        st, outp = rep.protect_batch(batch(2, 0x0020))
        res["status"] = list(st)
        res["out"] = [o.hex() if o else None for o in outp]
        res["blob"] = rep.export_blob().hex()
        res["roc"] = rep.get_roc(0x101)[1]
    shim.shim_comm_free(C.c_void_p(comm))
    with open(out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2], sys.argv[3], sys.argv[4])
