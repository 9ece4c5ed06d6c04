"""ctypes view of oracle/liboracle.so (the CPU restatement) and of the
reference build in oracle/_ref/.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by libsrtp_amd.
"""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_INT = os.path.join(HERE, "_ref", "libsrtp_ref_int.so")
REF_OSSL = os.path.join(HERE, "_ref", "libsrtp_ref_ossl.so")


def build():
    subprocess.check_call(["make", "-s", "-f", os.path.join(HERE, "Makefile")])


class Policy(C.Structure):
    """orc_policy_t (oracle/srtp_oracle.h)."""
    _fields_ = [
        ("ssrc_type", C.c_int), ("ssrc", C.c_uint32),
        ("cipher_type", C.c_uint32), ("cipher_key_len", C.c_size_t),
        ("auth_type", C.c_uint32), ("auth_key_len", C.c_size_t),
        ("auth_tag_len", C.c_size_t), ("sec_serv", C.c_int),
        ("num_master_keys", C.c_size_t),
        ("keys", C.c_void_p * 16), ("mki_ids", C.c_void_p * 16),
        ("use_mki", C.c_int), ("mki_size", C.c_size_t),
        ("window_size", C.c_size_t), ("allow_repeat_tx", C.c_int),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.c_char_p
        L.orc_aes_encrypt.argtypes = [P, C.c_size_t, P, P]
        L.orc_sha1.argtypes = [P, C.c_size_t, P]
        L.orc_hmac_sha1.argtypes = [P, C.c_size_t, P, C.c_size_t, P]
        L.orc_icm_xor.argtypes = [P, C.c_size_t, P, P, P, C.c_size_t, P]
        L.orc_gcm_seal.argtypes = [P, C.c_size_t, P, P, C.c_size_t, P,
                                   C.c_size_t, P, P, C.c_size_t]
        L.orc_gcm_open.argtypes = [P, C.c_size_t, P, P, C.c_size_t, P,
                                   C.c_size_t, P, C.c_size_t, P]
        L.orc_session_create.argtypes = [C.POINTER(C.c_void_p)]
        L.orc_session_add.argtypes = [C.c_void_p, C.POINTER(Policy)]
        L.orc_session_free.argtypes = [C.c_void_p]
        L.orc_protect.argtypes = [C.c_void_p, P, C.c_size_t, P,
                                  C.POINTER(C.c_size_t), C.c_size_t]
        L.orc_unprotect.argtypes = [C.c_void_p, P, C.c_size_t, P,
                                    C.POINTER(C.c_size_t)]
        L.orc_key_left.argtypes = [C.c_void_p, C.c_uint32, C.c_size_t,
                                   C.POINTER(C.c_uint64)]
        L.orc_get_roc.argtypes = [C.c_void_p, C.c_uint32,
                                  C.POINTER(C.c_uint32)]
        L.orc_set_roc.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_unprotect_many.restype = None
        L.orc_unprotect_many.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p]
        L.orc_protect_many.restype = C.c_size_t
        L.orc_protect_many.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_uint32]
        _lib = L
    return _lib


def aes_encrypt(key, block):
    out = C.create_string_buffer(16)
    assert lib().orc_aes_encrypt(key, len(key), block, out) == 0
    return out.raw


def sha1(msg):
    out = C.create_string_buffer(20)
    lib().orc_sha1(msg, len(msg), out)
    return out.raw


def hmac_sha1(key, msg):
    out = C.create_string_buffer(20)
    assert lib().orc_hmac_sha1(key, len(key), msg, len(msg), out) == 0
    return out.raw


def icm_xor(key, salt14, iv16, data):
    out = C.create_string_buffer(max(1, len(data)))
    rc = lib().orc_icm_xor(key, len(key), salt14, iv16, data, len(data), out)
    return rc, out.raw[:len(data)]


def gcm_seal(key, iv, aad, pt, tag_len):
    ct = C.create_string_buffer(max(1, len(pt)))
    tag = C.create_string_buffer(16)
    assert lib().orc_gcm_seal(key, len(key), iv, aad, len(aad), pt, len(pt),
                              ct, tag, tag_len) == 0
    return ct.raw[:len(pt)] + tag.raw[:tag_len]


def gcm_open(key, iv, aad, ct, tag):
    pt = C.create_string_buffer(max(1, len(ct)))
    rc = lib().orc_gcm_open(key, len(key), iv, aad, len(aad), ct, len(ct),
                            tag, len(tag), pt)
    return rc, pt.raw[:len(ct)]


class Session:
    """One oracle session built from golden-fixture style policy dicts."""

    def __init__(self, policies):
        self._keep = []
        h = C.c_void_p()
        assert lib().orc_session_create(C.byref(h)) == 0
        self.h = h
        for p in policies:
            rc = self.add(p)
            if rc:
                raise ValueError("orc_session_add failed: %d" % rc)

    def add(self, p):
        pol = Policy()
        pol.ssrc_type = p["ssrc_type"]
        pol.ssrc = p["ssrc"]
        for f in ("cipher_type", "cipher_key_len", "auth_type",
                  "auth_key_len", "auth_tag_len", "sec_serv"):
            setattr(pol, f, p[f])
        pol.mki_size = p.get("mki_size", 0)
        pol.window_size = p.get("window_size", 128)
        pol.use_mki = int(p.get("use_mki", 0))
        pol.allow_repeat_tx = int(p.get("allow_repeat_tx", 0))
        keys = [bytes.fromhex(k) if isinstance(k, str) else bytes(k)
                for k in p["keys"]]
        mkis = [bytes.fromhex(k) if isinstance(k, str) else bytes(k)
                for k in p.get("mki_ids", [])]
        pol.num_master_keys = len(keys) if pol.use_mki else 1
        for i, k in enumerate(keys[:pol.num_master_keys]):
            b = C.create_string_buffer(k, max(64, len(k)))
            self._keep.append(b)
            pol.keys[i] = C.cast(b, C.c_void_p)
        for i, m in enumerate(mkis):
            b = C.create_string_buffer(m, max(16, len(m)))
            self._keep.append(b)
            pol.mki_ids[i] = C.cast(b, C.c_void_p)
        return lib().orc_session_add(self.h, C.byref(pol))

    def protect(self, rtp, cap, mki_index=0):
        out = C.create_string_buffer(max(cap, len(rtp)) + 64)
        n = C.c_size_t(cap)
        rc = lib().orc_protect(self.h, rtp, len(rtp), out, C.byref(n),
                               mki_index)
        return rc, (out.raw[:n.value] if rc == 0 else None)

    def protect_many(self, arena, offs, lens, out_cap):
        """orc_protect_many over packets at arena[offs[i]:+lens[i]] (numpy
        uint8 / uint64 / uint32 arrays), in order, into a new arena of the
        arena with out_cap bytes per packet; returns (failures, outputs as
        an (n, out_cap) array, out lengths)"""
        import numpy as np
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        ooff = np.arange(len(lens), dtype=np.uint64) * np.uint64(out_cap)
        out = np.zeros(len(lens) * out_cap, dtype=np.uint8)
        olen = np.zeros(len(lens), dtype=np.uint32)
        bad = lib().orc_protect_many(
            self.h, len(lens), arena.ctypes.data, offs.ctypes.data,
            lens.ctypes.data, out.ctypes.data, ooff.ctypes.data,
            olen.ctypes.data, out_cap)
        return bad, out.reshape(len(lens), out_cap), olen

    def unprotect_many(self, arena, offs, lens, out_cap):
        """orc_unprotect_many: every packet at arena[offs[i]:+lens[i]], in
        order; returns (statuses, outputs as an (n, out_cap) array, plaintext
        lengths)"""
        import numpy as np
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = len(lens)
        ooff = np.arange(n, dtype=np.uint64) * np.uint64(out_cap)
        out = np.zeros(n * out_cap, dtype=np.uint8)
        olen = np.zeros(n, dtype=np.uint32)
        st = np.zeros(n, dtype=np.int32)
        lib().orc_unprotect_many(self.h, n, arena.ctypes.data, offs.ctypes.data,
                                 lens.ctypes.data, out.ctypes.data,
                                 ooff.ctypes.data, olen.ctypes.data, out_cap,
                                 st.ctypes.data)
        return st, out.reshape(n, out_cap), olen

    def unprotect(self, srtp, cap):
        out = C.create_string_buffer(max(cap, len(srtp)) + 64)
        n = C.c_size_t(cap)
        rc = lib().orc_unprotect(self.h, srtp, len(srtp), out, C.byref(n))
        return rc, (out.raw[:n.value] if rc == 0 else None)

    def get_roc(self, ssrc):
        r = C.c_uint32()
        rc = lib().orc_get_roc(self.h, ssrc, C.byref(r))
        return rc, r.value

    def set_roc(self, ssrc, roc):
        return lib().orc_set_roc(self.h, ssrc, roc)

    def key_left(self, ssrc, j=0):
        """uses left of master key j of the stream (key limit counter)"""
        v = C.c_uint64()
        rc = lib().orc_key_left(self.h, ssrc, j, C.byref(v))
        return rc, v.value

    def __del__(self):
        try:
            lib().orc_session_free(self.h)
        except Exception:
            pass
