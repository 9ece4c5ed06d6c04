"""ctypes binding of include/srtp_mi355x.h.

Mirrors the reference's operator surface (srtp_policy_t, srtp_create,
srtp_protect, srtp_unprotect, ... -- include/srtp.h of cisco/libsrtp 3.0.0)
with the same names, argument meaning and status codes, plus the batch
extension (srtp_protect_batch / srtp_unprotect_batch over host buffers and
srtp_protect_device / srtp_unprotect_device over HBM arenas).
"""
import ctypes as C
import enum
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# LIBSRTP_MI355X_LIB: timing experiments point at alternative builds
LIB_PATH = os.environ.get("LIBSRTP_MI355X_LIB",
                          os.path.join(HERE, "libsrtp_mi355x.so"))


def build():
    """Compile libsrtp_mi355x.so in-tree (hipcc for gfx950 + gcc)."""
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.check_call(["make", "-s", "-C", HERE, "-j" + jobs])


class Status(enum.IntEnum):
    """srtp_err_status_t, include/srtp.h:183-220."""
    ok = 0
    fail = 1
    bad_param = 2
    alloc_fail = 3
    dealloc_fail = 4
    init_fail = 5
    terminus = 6
    auth_fail = 7
    cipher_fail = 8
    replay_fail = 9
    replay_old = 10
    algo_fail = 11
    no_such_op = 12
    no_ctx = 13
    cant_check = 14
    key_expired = 15
    socket_err = 16
    signal_err = 17
    nonce_bad = 18
    read_fail = 19
    write_fail = 20
    parse_err = 21
    encode_err = 22
    semaphore_err = 23
    pfkey_err = 24
    bad_mki = 25
    pkt_idx_old = 26
    pkt_idx_adv = 27
    buffer_small = 28
    cryptex_err = 29


SSRC_SPECIFIC, SSRC_ANY_INBOUND, SSRC_ANY_OUTBOUND = 1, 2, 3


class CryptoPolicy(C.Structure):
    _fields_ = [("cipher_type", C.c_uint32), ("cipher_key_len", C.c_size_t),
                ("auth_type", C.c_uint32), ("auth_key_len", C.c_size_t),
                ("auth_tag_len", C.c_size_t), ("sec_serv", C.c_int)]


class SSRC(C.Structure):
    _fields_ = [("type", C.c_int), ("value", C.c_uint32)]


class MasterKey(C.Structure):
    _fields_ = [("key", C.c_void_p), ("mki_id", C.c_void_p)]


class Policy(C.Structure):
    pass


Policy._fields_ = [
    ("ssrc", SSRC), ("rtp", CryptoPolicy), ("rtcp", CryptoPolicy),
    ("key", C.c_void_p), ("keys", C.POINTER(C.POINTER(MasterKey))),
    ("num_master_keys", C.c_size_t), ("use_mki", C.c_bool),
    ("mki_size", C.c_size_t), ("window_size", C.c_size_t),
    ("allow_repeat_tx", C.c_bool), ("enc_xtn_hdr", C.c_void_p),
    ("enc_xtn_hdr_count", C.c_size_t), ("use_cryptex", C.c_bool),
    ("next", C.POINTER(Policy)),
]


class DeviceBatch(C.Structure):
    """srtp_device_batch_t."""
    _fields_ = [("n", C.c_size_t), ("in_", C.c_void_p), ("in_off", C.c_void_p),
                ("in_len", C.c_void_p), ("out", C.c_void_p),
                ("out_off", C.c_void_p), ("out_len", C.c_void_p),
                ("status", C.c_void_p), ("mki_index", C.c_void_p),
                ("stream", C.c_void_p)]


_lib = None


def lib():
    """Load libsrtp_mi355x.so; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        # torch bundles its own libamdhip64.so.7 (same soname as ROCm's):
        # whichever loads first serves the whole process, so let torch's
        # runtime win or torch cannot see the GPU afterwards
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("libsrtp_mi355x.so not built (run build() / "
                          "__graft_entry__.build()): " + LIB_PATH)
    L = C.CDLL(LIB_PATH)
    P, S, SP = C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)
    sig = {
        "srtp_init": ([], C.c_int), "srtp_shutdown": ([], C.c_int),
        "srtp_create": ([C.POINTER(C.c_void_p), C.POINTER(Policy)], C.c_int),
        "srtp_stream_add": ([P, C.POINTER(Policy)], C.c_int),
        "srtp_stream_remove": ([P, C.c_uint32], C.c_int),
        "srtp_update": ([P, C.POINTER(Policy)], C.c_int),
        "srtp_stream_update": ([P, C.POINTER(Policy)], C.c_int),
        "srtp_dealloc": ([P], C.c_int),
        "srtp_protect": ([P, C.c_char_p, S, P, SP, S], C.c_int),
        "srtp_unprotect": ([P, C.c_char_p, S, P, SP], C.c_int),
        "srtp_protect_rtcp": ([P, C.c_char_p, S, P, SP, S], C.c_int),
        "srtp_unprotect_rtcp": ([P, C.c_char_p, S, P, SP], C.c_int),
        "srtp_protect_batch": ([P, S, P, P, P, P, P, P], C.c_int),
        "srtp_unprotect_batch": ([P, S, P, P, P, P, P], C.c_int),
        "srtp_protect_rtcp_batch": ([P, S, P, P, P, P, P, P], C.c_int),
        "srtp_unprotect_rtcp_batch": ([P, S, P, P, P, P, P], C.c_int),
        "srtp_protect_device": ([P, C.POINTER(DeviceBatch)], C.c_int),
        "srtp_protect_device_async": ([P, C.POINTER(DeviceBatch)], C.c_int),
        "srtp_unprotect_device": ([P, C.POINTER(DeviceBatch)], C.c_int),
        "srtp_get_protect_trailer_length": ([P, S, SP], C.c_int),
        "srtp_get_protect_rtcp_trailer_length": ([P, S, SP], C.c_int),
        "srtp_stream_get_roc": ([P, C.c_uint32, C.POINTER(C.c_uint32)],
                                C.c_int),
        "srtp_stream_set_roc": ([P, C.c_uint32, C.c_uint32], C.c_int),
        "srtp_mi355x_set_timing": ([P, C.c_int], None),
        "srtp_mi355x_last_kernel_ms": ([P], C.c_double),
        "srtp_mi355x_gpu_available": ([], C.c_int),
        "srtp_mi355x_prepass_stats": ([P, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint64)], None),
        "srtp_mi355x_prepass_last_abort": ([P], C.c_int),
        "srtp_mi355x_prepass_sorted_batches": ([P], C.c_uint64),
        "srtp_mi355x_bucket_batches": ([P], C.c_uint64),
        "srtp_mi355x_inorder_stats": ([P, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint64)], None),
        "srtp_mi355x_debug_key_left": ([P, C.c_uint32, C.c_size_t,
                                        C.POINTER(C.c_uint64)], C.c_int),
        "srtp_mi355x_debug_set_key_limit": ([P, C.c_uint32, C.c_uint64],
                                            C.c_int),
        "srtp_mi355x_debug_inject_failure": ([C.c_int, C.c_int], None),
        "srtp_mi355x_set_key_buckets": ([C.c_int], None),
        "srtp_mi355x_unprotect_stats": ([P] + [C.POINTER(C.c_uint32)] * 3,
                                        None),
        "srtp_mi355x_session_export": ([P, P, S, SP], C.c_int),
        "srtp_mi355x_session_import": ([C.POINTER(C.c_void_p), P, S],
                                       C.c_int),
        "srtp_mi355x_session_broadcast": ([C.POINTER(C.c_void_p), P, C.c_int,
                                           P], C.c_int),

        "srtp_get_version_string": ([], C.c_char_p),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    for name in ("rtp_default", "rtcp_default", "aes_cm_128_hmac_sha1_32",
                 "aes_cm_128_null_auth", "null_cipher_hmac_sha1_80",
                 "null_cipher_hmac_null", "aes_cm_256_hmac_sha1_80",
                 "aes_cm_256_hmac_sha1_32", "aes_cm_256_null_auth",
                 "aes_cm_192_hmac_sha1_80", "aes_cm_192_hmac_sha1_32",
                 "aes_cm_192_null_auth", "aes_gcm_128_16_auth",
                 "aes_gcm_256_16_auth"):
        f = getattr(L, "srtp_crypto_policy_set_" + name)
        f.argtypes = [C.POINTER(CryptoPolicy)]
        f.restype = None
    _lib = L
    return L


def policy_setter(name):
    """CryptoPolicy filled by srtp_crypto_policy_set_<name>()."""
    cp = CryptoPolicy()
    getattr(lib(), "srtp_crypto_policy_set_" + name)(C.byref(cp))
    return cp


def _hex(b):
    return bytes.fromhex(b) if isinstance(b, str) else bytes(b)


class _PolicyHolder:
    """Builds an srtp_policy_t from a dict (the tests/golden format) and
    keeps every buffer it points to alive."""

    def __init__(self, d):
        self.keep = []
        p = Policy()
        p.ssrc.type = d["ssrc_type"]
        p.ssrc.value = d.get("ssrc", 0)
        for dst, pre in ((p.rtp, ""), (p.rtcp, "rtcp_")):
            dst.cipher_type = d.get(pre + "cipher_type", d["cipher_type"])
            dst.cipher_key_len = d.get(pre + "cipher_key_len",
                                       d["cipher_key_len"])
            dst.auth_type = d.get(pre + "auth_type", d["auth_type"])
            dst.auth_key_len = d.get(pre + "auth_key_len", d["auth_key_len"])
            dst.auth_tag_len = d.get(pre + "auth_tag_len", d["auth_tag_len"])
            dst.sec_serv = d.get(pre + "sec_serv", d["sec_serv"])
        keys = [_hex(k) for k in d["keys"]]
        mkis = [_hex(m) for m in d.get("mki_ids", [])]
        p.window_size = d.get("window_size", 128)
        p.allow_repeat_tx = bool(d.get("allow_repeat_tx", 0))
        if d.get("use_mki"):
            n = len(keys)
            arr = (C.POINTER(MasterKey) * n)()
            for i in range(n):
                kb = C.create_string_buffer(keys[i], max(64, len(keys[i])))
                mb = C.create_string_buffer(mkis[i], max(16, len(mkis[i])))
                mk = MasterKey(C.cast(kb, C.c_void_p), C.cast(mb, C.c_void_p))
                self.keep += [kb, mb, mk]
                arr[i] = C.pointer(mk)
            self.keep.append(arr)
            p.keys = C.cast(arr, C.POINTER(C.POINTER(MasterKey)))
            p.num_master_keys = n
            p.use_mki = True
            p.mki_size = d["mki_size"]
        else:
            kb = C.create_string_buffer(keys[0], max(64, len(keys[0])))
            self.keep.append(kb)
            p.key = C.cast(kb, C.c_void_p)
        ids = d.get("enc_xtn_hdr") or []
        if ids:
            xb = (C.c_uint8 * len(ids))(*ids)
            self.keep.append(xb)
            p.enc_xtn_hdr = C.cast(xb, C.c_void_p)
            p.enc_xtn_hdr_count = len(ids)
        p.use_cryptex = bool(d.get("use_cryptex", 0))
        self.policy = p


def session_broadcast(sess, comm_ptr, root, stream=0):
    """srtp_mi355x_session_broadcast over an RCCL communicator (ncclComm_t
    address, e.g. torch's ProcessGroupNCCL._comm_ptr()): on rank `root`
    `sess` is the session to replicate (returned as is), elsewhere pass None
    and get the replica."""
    L = lib()
    st = L.srtp_init()
    if st:
        raise RuntimeError("srtp_init failed: %s" % Status(st).name)
    h = C.c_void_p(sess.h.value if sess is not None else None)
    st = L.srtp_mi355x_session_broadcast(C.byref(h), C.c_void_p(comm_ptr),
                                         root, C.c_void_p(stream or None))
    if st:
        raise RuntimeError("session broadcast: %s" % Status(st).name)
    if sess is not None:
        return sess
    out = Session.__new__(Session)
    out.L = L
    out.h = h
    return out


class EventData(C.Structure):
    """srtp_event_data_t (include/srtp.h:1690-1700)"""
    _fields_ = [("session", C.c_void_p), ("ssrc", C.c_uint32),
                ("event", C.c_int)]


EVENT_HANDLER = C.CFUNCTYPE(None, C.POINTER(EventData))
_handler_keep = []


def install_event_handler(fn):
    """srtp_install_event_handler: fn(event, ssrc) per event; None removes"""
    L = lib()
    L.srtp_install_event_handler.argtypes = [C.c_void_p]
    L.srtp_install_event_handler.restype = C.c_int
    if fn is None:
        _handler_keep.clear()
        return L.srtp_install_event_handler(None)
    cb = EVENT_HANDLER(lambda p: fn(p.contents.event, p.contents.ssrc))
    _handler_keep[:] = [cb]
    return L.srtp_install_event_handler(C.cast(cb, C.c_void_p))


class Session:
    """An srtp_t.  `policies` is a list of dicts in the golden format:
    ssrc_type, ssrc, cipher_type, cipher_key_len, auth_type, auth_key_len,
    auth_tag_len, sec_serv, keys (hex), [use_mki, mki_size, mki_ids],
    window_size, allow_repeat_tx."""

    def __init__(self, policies):
        L = lib()
        st = L.srtp_init()
        if st:
            raise RuntimeError("srtp_init failed: %s" % Status(st).name)
        self.L = L
        self.h = C.c_void_p()
        holders = [_PolicyHolder(p) for p in policies]
        for a, b in zip(holders, holders[1:]):
            a.policy.next = C.pointer(b.policy)
        st = L.srtp_create(C.byref(self.h),
                           C.byref(holders[0].policy) if holders else None)
        if st:
            raise RuntimeError("srtp_create failed: %s" % Status(st).name)

    def export_blob(self):
        """srtp_mi355x_session_export: the session's streams, derived
        session keys and stream state as bytes (secret material)"""
        n = C.c_size_t()
        st = self.L.srtp_mi355x_session_export(self.h, None, 0, C.byref(n))
        if st:
            raise RuntimeError("session export: %s" % Status(st).name)
        buf = C.create_string_buffer(n.value)
        st = self.L.srtp_mi355x_session_export(self.h, buf, n.value,
                                               C.byref(n))
        if st:
            raise RuntimeError("session export: %s" % Status(st).name)
        return buf.raw[:n.value]

    @classmethod
    def from_blob(cls, blob):
        """srtp_mi355x_session_import: a replica of the exported session on
        the current HIP device"""
        L = lib()
        st = L.srtp_init()
        if st:
            raise RuntimeError("srtp_init failed: %s" % Status(st).name)
        self = cls.__new__(cls)
        self.L = L
        self.h = C.c_void_p()
        buf = C.create_string_buffer(bytes(blob), len(blob))
        st = L.srtp_mi355x_session_import(C.byref(self.h), buf, len(blob))
        if st:
            self.h = C.c_void_p()
            raise RuntimeError("session import: %s" % Status(st).name)
        return self

    def add_stream(self, policy):
        h = _PolicyHolder(policy)
        return Status(self.L.srtp_stream_add(self.h, C.byref(h.policy)))

    def remove_stream(self, ssrc):
        return Status(self.L.srtp_stream_remove(self.h, ssrc))

    def update(self, policy):
        h = _PolicyHolder(policy)
        return Status(self.L.srtp_update(self.h, C.byref(h.policy)))

    def update_all(self, policies):
        """srtp_update with a linked list of policies (one rekey call)"""
        holders = [_PolicyHolder(p) for p in policies]
        for a, b in zip(holders, holders[1:]):
            a.policy.next = C.pointer(b.policy)
        return Status(self.L.srtp_update(self.h, C.byref(holders[0].policy)))

    # -- single packet (srtp_protect / srtp_unprotect) ---------------------
    # inplace=True passes one buffer as both input and output, as the
    # reference's in-place calls do (cryptex behaves differently then)
    def protect(self, rtp, cap=None, mki_index=0, inplace=False):
        cap = len(rtp) + 144 if cap is None else cap
        out = C.create_string_buffer(max(cap, len(rtp), 1))
        n = C.c_size_t(cap)
        if inplace:
            C.memmove(out, rtp, len(rtp))
            src = out
        else:
            src = rtp
        st = self.L.srtp_protect(self.h, src, len(rtp), out, C.byref(n),
                                 mki_index)
        return Status(st), (out.raw[:n.value] if st == 0 else None)

    def unprotect(self, srtp, cap=None, inplace=False):
        cap = len(srtp) if cap is None else cap
        out = C.create_string_buffer(max(cap, len(srtp), 1))
        n = C.c_size_t(cap)
        if inplace:
            C.memmove(out, srtp, len(srtp))
            src = out
        else:
            src = srtp
        st = self.L.srtp_unprotect(self.h, src, len(srtp), out, C.byref(n))
        return Status(st), (out.raw[:n.value] if st == 0 else None)

    # -- SRTCP (srtp_protect_rtcp / srtp_unprotect_rtcp) -------------------
    def protect_rtcp(self, rtcp, cap=None, mki_index=0):
        cap = len(rtcp) + 148 if cap is None else cap
        out = C.create_string_buffer(max(cap, len(rtcp), 1))
        n = C.c_size_t(cap)
        st = self.L.srtp_protect_rtcp(self.h, rtcp, len(rtcp), out,
                                      C.byref(n), mki_index)
        return Status(st), (out.raw[:n.value] if st == 0 else None)

    def unprotect_rtcp(self, srtcp, cap=None):
        cap = len(srtcp) if cap is None else cap
        out = C.create_string_buffer(max(cap, len(srtcp), 1))
        n = C.c_size_t(cap)
        st = self.L.srtp_unprotect_rtcp(self.h, srtcp, len(srtcp), out,
                                        C.byref(n))
        return Status(st), (out.raw[:n.value] if st == 0 else None)

    # -- batch over host buffers -------------------------------------------
    def protect_batch(self, pkts, caps=None, mki=None,
                      fn="srtp_protect_batch", inplace=False):
        n = len(pkts)
        caps = [len(p) + 148 for p in pkts] if caps is None else caps
        if inplace:   # rtp[i] == srtp[i]
            ins = outs = [C.create_string_buffer(p, max(1, c, len(p)))
                          for c, p in zip(caps, pkts)]
        else:
            ins = [C.create_string_buffer(p, max(1, len(p))) for p in pkts]
            outs = [C.create_string_buffer(max(1, c, len(p)))
                    for c, p in zip(caps, pkts)]
        inp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in ins])
        outp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in outs])
        ilen = (C.c_size_t * n)(*[len(p) for p in pkts])
        olen = (C.c_size_t * n)(*caps)
        mk = (C.c_size_t * n)(*(mki or [0] * n))
        st = (C.c_int * n)()
        rc = getattr(self.L, fn)(self.h, n, inp, ilen, outp, olen, mk, st)
        if rc:
            raise RuntimeError("%s: %s" % (fn, Status(rc).name))
        return ([Status(s) for s in st],
                [outs[i].raw[:olen[i]] if st[i] == 0 else None
                 for i in range(n)])

    def unprotect_batch(self, pkts, caps=None, fn="srtp_unprotect_batch",
                        inplace=False):
        n = len(pkts)
        caps = [len(p) for p in pkts] if caps is None else caps
        if inplace:   # srtp[i] == rtp[i]
            ins = outs = [C.create_string_buffer(p, max(1, c, len(p)))
                          for c, p in zip(caps, pkts)]
        else:
            ins = [C.create_string_buffer(p, max(1, len(p))) for p in pkts]
            outs = [C.create_string_buffer(max(1, c, len(p)))
                    for c, p in zip(caps, pkts)]
        inp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in ins])
        outp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in outs])
        ilen = (C.c_size_t * n)(*[len(p) for p in pkts])
        olen = (C.c_size_t * n)(*caps)
        st = (C.c_int * n)()
        rc = getattr(self.L, fn)(self.h, n, inp, ilen, outp, olen, st)
        if rc:
            raise RuntimeError("%s: %s" % (fn, Status(rc).name))
        return ([Status(s) for s in st],
                [outs[i].raw[:olen[i]] if st[i] == 0 else None
                 for i in range(n)])

    def protect_rtcp_batch(self, pkts, caps=None, mki=None):
        return self.protect_batch(pkts, caps, mki, "srtp_protect_rtcp_batch")

    def unprotect_rtcp_batch(self, pkts, caps=None):
        return self.unprotect_batch(pkts, caps, "srtp_unprotect_rtcp_batch")

    # -- batch over device (HBM) arenas: torch tensors on cuda --------------
    def _device(self, fn, arena_in, in_off, in_len, arena_out, out_off,
                out_len, status, mki=None, stream=None):
        b = DeviceBatch()
        b.n = in_off.numel()
        b.in_ = arena_in.data_ptr()
        b.in_off = in_off.data_ptr()
        b.in_len = in_len.data_ptr()
        b.out = arena_out.data_ptr()
        b.out_off = out_off.data_ptr()
        b.out_len = out_len.data_ptr()
        b.status = status.data_ptr()
        keep = None
        if mki is not None:
            keep = (C.c_uint8 * len(mki))(*mki)
            b.mki_index = C.cast(keep, C.c_void_p)
        b.stream = stream
        return Status(fn(self.h, C.byref(b)))

    def protect_device(self, *a, **k):
        return self._device(self.L.srtp_protect_device, *a, **k)

    # A batch descriptor built once and submitted many times (the arenas it
    # points at keep their addresses): what a C caller does, without the
    # per-call ctypes marshalling of nine tensor pointers.
    @staticmethod
    def prepare_device(arena_in, in_off, in_len, arena_out, out_off, out_len,
                       status, stream=None):
        b = DeviceBatch()
        b.n = in_off.numel()
        b.in_ = arena_in.data_ptr()
        b.in_off = in_off.data_ptr()
        b.in_len = in_len.data_ptr()
        b.out = arena_out.data_ptr()
        b.out_off = out_off.data_ptr()
        b.out_len = out_len.data_ptr()
        b.status = status.data_ptr()
        b.stream = stream
        return b

    def protect_prepared(self, b):
        return self.L.srtp_protect_device(self.h, C.byref(b))

    def protect_prepared_async(self, b):
        """srtp_protect_device_async: returns once the GPU pre-pass has
        committed the batch; the bytes are done when the stream is."""
        return self.L.srtp_protect_device_async(self.h, C.byref(b))

    def unprotect_prepared(self, b):
        return self.L.srtp_unprotect_device(self.h, C.byref(b))

    def unprotect_device(self, *a, **k):
        return self._device(self.L.srtp_unprotect_device, *a, **k)

    # -- misc ----------------------------------------------------------------
    def get_roc(self, ssrc):
        r = C.c_uint32()
        st = self.L.srtp_stream_get_roc(self.h, ssrc, C.byref(r))
        return Status(st), r.value

    def set_roc(self, ssrc, roc):
        return Status(self.L.srtp_stream_set_roc(self.h, ssrc, roc))

    def trailer_length(self, mki_index=0):
        n = C.c_size_t()
        st = self.L.srtp_get_protect_trailer_length(self.h, mki_index,
                                                    C.byref(n))
        return Status(st), n.value

    def rtcp_trailer_length(self, mki_index=0):
        n = C.c_size_t()
        st = self.L.srtp_get_protect_rtcp_trailer_length(self.h, mki_index,
                                                         C.byref(n))
        return Status(st), n.value

    def set_timing(self, on=True):
        self.L.srtp_mi355x_set_timing(self.h, 1 if on else 0)

    def last_kernel_ms(self):
        return self.L.srtp_mi355x_last_kernel_ms(self.h)

    def prepass_last_abort(self):
        """reason bits of the most recent device pre-pass fallback (0: none)"""
        return self.L.srtp_mi355x_prepass_last_abort(self.h)

    def prepass_stats(self):
        """(device-API batches done by the GPU pre-pass, by the host)"""
        d, h = C.c_uint64(), C.c_uint64()
        self.L.srtp_mi355x_prepass_stats(self.h, C.byref(d), C.byref(h))
        return d.value, h.value

    def debug_key_left(self, ssrc, j=0):
        """uses left of master key j of the stream (key limit counter)"""
        v = C.c_uint64()
        rc = self.L.srtp_mi355x_debug_key_left(self.h, ssrc, j, C.byref(v))
        return Status(rc), v.value

    def debug_set_key_limit(self, ssrc, num_left):
        return Status(self.L.srtp_mi355x_debug_set_key_limit(self.h, ssrc,
                                                             num_left))

    def prepass_sorted_batches(self):
        """device pre-pass batches that needed the sorted chain path"""
        return self.L.srtp_mi355x_prepass_sorted_batches(self.h)

    def bucket_batches(self):
        """device batches whose crypto ran from key buckets"""
        return self.L.srtp_mi355x_bucket_batches(self.h)

    def inorder_stats(self):
        """(batches the one-stream in-order form committed, declined)"""
        r, d = C.c_uint64(), C.c_uint64()
        self.L.srtp_mi355x_inorder_stats(self.h, C.byref(r), C.byref(d))
        return r.value, d.value

    def unprotect_stats(self):
        """(rounds, crypto launches, undo launches) of the last unprotect
        batch"""
        v = [C.c_uint32() for _ in range(3)]
        self.L.srtp_mi355x_unprotect_stats(self.h, *[C.byref(x) for x in v])
        return tuple(x.value for x in v)

    def close(self):
        if self.h:
            self.L.srtp_dealloc(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
