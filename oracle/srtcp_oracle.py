"""CPU restatement of libsrtp's SRTCP path (AES-ICM / null cipher with
HMAC-SHA1 / null auth, and AES-GCM), built on the oracle primitives of
pyoracle.

TEST INFRASTRUCTURE ONLY: imported by tests/ -- never by libsrtp_amd.
Pinned against tests/golden/ref_rtcp.json and ref_rtcp_gcm.json (the
reference's own outputs, oracle/gen_golden_rtcp.c) by
tests/test_oracle_golden.py.

Follows cisco/libsrtp 3.0.0:
  srtp_protect_rtcp      srtp/srtp.c:4304-4544
  srtp_unprotect_rtcp    srtp/srtp.c:4546-4837
  RTCP session keys      srtp/srtp.c:1527-1600 (KDF labels 3, 4, 5), KDF
                         srtp.c:1070-1142
  replay database        crypto/replay/rdb.c:63-140
  MKI lookup             srtp/srtp.c:1961-2035
  AEAD SRTCP             srtp/srtp.c:3894-4300 (IV 3894-3930)
"""
from oracle import pyoracle as O

OK, BAD_PARAM, AUTH_FAIL, REPLAY_FAIL, REPLAY_OLD = 0, 2, 7, 9, 10
NO_CTX, CANT_CHECK, KEY_EXPIRED, BAD_MKI, BUFFER_SMALL = 13, 14, 15, 25, 28
NO_SUCH_OP = 12

NULL_CIPHER, ICM_128, ICM_192, ICM_256 = 0, 1, 4, 5
GCM_128, GCM_256 = 6, 7
HMAC_SHA1 = 3
SEC_CONF, SEC_AUTH = 1, 2
SSRC_SPECIFIC, SSRC_ANY_INBOUND, SSRC_ANY_OUTBOUND = 1, 2, 3
DIR_UNKNOWN, DIR_SENDER, DIR_RECEIVER = 0, 1, 2
RDB_BITS = 128


def _kdf(key, salt14, label, n):
    # srtp_kdf_generate (srtp.c:1105-1128): AES-ICM keystream, label at byte 7
    if n == 0:
        return b""
    nonce = bytes(7) + bytes([label]) + bytes(8)
    rc, out = O.icm_xor(key, salt14, nonce, bytes(n))
    assert rc == 0
    return out


class _Key:
    def __init__(self, pol, master, mki):
        self.gcm = pol["rtcp_cipher_type"] in (GCM_128, GCM_256)
        # srtp_stream_init_keys, srtp.c:1262-1320: the master key is used up
        # to input_keylen and zero-padded to the KDF key length
        full = {ICM_128: 30, ICM_192: 38, ICM_256: 46, GCM_128: 28,
                GCM_256: 44}
        inp = max(full.get(pol["cipher_type"], 0),
                  full.get(pol["rtcp_cipher_type"], 0),
                  30 if HMAC_SHA1 in (pol["auth_type"], pol["rtcp_auth_type"])
                  else 0)
        master = master[:inp] + bytes(64)
        kdf_len = max(30, pol["cipher_key_len"], pol["rtcp_cipher_key_len"],
                      inp)
        if kdf_len in (28, 44):
            kdf_len += 2                 # srtp.c:1309-1312
        kdf_key = master[:kdf_len - 14]
        kdf_salt = master[kdf_len - 14:kdf_len]
        self.null = pol["rtcp_cipher_type"] == NULL_CIPHER
        if self.gcm:
            base = pol["rtcp_cipher_key_len"] - 12
            self.ek = _kdf(kdf_key, kdf_salt, 3, base)
            self.salt = _kdf(kdf_key, kdf_salt, 5, 12)
            self.hmac, self.ak = False, b""
            self.tag_len = pol["rtcp_auth_tag_len"]
            self.mki = mki
            return
        if not self.null:
            base = pol["rtcp_cipher_key_len"] - 14
            self.ek = _kdf(kdf_key, kdf_salt, 3, base)
            self.salt = _kdf(kdf_key, kdf_salt, 5, 14)
        self.hmac = pol["rtcp_auth_type"] == HMAC_SHA1
        self.ak = _kdf(kdf_key, kdf_salt, 4, pol["rtcp_auth_key_len"]) \
            if self.hmac else b""
        self.tag_len = pol["rtcp_auth_tag_len"]
        self.mki = mki

    def crypt(self, ssrc4, idx, data):
        if self.null:
            return data
        iv = bytes(4) + ssrc4 + (idx >> 16).to_bytes(4, "big") + \
            ((idx << 16) & 0xffffffff).to_bytes(4, "big")
        rc, out = O.icm_xor(self.ek, self.salt, iv, data)
        assert rc == 0
        return out

    def aead_iv(self, ssrc4, idx):
        x = bytes(2) + ssrc4 + bytes(2) + idx.to_bytes(4, "big")
        return bytes(a ^ b for a, b in zip(x, self.salt))

    def tag(self, msg):
        if not self.hmac:
            return b""
        return O.hmac_sha1(self.ak, msg)[:self.tag_len]


class _Stream:
    def __init__(self, ssrc, direction, services, keys, mki_size):
        self.ssrc, self.direction = ssrc, direction
        self.services, self.keys, self.mki_size = services, keys, mki_size
        self.start, self.bm = 0, 0

    def clone(self, ssrc):
        return _Stream(ssrc, self.direction, self.services, self.keys,
                       self.mki_size)

    # rdb.c:74-127
    def check(self, idx):
        if idx >= self.start + RDB_BITS:
            return OK
        if idx < self.start:
            return REPLAY_OLD
        return REPLAY_FAIL if (self.bm >> (idx - self.start)) & 1 else OK

    def add(self, idx):
        if idx < self.start:
            return
        d = idx - self.start
        if d < RDB_BITS:
            self.bm |= 1 << d
        else:
            d -= RDB_BITS - 1
            self.bm = (self.bm >> d) | (1 << (RDB_BITS - 1))
            self.start += d


class SrtcpSession:
    def __init__(self, policies):
        self.streams, self.templ = {}, None
        for p in policies:
            mkis = p.get("mki_ids") or []
            keys = [_Key(p, bytes.fromhex(k),
                         bytes.fromhex(mkis[i]) if p["use_mki"] else b"")
                    for i, k in enumerate(p["keys"])]
            t = p["ssrc_type"]
            d = {SSRC_ANY_OUTBOUND: DIR_SENDER,
                 SSRC_ANY_INBOUND: DIR_RECEIVER}.get(t, DIR_UNKNOWN)
            s = _Stream(p["ssrc"], d, p["rtcp_sec_serv"], keys,
                        p["mki_size"] if p["use_mki"] else 0)
            if t == SSRC_SPECIFIC:
                self.streams[p["ssrc"]] = s
            else:
                self.templ = s

    def protect_rtcp(self, rtcp, cap, mki_index=0):
        if len(rtcp) < 8:
            return BAD_PARAM, None
        ssrc = int.from_bytes(rtcp[4:8], "big")
        st = self.streams.get(ssrc)
        if st is None:
            if self.templ is None:
                return NO_CTX, None
            st = self.streams[ssrc] = self.templ.clone(ssrc)
        if st.direction != DIR_SENDER and st.direction == DIR_UNKNOWN:
            st.direction = DIR_SENDER
        if st.mki_size and mki_index >= len(st.keys):
            return BAD_MKI, None
        k = st.keys[mki_index if st.mki_size else 0]
        out_len = len(rtcp) + 4 + st.mki_size + k.tag_len
        if cap < out_len:
            return BUFFER_SMALL, None
        if st.start >= 0x7fffffff:
            return KEY_EXPIRED, None
        st.start += 1
        idx = st.start
        conf = bool(st.services & SEC_CONF)
        if k.gcm:   # srtp_protect_rtcp_aead, srtp.c:3939-4100
            tr = (((1 << 31) if conf else 0) | idx).to_bytes(4, "big")
            iv = k.aead_iv(rtcp[4:8], idx)
            if conf:
                ct = O.gcm_seal(k.ek, iv, rtcp[:8] + tr, rtcp[8:], k.tag_len)
                return OK, rtcp[:8] + ct + tr + k.mki
            t = O.gcm_seal(k.ek, iv, rtcp + tr, b"", k.tag_len)
            return OK, rtcp + t + tr + k.mki
        body = k.crypt(rtcp[4:8], idx, rtcp[8:]) if conf else rtcp[8:]
        msg = rtcp[:8] + body + (((1 << 31) if conf else 0) | idx).to_bytes(
            4, "big")
        return OK, msg + k.mki + k.tag(msg)

    def unprotect_rtcp(self, srtcp, cap):
        n = len(srtcp)
        if n < 12:
            return BAD_PARAM, None
        ssrc = int.from_bytes(srtcp[4:8], "big")
        st = self.streams.get(ssrc)
        provisional = False
        if st is None:
            if self.templ is None:
                return NO_CTX, None
            st, provisional = self.templ, True
        k = st.keys[0]
        if st.mki_size:
            tl = 0 if k.gcm else k.tag_len
            if tl > n or st.mki_size > n - tl:
                return BAD_MKI, None
            m = srtcp[n - tl - st.mki_size:n - tl]
            k = next((x for x in st.keys if x.mki == m), None)
            if k is None:
                return BAD_MKI, None
        tl = k.tag_len
        if n < 8 + 4 + st.mki_size + tl:
            return BAD_PARAM, None
        if k.gcm:   # srtp_unprotect_rtcp_aead, srtp.c:4102-4300
            tp = n - 4 - st.mki_size
            idx = int.from_bytes(srtcp[tp:tp + 4], "big") & 0x7fffffff
            rc = st.check(idx)
            if rc:
                return rc, None
            out_len = n - tl - 4 - st.mki_size
            if cap < out_len:
                return BUFFER_SMALL, None
            iv = k.aead_iv(srtcp[4:8], idx)
            tr = srtcp[tp:tp + 4]
            tag = srtcp[out_len:out_len + tl]
            if srtcp[tp] & 0x80:
                rc, pt = O.gcm_open(k.ek, iv, srtcp[:8] + tr, srtcp[8:out_len],
                                    tag)
                out = srtcp[:8] + pt
            else:
                rc, _ = O.gcm_open(k.ek, iv, srtcp[:out_len] + tr, b"", tag)
                out = srtcp[:out_len]
            if rc:
                return rc, None
            return self._accept(st, provisional, ssrc, idx, out)
        conf = st.services in (SEC_CONF, SEC_CONF | SEC_AUTH)
        tp = n - (tl + st.mki_size + 4)
        if bool(srtcp[tp] & 0x80) != conf:
            return CANT_CHECK, None
        auth_len = n - tl - st.mki_size
        idx = int.from_bytes(srtcp[tp:tp + 4], "big") & 0x7fffffff
        rc = st.check(idx)
        if rc:
            return rc, None
        if k.tag(srtcp[:auth_len]) != srtcp[auth_len + st.mki_size:]:
            return AUTH_FAIL, None
        out_len = auth_len - 4
        if cap < out_len:
            return BUFFER_SMALL, None
        body = srtcp[8:out_len]
        out = srtcp[:8] + (k.crypt(srtcp[4:8], idx, body) if conf else body)
        return self._accept(st, provisional, ssrc, idx, out)

    def _accept(self, st, provisional, ssrc, idx, out):
        if st.direction == DIR_UNKNOWN:
            st.direction = DIR_RECEIVER
        if provisional:
            st = self.streams[ssrc] = self.templ.clone(ssrc)
        st.add(idx)
        return OK, out
